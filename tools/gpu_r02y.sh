#!/bin/bash
# r02y: GPU tests; cfg3 / cfg2 with the seqnum prefix on its own pipeline stream.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02y
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_bench.sh gpurun_out/r02y cfg3 2 base || exit 1
bash tools/ab_bench.sh gpurun_out/r02y cfg2 2 base || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr3 -o run -- \
    python $R/bench.py --config cfg3 --steps 6 --warmup 2 --no-check --no-cpu --no-host-inclusive --no-open --no-derive > $O/cfg3t.json 2> $O/cfg3t.err || { tail -5 $O/cfg3t.err; exit 1; }
python $R/tools/trace_timeline.py $O/tr3 12 > $O/cfg3_timeline.txt
echo done
