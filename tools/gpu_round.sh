#!/bin/bash
# One GPU session: parity tests, open-path smoke, benches for every config, rocprof
# kernel-trace summary of the headline.  Every GPU step has its own time limit and
# the script stops at the first failure.  Usage (GPU box): bash tools/gpu_round.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/dbg_open.py 4096 > $O/dbg_open.log 2>&1 || { echo "dbg_open failed"; cat $O/dbg_open.log; exit 1; }
cat $O/dbg_open.log
timeout -k 10 300 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo "bench failed"; tail -20 $O/bench_cfg2.err; exit 1; }
cut -c1-600 $O/bench_cfg2.json
for c in cfg3 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-host-inclusive > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -20 $O/bench_$c.err; exit 1; }
  cut -c1-300 $O/bench_$c.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --no-check --no-cpu --no-host-inclusive --no-open --no-derive --steps 50 > $O/bench_prof.json 2> $O/bench_prof.err \
    || { echo "rocprof failed"; tail -20 $O/bench_prof.err; exit 1; }
grep '^{' $O/bench_prof.json | cut -c1-300
echo done
