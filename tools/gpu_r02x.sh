#!/bin/bash
# r02x: GPU tests (idle-quad mirroring in cbc_kernel), cfg4 at 4096/512 chains,
# MAC / cipher wave priorities on cfg3 and cfg2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02x
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for n in 512 4096; do
  timeout -k 10 300 python bench.py --config cfg4 --records $n --steps 2 --warmup 1 --no-cpu --no-host-inclusive --no-open --no-derive > $O/cfg4_$n.json 2> $O/cfg4_$n.err || { tail -5 $O/cfg4_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/cfg4_$n.json'));print('cfg4 conns $n', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['bit_exact'])"
done
bash tools/ab_bench.sh gpurun_out/r02x cfg3 2 base mp2 mp1c0 || exit 1
bash tools/ab_bench.sh gpurun_out/r02x cfg2 2 base mp2 mp1c0 || exit 1
echo done
