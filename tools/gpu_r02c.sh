#!/bin/bash
# r02c: quad-cooperative MAC loads (coalesced, butterfly transposes); group-of-8 CBC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02c
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_bench.sh gpurun_out/r02c/ab cfg2 2 base nomac || exit 1
AB_ARGS="--steps 10 --warmup 2" bash tools/ab_bench.sh gpurun_out/r02c/ab cfg3 1 base nomac || exit 1
AB_ARGS="--steps 10 --warmup 2" bash tools/ab_bench.sh gpurun_out/r02c/ab cfg5 1 base || exit 1
timeout -k 10 300 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -20 $O/bench_cfg2.err; exit 1; }
cut -c1-1500 $O/bench_cfg2.json
echo done
