#!/bin/bash
# prefix kernel: state header loaded without short-circuit branches (product) vs prevrec; GPU suite first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_rechoist
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_ARGS="--steps 200 --warmup 200" bash tools/ab_bench.sh $O cfg3 3 base prevrec || exit 1
AB_ARGS="--steps 200 --warmup 200" bash tools/ab_bench.sh $O cfg2 2 base prevrec || exit 1
AB_ARGS="--steps 200 --warmup 200" bash tools/ab_bench.sh $O cfg5 2 base prevrec || exit 1
