#!/bin/bash
# round 3: SHA-1 rounds with 2-cycle v_add_u32 instead of v_add3_u32 (add2) vs product
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_add2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_bench.sh $O cfg2 3 base add2 || exit 1
bash tools/ab_bench.sh $O cfg3 1 base add2 || exit 1
