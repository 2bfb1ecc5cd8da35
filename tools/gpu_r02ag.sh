#!/bin/bash
# r02ag: global (not flat) cooperative MAC loads; 3DES address by v_bitop3 (base) vs v_and_or.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02ag
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_bench.sh gpurun_out/r02ag cfg5 2 base desandor || exit 1
bash tools/ab_bench.sh gpurun_out/r02ag cfg2 2 base macflat || exit 1
bash tools/ab_bench.sh gpurun_out/r02ag cfg3 2 base macflat || exit 1
echo done
