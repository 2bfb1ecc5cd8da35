#!/bin/bash
# r02ae: byte-1 address by v_bitop3 and bitop3 transposes (base) vs the v_perm / v_cndmask forms.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02ae
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_bench.sh gpurun_out/r02ae cfg2 3 base oldaddr oldsel || exit 1
bash tools/ab_bench.sh gpurun_out/r02ae cfg3 2 base oldaddr oldsel || exit 1
echo done
