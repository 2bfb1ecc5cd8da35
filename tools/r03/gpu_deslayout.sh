#!/bin/bash
# combined-table layouts for tdes4_kernel: j in the bank bits (desl1), + 2 copies (desl2) vs base
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_deslayout
mkdir -p $O
for v in desl1 desl2; do
  TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "3DES or 3des or tdes or batch" > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -40 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
bash tools/ab_bench.sh $O cfg5 3 base desl1 desl2 || exit 1
