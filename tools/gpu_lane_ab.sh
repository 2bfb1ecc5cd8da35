#!/bin/bash
# lane seal kernel (A/B build tools/ab/lane): parity at scale, then cfg3 against the split path
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02l9
mkdir -p $O
for v in lane; do
TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_seal.py -x -v --timeout 200 --timeout-method thread -k "lane" > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -40 $O/pytest_$v.log; exit 1; }
tail -1 $O/pytest_$v.log
done
bash tools/ab_bench.sh $O/ab cfg3 2 base lane || exit 1
