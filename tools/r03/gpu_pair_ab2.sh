#!/bin/bash
# round 3: pair layout with 4-block prefetch groups (<= 88 / 96 VGPRs: two MAC waves per
# SIMD beside two cipher waves) and the 128-VGPR MAC kernel in the pair regime
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_pair2
mkdir -p $O
TLSGPU_LIB=$R/tools/ab/pg4/libtlsgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_seal.py -x -q -m gpu -k "many or pipeline or generations" --timeout 200 --timeout-method thread > $O/pytest_pg4.log 2>&1 || { echo "pg4 pytest failed"; tail -40 $O/pytest_pg4.log; exit 1; }
tail -1 $O/pytest_pg4.log
bash tools/ab_bench.sh $O cfg2 3 base pair8m8 pg4 pg4mm || exit 1
bash tools/ab_bench.sh $O cfg3 2 base pair8m8 pg4 || exit 1
bash tools/ab_prof.sh $O/prof cfg2 base pg4 pg4mm || exit 1
