#!/bin/bash
# r02af: cfg3 with 12 cipher waves per CU and / or MAC prefetch 1 (two MAC waves per SIMD beside the cipher).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/ab_bench.sh gpurun_out/r02af cfg3 2 base w12pf1 pf1 w12 || exit 1
bash tools/ab_bench.sh gpurun_out/r02af cfg2 1 base pf1 || exit 1
echo done
