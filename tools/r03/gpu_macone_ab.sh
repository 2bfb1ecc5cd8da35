#!/bin/bash
# cfg3 (pair many-chains regime): the 128-VGPR one-chunk-prefetch MAC kernel (base) vs the
# one-generation MAC kernel (168-VGPR cap, two-chunk prefetch, no spills): both give 2 MAC
# waves per SIMD beside the two 88-VGPR pair waves
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_macone
mkdir -p $O
bash tools/ab_bench.sh $O cfg3 3 base macone || exit 1
