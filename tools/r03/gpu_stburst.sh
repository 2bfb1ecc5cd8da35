#!/bin/bash
# pair kernel: a group's ciphertext stored at the group's end (stburst) vs one store per block
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_stburst
mkdir -p $O
bash tools/ab_bench.sh $O cfg2 3 base stburst || exit 1
bash tools/ab_bench.sh $O cfg3 2 base stburst || exit 1
