#!/bin/bash
# timing probe of a fused seal kernel: one hash compression per 8 (cfg2) / 8 (fuse8, cfg3)
# / 4 (fuse, cfg3: twice the MAC work) cipher blocks inside cbc_pair_kernel, MAC bulk skipped
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_fuse
mkdir -p $O
bash tools/ab_bench.sh $O cfg2 2 base nomac fuse || exit 1
bash tools/ab_bench.sh $O cfg3 2 base nomac fuse8 fuse || exit 1
