#!/bin/bash
# prefix (meta clear + seqnum walk) of call k+1 on its own pipeline stream beside the MAC
# phase of call k (base) vs the previous library (prefix in the MAC stream's order); GPU suite first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_prestream2
mkdir -p $O


bash tools/ab_bench.sh $O cfg3 2 prehi prelo prev || exit 1
bash tools/ab_bench.sh $O cfg2 2 prehi prelo prev || exit 1
