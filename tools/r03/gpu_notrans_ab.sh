#!/bin/bash
# timing only: what the MAC's quad transposes cost in the pipelined cfg2 step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_notrans
mkdir -p $O
bash tools/ab_bench.sh $O cfg2 3 base notrans || exit 1
