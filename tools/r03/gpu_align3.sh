#!/bin/bash
# product (head + first-group loads together, aligned groups from 16 blocks) vs headfirst (head loads
# exposed before the first group's, aligned groups from 256 blocks), same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_align3
mkdir -p $O
bash tools/ab_bench.sh $O cfg2 3 base headfirst || exit 1
bash tools/ab_bench.sh $O cfg3 2 base headfirst || exit 1
