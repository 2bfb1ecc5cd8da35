#!/bin/bash
# cfg2: the MAC phase's plaintext loads cost the cipher phase 0.13 ms (noload probe); deeper
# cipher prefetch groups (12, 16 blocks) against the 8-block base
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_pairg
mkdir -p $O
bash tools/ab_bench.sh $O cfg2 3 base g12 g16 || exit 1
