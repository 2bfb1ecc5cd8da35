#!/bin/bash
# cfg2: what slows the cipher phase beside the MAC phase -- MAC compressions without their
# plaintext loads (noload, timing only) vs no MAC compressions (nomac) vs the product
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_cfg2noload
mkdir -p $O
bash tools/ab_bench.sh $O cfg2 3 base noload nomac || exit 1
