#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/r03/gpu_des_ab.sh || exit 1
cd $R
bash tools/r03/gpu_pmc_a.sh || exit 1
