#!/bin/bash
# record run 4 + PMC of the dominant kernels on the final tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_record_run.sh r03final4 || exit 1
bash tools/r03/gpu_pmc_final.sh || exit 1
