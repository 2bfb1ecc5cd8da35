#!/bin/bash
# final record run of the round (bench defaults 500 + 500 steps) + PMC of cfg2 / cfg3 / cfg5
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_record_run.sh r03final6 || exit 1
sed -i 's#O=gpurun_out/r03_pmcfinal4#O=gpurun_out/r03_pmcfinal6#' tools/r03/gpu_pmc_final.sh
bash tools/r03/gpu_pmc_final.sh || exit 1
