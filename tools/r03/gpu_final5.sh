#!/bin/bash
# final record run of the round + cfg2 PMC + cfg2 clock probe (product / noload / nomac)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_record_run.sh r03final5 || exit 1
O=gpurun_out/r03_pmcfinal5
mkdir -p $O
bash tools/pmc_kernels.sh cfg2 $O/pmc_cfg2 > $O/pmc_cfg2.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc_cfg2.log; exit 1; }
cp $R/profiles/pmc_cfg2.json $O/pmc_cfg2.json
bash tools/r03/gpu_clock.sh || exit 1
