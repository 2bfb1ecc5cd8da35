#!/bin/bash
# HBM traffic of the seal kernel from PMC counters (MI355X_MICROARCH.md §HBM):
# FETCH_SIZE and WRITE_SIZE in SEPARATE passes (TCC slots), kernel-trace only.
# Usage (GPU box): bash tools/pmc_traffic.sh <config> <outdir>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-cfg2}
OUT=${2:-$R/gpurun_out/pmc_$CFG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$C -o run -- \
      python $R/bench.py --config $CFG --steps 3 --warmup 1 --no-check --no-cpu --no-host-inclusive > $OUT/$C.log 2>&1
done
python $R/tools/pmc_summarize.py $OUT $CFG
