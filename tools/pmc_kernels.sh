#!/bin/bash
# Per-kernel PMC counters of one seal config (MI355X_MICROARCH.md §PMC/§HBM):
# each counter group in its own rocprofv3 pass, --kernel-trace only (no other
# trace domains with --pmc).  HBM read bytes come from the request-size counters
# (32·RDREQ_32B + 64·RDREQ_64B + 128·RDREQ_128B: exact for every access pattern,
# where FETCH_SIZE tallies 128-B requests at 64 B -- tools/traffic_calib.hip).  PMC
# mode serialises dispatches, so every kernel is measured on its own.  Usage (GPU box):
#   bash tools/pmc_kernels.sh <config> <outdir> [extra bench args]
# PMC_NAME=<name>: write profiles/<name>.json (default pmc_<config>); with --open among the
# extra args the open leg's kernels are counted too (open_call_hbm_bytes).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-cfg2}
OUT=${2:-gpurun_out/pmck_$CFG}
case $OUT in /*) ;; *) OUT=$R/$OUT ;; esac
shift 2 || true
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY" \
         "SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $OUT/g$i -o run -- \
      python $R/bench.py --config $CFG --steps 3 --warmup 1 --no-check --no-cpu --no-host-inclusive --no-open --no-derive "$@" > $OUT/g$i.log 2>&1
  i=$((i+1))
done
python $R/tools/pmc_summarize.py $OUT $CFG ${PMC_NAME:-pmc_$CFG}
