#!/bin/bash
# r02v: PMC passes for cfg3 and cfg2 (current code); effective clock (GRBM_GUI_ACTIVE) of the
# cfg4 cipher kernel at 4096 and 512 chains.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/pmc_kernels.sh cfg3 gpurun_out/r02v_cfg3 > gpurun_out/r02v_cfg3.log 2>&1 || { tail -5 gpurun_out/r02v_cfg3.log; exit 1; }
bash tools/pmc_kernels.sh cfg2 gpurun_out/r02v_cfg2 > gpurun_out/r02v_cfg2.log 2>&1 || { tail -5 gpurun_out/r02v_cfg2.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for n in 4096 512; do
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/r02v_cfg4_$n -o run -- \
      python $R/bench.py --config cfg4 --records $n --steps 2 --warmup 1 --no-check --no-cpu --no-host-inclusive --no-open --no-derive > $R/gpurun_out/r02v_cfg4_$n.log 2>&1 || { tail -5 $R/gpurun_out/r02v_cfg4_$n.log; exit 1; }
done
echo done
