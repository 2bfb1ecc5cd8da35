#!/bin/bash
# round 3 PMC: calibration with the request-size counters, then every config's kernels
#   bash tools/r03/gpu_pmc_b.sh "cfg2 cfg3"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_pmc2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ ! -f $O/calib_req.txt ]; then
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d $O/calib_req -o run -- $R/tools/bin/traffic_calib > $O/calib_req.log 2>&1 || { echo "calib failed"; tail $O/calib_req.log; exit 1; }
  python $R/tools/traffic_calib_summary.py $O/calib_req 1509949440 > $O/calib_req.txt
  cat $O/calib_req.txt
fi
cd $R
for cfg in $1; do
  extra=""
  timeout -k 10 600 bash tools/pmc_kernels.sh $cfg gpurun_out/r03_pmc2/$cfg $extra > $O/pmc_$cfg.out 2>&1 || { echo "pmc $cfg failed"; tail -20 $O/pmc_$cfg.out; exit 1; }
  cp profiles/pmc_$cfg.json $O/
  python -c "import json;d=json.load(open('profiles/pmc_$cfg.json'));print('$cfg', d['dominant_kernel'], d['hbm_bytes_per_launch'], d['seal_call_hbm_bytes'])"
done
