#!/bin/bash
# round 3 PMC pass A: the gfx950 counter list, FETCH/WRITE calibration of the access
# patterns (incl. scattered narrow state reads), per-kernel counters of cfg2 and cfg3
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r03_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_avail.txt 2>&1 || echo "list failed (ignored)"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/calib_$C -o run -- $R/tools/bin/traffic_calib > $O/calib_$C.log 2>&1 || { echo "calib $C failed"; tail $O/calib_$C.log; exit 1; }
done
python $R/tools/traffic_calib_summary.py $O/calib_FETCH_SIZE 1509949440 > $O/calib.txt
python $R/tools/traffic_calib_summary.py $O/calib_WRITE_SIZE 1509949440 >> $O/calib.txt
cat $O/calib.txt
cd $R
for cfg in cfg2 cfg3; do
  timeout -k 10 500 bash tools/pmc_kernels.sh $cfg gpurun_out/r03_pmc/$cfg > $O/pmc_$cfg.out 2>&1 || { echo "pmc $cfg failed"; tail -20 $O/pmc_$cfg.out; exit 1; }
  cp profiles/pmc_$cfg.json $O/
  python -c "import json;d=json.load(open('profiles/pmc_$cfg.json'));print('$cfg', d['dominant_kernel'], d['hbm_bytes_per_launch'], d['seal_call_hbm_bytes'])"
done
