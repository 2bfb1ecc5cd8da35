#!/bin/bash
# r02j: 3DES layout microbench (d2/d1 added), host pipeline sweep, pipeline workspace rotation 3 vs 2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02j
mkdir -p $O
cd $R
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/des_layout_microbench.hip -o $O/dmb.bin 2> /dev/null || { echo "dmb build failed"; exit 1; }
timeout -k 10 120 $O/dmb.bin 256 > $O/dmb.log 2>&1 || { cat $O/dmb.log; exit 1; }
cat $O/dmb.log
bash tools/ab_bench.sh gpurun_out/r02j cfg2 3 base ws2 || exit 1
bash tools/ab_bench.sh gpurun_out/r02j cfg3 2 base ws2 || exit 1
timeout -k 10 400 python -u tools/hostpipe_sweep.py > $O/hostpipe.log 2>&1 || { tail -20 $O/hostpipe.log; exit 1; }
cat $O/hostpipe.log
echo done
