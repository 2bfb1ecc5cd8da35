#!/bin/bash
# r02d: wave-priority A/B with the cooperative MAC; kernel trace of the pipelined cfg2 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02d
mkdir -p $O
cd $R
bash tools/ab_bench.sh gpurun_out/r02d/ab cfg2 2 base nomac m1c1 m2c1 m0c0 m1c2 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $R/bench.py --no-check --no-cpu --no-host-inclusive --no-open --no-derive --steps 30 > $O/bench_prof.json 2> $O/bench_prof.err \
    || { echo "rocprof failed"; tail -20 $O/bench_prof.err; exit 1; }
cut -c1-300 $O/bench_prof.json
find $O/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
echo done
