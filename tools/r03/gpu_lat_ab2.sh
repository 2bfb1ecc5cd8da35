#!/bin/bash
# round 3: LAT round with the addresses scheduled before the reads (cfg4); A/B vs the same
# round without the schedule (oldsched) and the previous commit (prev)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_lat2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 ./tools/bin/aes_round_latency > $O/round_latency.log 2>&1 || { tail $O/round_latency.log; exit 1; }
grep -E "quad_lat|pair|quad_thr" $O/round_latency.log
AB_ARGS="--records 512 --steps 3 --warmup 1" bash tools/ab_bench.sh $O cfg4 2 base oldsched prev || exit 1
AB_ARGS="--steps 3 --warmup 1" bash tools/ab_bench.sh $O cfg4 1 base prev || exit 1
bash tools/ab_bench.sh $O cfg2 2 base prev || exit 1
