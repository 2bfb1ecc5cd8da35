#!/bin/bash
# round 3: LAT quad round with the key folded into the last XOR (cfg4) and the pair round's
# partner join as v_mov_dpp + v_bitop3; A/B against the previous commit's library (prev)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_lat
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 ./tools/bin/aes_round_latency > $O/round_latency.log 2>&1 || { tail $O/round_latency.log; exit 1; }
grep -E "quad_lat|pair|quad_thr" $O/round_latency.log
AB_ARGS="--records 512 --steps 3 --warmup 1" bash tools/ab_bench.sh $O cfg4 2 base prev || exit 1
bash tools/ab_bench.sh $O cfg2 3 base prev xdpp || exit 1
bash tools/ab_bench.sh $O cfg3 1 base prev || exit 1
