#!/bin/bash
# round 3: product = pair layout (cfg2: G=8, cfg3: G=4 + MAC-many) + MAC ring unrolled;
# A/B against the quad layout (nopair) and the earlier pair build with the old MAC loop
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_pair3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 ./tools/bin/valu_rate > $O/valu_mix.log 2>&1 || exit 1
grep -i "mix\|alignbit\|v_xor_b32 (asm)\|perm_b32 (asm)" $O/valu_mix.log
bash tools/ab_bench.sh $O cfg2 3 base nopair pair8m8 || exit 1
bash tools/ab_bench.sh $O cfg3 2 base nopair || exit 1
timeout -k 10 120 ./tools/bin/aes_round_latency > $O/round_latency.log 2>&1 || { tail $O/round_latency.log; exit 1; }
cat $O/round_latency.log
