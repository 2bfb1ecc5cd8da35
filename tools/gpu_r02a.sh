#!/bin/bash
# Round-2 first GPU session: parity, smoke, default bench, A/B of compile-time
# variants, AES layout microbenchmark (latency + throughput regimes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -20 $O/bench_cfg2.err; exit 1; }
cut -c1-400 $O/bench_cfg2.json
timeout -k 10 120 ./tools/aes_layout_mb.bin 1027 lat > $O/mb_lat.log 2>&1 || { cat $O/mb_lat.log; exit 1; }
cat $O/mb_lat.log
timeout -k 10 200 ./tools/aes_layout_mb.bin 1027 > $O/mb_tput.log 2>&1 || { cat $O/mb_tput.log; exit 1; }
cat $O/mb_tput.log
bash tools/ab_bench.sh gpurun_out/r02a/ab cfg2 2 base nomac macnt roundb cbcntst || exit 1
AB_ARGS="--steps 5 --warmup 1" bash tools/ab_bench.sh gpurun_out/r02a/ab cfg4 1 base roundb || exit 1
AB_ARGS="--steps 5 --warmup 1 --records 512" bash tools/ab_bench.sh gpurun_out/r02a/ab4s cfg4 1 base roundb || exit 1
echo done
