#!/bin/bash
# r02b: CBC prefetch ring (per-block load/store order) -- cfg2 with and without the MAC
# bulk, cfg4 at 4096 and 512 connections, AES layout microbenchmark (latency regime).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02b
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_seal.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 ./tools/aes_layout_mb.bin 1027 lat > $O/mb_lat.log 2>&1 || { cat $O/mb_lat.log; exit 1; }
cat $O/mb_lat.log
bash tools/ab_bench.sh gpurun_out/r02b/ab cfg2 2 base nomac || exit 1
AB_ARGS="--steps 5 --warmup 1" bash tools/ab_bench.sh gpurun_out/r02b/ab cfg4 1 base || exit 1
AB_ARGS="--steps 5 --warmup 1 --records 512" bash tools/ab_bench.sh gpurun_out/r02b/ab4s cfg4 1 base || exit 1
AB_ARGS="--steps 10 --warmup 2" bash tools/ab_bench.sh gpurun_out/r02b/ab cfg3 1 base || exit 1
echo done
