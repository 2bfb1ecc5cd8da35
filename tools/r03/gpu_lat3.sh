#!/bin/bash
# cfg4 LAT round with three parallel lane moves + two 3-input XORs (lat3) vs the 2-level DPP tree (base)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_lat3
mkdir -p $O
TLSGPU_LIB=$R/tools/ab/lat3/libtlsgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_seal.py tests/test_gpu_factory.py tests/test_batch_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_lat3.log 2>&1 || { echo "pytest lat3 failed"; tail -40 $O/pytest_lat3.log; exit 1; }
tail -1 $O/pytest_lat3.log
TLSGPU_LIB=$R/tools/ab/lat3/libtlsgpu.so timeout -k 10 300 python bench.py --config cfg4 --records 512 --steps 3 --warmup 1 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check.json 2> $O/check.err || { tail -20 $O/check.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check.json'));print('check lat3 cfg4/512', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
AB_ARGS="--records 512 --steps 3 --warmup 1" bash tools/ab_bench.sh $O cfg4 2 base lat3 || exit 1
