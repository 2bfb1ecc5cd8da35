#!/bin/bash
# pair kernel: burst stores per group (stburst) and line-aligned groups (stalign = stburst + head
# blocks up to the output's next 128-B line); parity of stalign first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_stalign
mkdir -p $O
for v in stburst stalign; do
TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_seal.py tests/test_batch_golden.py tests/test_session_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -40 $O/pytest_$v.log; exit 1; }
tail -1 $O/pytest_$v.log
TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so timeout -k 10 300 python bench.py --config cfg2 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check_$v.json 2> $O/check_$v.err || { tail -20 $O/check_$v.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_$v.json'));print('check $v', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
done
bash tools/ab_bench.sh $O cfg2 3 base stburst stalign || exit 1
bash tools/ab_bench.sh $O cfg3 2 base stburst stalign || exit 1
