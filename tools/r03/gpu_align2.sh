#!/bin/bash
# pcbc_bulk with the head's and the first group's loads issued together; product (align >= 256
# blocks) vs al16 (align >= 16 blocks: cfg3 too) vs prev (burst stores + aligned groups, head
# loads exposed); tdes4 burst stores in the product
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_align2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TLSGPU_LIB=$R/tools/ab/al16/libtlsgpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_seal.py tests/test_batch_golden.py tests/test_session_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_al16.log 2>&1 || { echo "pytest al16 failed"; tail -40 $O/pytest_al16.log; exit 1; }
tail -1 $O/pytest_al16.log
for c in cfg2 cfg3 cfg5; do
timeout -k 10 300 python bench.py --config $c --no-host-inclusive --no-open --no-derive --no-cpu > $O/check_$c.json 2> $O/check_$c.err || { tail -20 $O/check_$c.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_$c.json'));print('check $c', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
done
TLSGPU_LIB=$R/tools/ab/al16/libtlsgpu.so timeout -k 10 300 python bench.py --config cfg3 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check_al16.json 2> $O/check_al16.err || { tail -20 $O/check_al16.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_al16.json'));print('check al16 cfg3', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
bash tools/ab_bench.sh $O cfg2 2 base prev || exit 1
bash tools/ab_bench.sh $O cfg3 3 base al16 prev || exit 1
