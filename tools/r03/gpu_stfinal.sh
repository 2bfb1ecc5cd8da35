#!/bin/bash
# product with burst stores + line-aligned groups: GPU suite, checked cfg2/cfg3 bench, A/B vs the previous library
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_stfinal
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in cfg2 cfg3; do
timeout -k 10 300 python bench.py --config $c --no-host-inclusive --no-open --no-derive --no-cpu > $O/check_$c.json 2> $O/check_$c.err || { tail -20 $O/check_$c.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_$c.json'));print('check $c', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
done
bash tools/ab_bench.sh $O cfg2 3 base prev || exit 1
bash tools/ab_bench.sh $O cfg3 2 base prev || exit 1
# 3DES: burst stores per 8-block group (desst) vs per-block stores
TLSGPU_LIB=$R/tools/ab/desst/libtlsgpu.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "3DES or 3des or tdes or batch" > $O/pytest_desst.log 2>&1 || { echo "pytest desst failed"; tail -40 $O/pytest_desst.log; exit 1; }
tail -1 $O/pytest_desst.log
TLSGPU_LIB=$R/tools/ab/desst/libtlsgpu.so timeout -k 10 300 python bench.py --config cfg5 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check_desst.json 2> $O/check_desst.err || { tail -20 $O/check_desst.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_desst.json'));print('check desst', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
bash tools/ab_bench.sh $O cfg5 3 base desst || exit 1
