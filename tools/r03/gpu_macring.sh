#!/bin/bash
# MAC ring reloaded as a whole (product, PF=2) -- GPU suite + checks; A/B vs a 4-chunk ring (pf4, <= 256 VGPRs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_macring
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in cfg2 cfg3; do
timeout -k 10 300 python bench.py --config $c --no-host-inclusive --no-open --no-derive --no-cpu > $O/check_$c.json 2> $O/check_$c.err || { tail -20 $O/check_$c.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_$c.json'));print('check $c', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
done
TLSGPU_LIB=$R/tools/ab/pf4/libtlsgpu.so timeout -k 10 300 python bench.py --config cfg2 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check_pf4.json 2> $O/check_pf4.err || { tail -20 $O/check_pf4.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_pf4.json'));print('check pf4', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
bash tools/ab_bench.sh $O cfg2 3 base pf4 || exit 1
