#!/bin/bash
# workload wire layout: bodies congruent to their plaintext mod 128 B (new) vs packed 16-B slots (old);
# GPU suite on the new layout first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_layout
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in cfg2 cfg3 cfg5; do
timeout -k 10 300 python bench.py --config $c --no-host-inclusive --no-derive --no-cpu > $O/check_$c.json 2> $O/check_$c.err || { tail -20 $O/check_$c.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_$c.json'));print('check $c', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')}, d['open']['value'], d['open']['roundtrip_exact'])"
done
for i in 1 2; do for c in cfg2 cfg3 cfg5; do for lay in new old; do
  if [ $lay = old ]; then export TLSGPU_WL_OLD_LAYOUT=1; else unset TLSGPU_WL_OLD_LAYOUT; fi
  timeout -k 10 300 python bench.py --config $c --no-host-inclusive --no-open --no-derive --no-cpu --no-check > $O/${c}_${lay}_$i.json 2> $O/${c}_${lay}_$i.err || { tail -20 $O/${c}_${lay}_$i.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/${c}_${lay}_$i.json'));print('$c $lay', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
done; done; done
