#!/bin/bash
# round 3: GPU suite on the product build, the pair-layout cipher phase (TG_AB_PAIR)
# through the many-chains tests and a full-size bench parity check, then same-box A/Bs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_pair
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TLSGPU_LIB=$R/tools/ab/pair8/libtlsgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_seal.py -x -q -m gpu -k "many or pipeline or generations" --timeout 200 --timeout-method thread > $O/pytest_pair8.log 2>&1 || { echo "pair8 pytest failed"; tail -40 $O/pytest_pair8.log; exit 1; }
tail -2 $O/pytest_pair8.log
for cfg in cfg2 cfg3; do
  TLSGPU_LIB=$R/tools/ab/pair8/libtlsgpu.so timeout -k 10 300 python bench.py --config $cfg --no-host-inclusive --no-open --no-derive --no-cpu --steps 20 > $O/check_$cfg.json 2> $O/check_$cfg.err || { tail -20 $O/check_$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('$O/check_$cfg.json'));print('check $cfg pair8', d['value'], d['bit_exact'], d['timed_bit_exact'], d['roofline']['kernel'], d['roofline']['frac_of_copy'])"
done
bash tools/ab_bench.sh $O cfg2 3 base pair8 || exit 1
bash tools/ab_bench.sh $O cfg3 2 base pair8 pair8m12 pair8m8 || exit 1
