#!/bin/bash
# tdes4 round in the lane's rotated frame (next address = x ^ (rotr(f) & m), product build) vs the
# previous combined-table round (desprev); full GPU suite on the product first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_desrot
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config cfg5 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check_cfg5.json 2> $O/check_cfg5.err || { tail -20 $O/check_cfg5.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_cfg5.json'));print('check', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
bash tools/ab_bench.sh $O cfg5 3 base desprev || exit 1
