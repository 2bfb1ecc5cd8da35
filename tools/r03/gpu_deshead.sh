#!/bin/bash
# tdes4: head blocks up to the output's 64-B sector before the 8-block store groups (base) vs prevdes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_deshead
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "3DES or 3des or tdes or batch or session" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config cfg5 --no-host-inclusive --no-open --no-derive --no-cpu > $O/check_cfg5.json 2> $O/check_cfg5.err || { tail -20 $O/check_cfg5.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check_cfg5.json'));print('check cfg5', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
bash tools/ab_bench.sh $O cfg5 3 base prevdes || exit 1
