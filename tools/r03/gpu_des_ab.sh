#!/bin/bash
# round 3: 3DES on byte-row SP tables (one v_perm per even lookup) vs the 32-copy tables
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_des
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config cfg5 --no-host-inclusive --no-open --no-derive --no-cpu --steps 20 > $O/check_cfg5.json 2> $O/check_cfg5.err || { tail -20 $O/check_cfg5.err; exit 1; }
python -c "import json;d=json.load(open('$O/check_cfg5.json'));print('check cfg5', d['value'], d['bit_exact'], d['timed_bit_exact'], d['roofline']['kernel'], d['roofline']['kernel_avg_ms'])"
bash tools/ab_bench.sh $O cfg5 3 base desold || exit 1
