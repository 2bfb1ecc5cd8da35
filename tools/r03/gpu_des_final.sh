#!/bin/bash
# product library with the combined-table tdes4_kernel: GPU suite, checked cfg5 bench, PMC of cfg5
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_desfinal
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --config cfg5 --no-host-inclusive > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench_cfg5.json'));print({k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')}, d['roofline'], d.get('open'))"
bash tools/pmc_kernels.sh cfg5 $O/pmc_cfg5 || exit 1
cp profiles/pmc_cfg5.json $O/ 2>/dev/null; true
