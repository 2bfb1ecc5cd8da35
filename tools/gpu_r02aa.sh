#!/bin/bash
# r02aa: batch-golden + host pipeline GPU tests; host-inclusive rate (pinned / pageable) on cfg2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02aa
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_batch_golden.py tests/test_gpu_seal.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-open --no-derive > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
python -c "import json;d=json.load(open('$O/b.json'));h=d['host_inclusive'];print(d['value'], h['pinned'], h['pageable'], h['pcie_ceiling'])"
