#!/bin/bash
# r02ab: VALU issue-rate microbench (block span), batch-golden + seal GPU tests,
# host pipeline pinned/pageable, cfg5 PMC with tdes4_kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02ab
mkdir -p $O
cd $R
hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/valu_rate_microbench.hip -o $O/vr.bin 2>/dev/null || { echo "vr build failed"; exit 1; }
timeout -k 10 120 $O/vr.bin > $O/vr.log 2>&1 || { cat $O/vr.log; exit 1; }
cat $O/vr.log
timeout -k 10 300 python -u -m pytest tests/test_batch_golden.py tests/test_gpu_seal.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-open --no-derive > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
python -c "import json;d=json.load(open('$O/b.json'));h=d['host_inclusive'];print(d['value'], h['pinned'], h['pageable'], h['pcie_ceiling'])"
bash tools/pmc_kernels.sh cfg5 gpurun_out/r02ab_cfg5 > $O/pmc5.log 2>&1 || { tail -5 $O/pmc5.log; exit 1; }
echo done
