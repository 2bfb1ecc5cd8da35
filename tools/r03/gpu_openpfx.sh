#!/bin/bash
# open_prefix_kernel: state header without short-circuit branches (product) vs prevop; open suite + open timings
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_openpfx
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_open.py tests/test_keys_loopback.py tests/test_session_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do for v in base prevop; do
  if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
  timeout -k 10 300 python bench.py --config cfg3 --steps 20 --warmup 20 --no-host-inclusive --no-derive --no-cpu --no-check > $O/cfg3_${v}_$i.json 2> $O/cfg3_${v}_$i.err || { tail -20 $O/cfg3_${v}_$i.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/cfg3_${v}_$i.json'));print('cfg3 $v open', d['open']['value'], d['open']['ms'], d['open']['roundtrip_exact'])"
done; done
unset TLSGPU_LIB
