#!/bin/bash
# A/B of the CBC lane layouts (TLSGPU_CBC_LAYOUT=pair|quad) after the seal parity tests.
# Usage (GPU box): bash tools/ab_layout.sh <outdir>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${1:-gpurun_out/ab_layout}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_seal.py tests/test_gpu_open.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in cfg2 cfg3; do
  for lay in pair quad; do
    TLSGPU_CBC_LAYOUT=$lay timeout -k 10 300 python bench.py --config $cfg --no-host-inclusive --no-open --no-derive --no-cpu > $O/${cfg}_$lay.json 2> $O/${cfg}_$lay.err || { tail -20 $O/${cfg}_$lay.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/${cfg}_$lay.json'));print('$cfg $lay', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['ms_per_seal_call'], d['bit_exact'])"
  done
done
