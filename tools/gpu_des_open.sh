#!/bin/bash
# open path: RC4 open decrypting + MACing 64-byte chunks from registers; parity, then
# cfg5 open and a cfg2 seal A/B against the previous commit's library (tools/ab/prev)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02o4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_open.py tests/test_keys_loopback.py tests/test_gpu_factory.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config cfg5 --steps 5 --warmup 1 --no-host-inclusive --no-cpu --no-derive > $O/cfg5.json 2> $O/cfg5.err || { tail -20 $O/cfg5.err; exit 1; }
python -c "import json;d=json.load(open('$O/cfg5.json'));print('cfg5', d['value'], d['bit_exact'], d['open']['value'], d['open']['ms'], d['open']['roundtrip_exact'])"
bash tools/ab_bench.sh $O/ab cfg2 3 base prev || exit 1
