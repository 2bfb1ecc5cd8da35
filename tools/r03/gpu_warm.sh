#!/bin/bash
# cfg2 value vs warmup / steps (does the GPU reach a faster steady state under sustained load?)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_warm
mkdir -p $O
for ws in "5 50" "500 50" "500 500" "2000 200" "5 50"; do
  set -- $ws
  timeout -k 10 300 python bench.py --config cfg2 --no-host-inclusive --no-open --no-derive --no-cpu --no-check --warmup $1 --steps $2 > $O/w$1_s$2.json 2> $O/w$1_s$2.err || { tail -20 $O/w$1_s$2.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/w$1_s$2.json'));print('warmup $1 steps $2', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
done
