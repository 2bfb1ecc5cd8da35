#!/bin/bash
# Pipelined cfg2 seal under different CBC/MAC wave priorities (TLSGPU_DEBUG_SKIP bits 4-7).
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in 0 80 144 208 112 160; do
  echo -n "skip=$v "
  TLSGPU_DEBUG_SKIP=$v timeout -k 10 120 python $R/bench.py --no-check --no-cpu --no-host-inclusive --no-open --steps 100 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['ms_per_seal_call'])" || exit 1
done
