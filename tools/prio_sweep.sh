#!/bin/bash
# Pipelined cfg2 seal under different kernel choices / wave priorities
# (TLSGPU_CBC_ILP, TLSGPU_DEBUG_SKIP bits 4-7).  Timing experiments only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-cfg2}
for combo in "1 0" "2 0" "1 80" "1 144" "1 208" "1 112" "2 80" "2 144"; do
  set -- $combo
  echo -n "ilp=$1 skip=$2 "
  TLSGPU_CBC_ILP=$1 TLSGPU_DEBUG_SKIP=$2 timeout -k 10 120 python $R/bench.py --config $CFG --no-check --no-cpu \
      --no-host-inclusive --no-open --steps 100 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['ms_per_seal_call'])" || exit 1
done
