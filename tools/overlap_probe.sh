#!/bin/bash
# Pipelined cfg2 seal with parts of the work removed (TLSGPU_DEBUG_SKIP: 1 = no CBC
# bulk blocks, 2 = no MAC bulk chunks): how much the MAC phase of batch k+1 slows
# the CBC phase of batch k; 4096 / 8192 = CBC bulk without plaintext loads / ciphertext
# stores (cbc_bulk PROBE).  (The MAC-phase probes of round 1 -- compressions only, loads
# only, coalesced loads -- led to mac_bulk_quad and were removed.)  Timing experiments only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for skip in ${SKIPS:-0 2 1 4096 8192 0}; do
  echo -n "skip=$skip ilp=${TLSGPU_CBC_ILP:-1} "
  TLSGPU_DEBUG_SKIP=$skip timeout -k 10 120 python $R/bench.py --no-check --no-cpu --no-host-inclusive --no-open \
      --steps 60 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('GiB/s', d['value'], 'step', d['ms_per_step'], 'cbc', d['roofline']['kernel_avg_ms'], 'call', d['ms_per_seal_call'])" || exit 1
done
