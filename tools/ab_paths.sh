#!/bin/bash
# A/B of the AES seal memory paths on the pipelined cfg2 bench: every combination of
# TLSGPU_CBC_IO (column words default / 16) and TLSGPU_MAC_LOAD (per-lane default / quad),
# plus extra "VAR=value" sets given as arguments.  One line per variant.
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {
  echo -n "$* : "
  env "$@" timeout -k 10 120 python $R/bench.py --no-check --no-cpu --no-host-inclusive --no-open --steps 60 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('GiB/s', d['value'], 'step', d['ms_per_step'], 'cbc', d['roofline']['kernel_avg_ms'], 'call', d['ms_per_seal_call'])" || exit 1
}
run TLSGPU_X=default
run TLSGPU_CBC_IO=16
run TLSGPU_MAC_LOAD=quad
run TLSGPU_CBC_IO=16 TLSGPU_MAC_LOAD=quad
run TLSGPU_DEBUG_SKIP=2
for v in "$@"; do run $v; done
run TLSGPU_X=default
