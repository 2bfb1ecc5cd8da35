#!/bin/bash
# Same-box A/B of environment settings on the cfg2 headline (alternating per round).
# Usage (GPU box): bash tools/ab_env.sh <outdir> <rounds> "VAR=a" "VAR=b" ...   ("-" = no setting)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
N=$2
shift 2
mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  for v in "$@"; do
    tag=$(echo "$v" | tr '=/' '__')
    if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py --no-host-inclusive --no-open --no-derive --no-cpu > $O/${tag}_$i.json 2> $O/${tag}_$i.err || { tail -20 $O/${tag}_$i.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/${tag}_$i.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['ms_per_seal_call'], d['bit_exact'])"
  done
done
