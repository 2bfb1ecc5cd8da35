#!/bin/bash
# Same-box A/B of builds of libtlsgpu.so on the cfg2 headline, alternating
# base, alt1, alt2, ... per round; box-to-box variation is ~10 %, so only
# same-call comparisons are meaningful.
# Usage (GPU box): bash tools/ab_lib.sh <outdir> <rounds> <alt .so> [<alt .so> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
N=$2
shift 2
mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  for v in base "$@"; do
    tag=$(basename $v .so)
    if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/$v; fi
    timeout -k 10 300 python bench.py --no-host-inclusive --no-open --no-derive --no-cpu > $O/${tag}_$i.json 2> $O/${tag}_$i.err || { tail -20 $O/${tag}_$i.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/${tag}_$i.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['ms_per_seal_call'], d['bit_exact'])"
  done
done
