#!/bin/bash
# Same-call A/B of library builds (tools/build_ab.sh) on one bench config.
#   bash tools/ab_bench.sh <outdir> <config> <rounds> <variant> [<variant> ...]
# variant "base" = the product library; any other name = tools/ab/<name>/libtlsgpu.so.
# Extra bench arguments can be passed in AB_ARGS.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; CFG=$2; N=$3
shift 3
mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  for v in "$@"; do
    if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
    timeout -k 10 300 python bench.py --config $CFG --no-host-inclusive --no-open --no-derive --no-cpu --no-check $AB_ARGS \
        > $O/${CFG}_${v}_$i.json 2> $O/${CFG}_${v}_$i.err || { tail -20 $O/${CFG}_${v}_$i.err; exit 1; }
    python -c "
import json;d=json.load(open('$O/${CFG}_${v}_$i.json'));o=d.get('open') or {};print('$CFG $v', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['ms_per_seal_call'], 'open', o.get('value'), (o.get('concurrent') or {}).get('value'))"
  done
done
unset TLSGPU_LIB
