#!/bin/bash
# Same-call A/B of the host-buffer pipeline's rate (bench.py's host_inclusive leg, cfg2)
# across library builds ("base" = the product library, else tools/ab/<name>/).
#   bash tools/hostpipe_ab.sh <outdir> <rounds> <variant>...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; N=$2
shift 2
mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  for v in "$@"; do
    if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
    timeout -k 10 300 python bench.py --config cfg2 --steps 20 --warmup 5 --no-cpu --no-check --no-open --no-derive \
        > $O/hp_${v}_$i.json 2> $O/hp_${v}_$i.err || { tail -20 $O/hp_${v}_$i.err; exit 1; }
    python3 -c "
import json;d=json.loads([l for l in open('$O/hp_${v}_$i.json') if l.startswith('{')][-1]);h=d['host_inclusive']
print('$v', 'pinned', h['pinned']['value'], h['pinned']['ms'], 'pageable', h['pageable']['value'], 'ceiling', h['pcie_ceiling'], 'exact', h['pinned']['bit_exact'], h['pageable']['bit_exact'])"
  done
done
unset TLSGPU_LIB
