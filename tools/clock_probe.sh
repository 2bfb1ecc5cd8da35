#!/bin/bash
# Shader clock under sustained cfg2 load, per library build ("base" = the product library,
# any other name = tools/ab/<name>/libtlsgpu.so): a long bench run in the background and
# rocm-smi samples during it.
#   bash tools/clock_probe.sh <outdir> <variant>...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1
shift
mkdir -p $O
cd $R
for v in "$@"; do
  if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
  timeout -k 10 300 python bench.py --config cfg2 --no-host-inclusive --no-open --no-derive --no-cpu --no-check \
      --steps 6000 --warmup 5 > $O/$v.json 2> $O/$v.err &
  BP=$!
  sleep 6
  for i in $(seq 1 20); do timeout 10 rocm-smi --showclocks 2>&1 | grep -E "sclk" | head -1 >> $O/clk_$v.txt; sleep 0.3; done
  wait $BP || { echo "bench $v failed"; tail -5 $O/$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
  sort $O/clk_$v.txt | uniq -c | sort -rn | head -4
done
unset TLSGPU_LIB
