#!/bin/bash
# shader clock during long cfg2 pipelined runs: product vs noload (MAC without its loads) vs nomac
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_clock2
mkdir -p $O
(timeout 20 rocm-smi --showclocks > $O/smi_probe.txt 2>&1; true)
for v in base noload nomac; do
  if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
  timeout -k 10 300 python bench.py --config cfg2 --no-host-inclusive --no-open --no-derive --no-cpu --no-check --steps 8000 --warmup 5 > $O/$v.json 2> $O/$v.err &
  BP=$!
  sleep 5
  for i in $(seq 1 30); do timeout 10 rocm-smi --showclocks 2>&1 | grep -E "sclk|fclk|mclk" | head -3 >> $O/clk_$v.txt; echo "--" >> $O/clk_$v.txt; sleep 0.4; done
  wait $BP || exit 1
  python -c "import json;d=json.load(open('$O/$v.json'));print('$v', d['value'], d['ms_per_step'])"
  grep -c sclk $O/clk_$v.txt; grep sclk $O/clk_$v.txt | sort | uniq -c | sort -rn | head -6
done
