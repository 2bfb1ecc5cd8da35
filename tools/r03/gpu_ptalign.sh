#!/bin/bash
# cfg3 plaintext records on 128-B boundaries (bench default) vs packed at 16 B (TLSGPU_BENCH_PT_ALIGN=16)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_ptalign
mkdir -p $O
timeout -k 10 300 python bench.py --config cfg3 --steps 100 --warmup 100 --no-host-inclusive --no-derive --no-cpu > $O/check.json 2> $O/check.err || { tail -20 $O/check.err; exit 1; }
python -c "
import json;d=json.load(open('$O/check.json'));print('check cfg3 a128', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')}, d['open']['value'], d['open']['roundtrip_exact'])"
for i in 1 2 3; do for a in 128 16; do
  TLSGPU_BENCH_PT_ALIGN=$a timeout -k 10 300 python bench.py --config cfg3 --steps 200 --warmup 200 --no-host-inclusive --no-open --no-derive --no-cpu --no-check > $O/a${a}_$i.json 2> $O/a${a}_$i.err || { tail -20 $O/a${a}_$i.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/a${a}_$i.json'));print('cfg3 align $a', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
done; done
