#!/bin/bash
# cfg3 / cfg5 at the driver's short step counts (20 timed + 5 warmup), beside the record runs'
# 500 + 500, to show the short-run gap per config.  One step at a time, each under its own limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_short
mkdir -p $O
for c in cfg3 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['bit_exact'], d['timed_bit_exact'])"
done
