#!/bin/bash
# r02aj: rocprofv3 --kernel-trace --stats of the bench for cfg2..cfg5 (profiles/r02/stats_*).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02aj
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in cfg2 cfg3 cfg4 cfg5; do
  st=20; [ $c = cfg4 ] && st=4
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o run -- \
      python $R/bench.py --config $c --steps $st --warmup 2 --no-check --no-cpu --no-host-inclusive --no-open --no-derive > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$c.json'));print('$c', d['value'], d['roofline']['kernel'], d['roofline']['kernel_avg_ms'])"
done
echo done
