#!/bin/bash
# r02w: kernel timeline of the cfg3 pipeline; cfg4 cipher time against the chain count.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr3 -o run -- \
    python $R/bench.py --config cfg3 --steps 6 --warmup 2 --no-check --no-cpu --no-host-inclusive --no-open --no-derive > $O/cfg3.json 2> $O/cfg3.err || { tail -5 $O/cfg3.err; exit 1; }
python $R/tools/trace_timeline.py $O/tr3 12 > $O/cfg3_timeline.txt
cd $R
for n in 256 1024 2048; do
  timeout -k 10 300 python bench.py --config cfg4 --records $n --steps 2 --warmup 1 --no-check --no-cpu --no-host-inclusive --no-open --no-derive > $O/cfg4_$n.json 2> $O/cfg4_$n.err || { tail -5 $O/cfg4_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/cfg4_$n.json'));print('cfg4 conns $n', d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
done
echo done
