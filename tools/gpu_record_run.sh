#!/bin/bash
# The record run of a round on one MI355X -- full GPU tests, smoke, every bench config, a
# 2-rank torch.distributed.run launch of bench.py (both ranks on this box's one GPU: the
# launcher's env contract and the shard rendezvous, not a scaling number), and rocprofv3
# kernel-trace statistics of each config.  Stops at the first failure.
#   bash tools/gpu_record_run.sh <tag>     (outputs under gpurun_out/<tag>)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-record}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -20 $O/bench_cfg2.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench_cfg2.json'));print({k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact','ms_per_seal_call')}, d['roofline']['kernel'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['roofline']['frac_of_copy'], d['roofline']['traffic'], d['host_inclusive'] and d['host_inclusive'].get('value'), d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
for c in cfg3 cfg4 cfg5; do
  st=""; [ $c = cfg4 ] && st="--steps 10 --warmup 2"
  timeout -k 10 400 python bench.py --config $c $st --no-host-inclusive > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -20 $O/bench_$c.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/bench_$c.json'));print('$c', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')}, d['roofline']['kernel'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['roofline']['traffic'])"
done
timeout -k 10 300 python bench.py --config cfg4 --records 512 --steps 5 --warmup 1 --no-host-inclusive --no-cpu > $O/bench_cfg4_512.json 2> $O/bench_cfg4_512.err || { tail -20 $O/bench_cfg4_512.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench_cfg4_512.json'));print('cfg4/512', {k:d[k] for k in ('value','ms_per_step','bit_exact','timed_bit_exact')})"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_cfg2_2ranks.json 2> $O/bench_cfg2_2ranks.err || { tail -30 $O/bench_cfg2_2ranks.err; exit 1; }
grep '^{' $O/bench_cfg2_2ranks.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
for c in cfg2 cfg3 cfg4 cfg5; do
  st=20; [ $c = cfg4 ] && st=3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- \
      python3 $R/bench.py --config $c --no-check --no-cpu --no-host-inclusive --no-open --no-derive --steps $st --warmup 1 > $O/bench_prof_$c.json 2> $O/bench_prof_$c.err \
      || { echo "rocprof $c failed"; tail -20 $O/bench_prof_$c.err; exit 1; }
done
echo done
