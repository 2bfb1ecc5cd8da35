#!/bin/bash
# r02final: full GPU tests + every config on the final round-2 tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02final
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -20 $O/bench_cfg2.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench_cfg2.json'));print({k:d[k] for k in ('value','ms_per_step','bit_exact','ms_per_seal_call')}, d['roofline']['kernel_avg_ms'], d['host_inclusive'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
for c in cfg3 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-host-inclusive > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -20 $O/bench_$c.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/bench_$c.json'));print('$c', {k:d[k] for k in ('value','ms_per_step','bit_exact')}, d['roofline']['kernel'], d['roofline']['kernel_avg_ms'])"
done
timeout -k 10 300 python bench.py --config cfg4 --records 512 --steps 5 --warmup 1 --no-host-inclusive --no-cpu > $O/bench_cfg4_512.json 2> $O/bench_cfg4_512.err || { tail -20 $O/bench_cfg4_512.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench_cfg4_512.json'));print('cfg4/512', {k:d[k] for k in ('value','ms_per_step','bit_exact')})"
echo done
