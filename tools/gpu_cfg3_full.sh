#!/bin/bash
# cfg3 and cfg5 at bench.py's default step counts (50 timed, 5 warmup: a 10-step run pays the
# pipeline's first, unoverlapped MAC phase on 1/10 of the steps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r02final4b
mkdir -p $O
for c in cfg3 cfg5; do
  timeout -k 10 400 python bench.py --config $c --no-host-inclusive > $O/bench_${c}_50.json 2> $O/bench_${c}_50.err || { tail -20 $O/bench_${c}_50.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_${c}_50.json'));print('$c', d['value'], d['ms_per_step'], d['bit_exact'], d['roofline']['kernel_avg_ms'], d['open']['value'])"
done
# PMC traffic of cfg3's many-chains configuration -> profiles/pmc_cfg3.json (box-side; copied back via gpurun_out)
bash tools/pmc_kernels.sh cfg3 $O/pmc3 > $O/pmc3.log 2>&1 || { tail -20 $O/pmc3.log; exit 1; }
cp profiles/pmc_cfg3.json $O/pmc_cfg3.json
python -c "import json;d=json.load(open('$O/pmc_cfg3.json'));print(d['dominant_kernel'], d['hbm_bytes_per_launch'], d['seal_call_hbm_bytes'])"
