#!/bin/bash
# PMC of the dominant kernels after the whole-line stores (cfg2, cfg3, cfg5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_pmcfinal4
mkdir -p $O
for c in cfg2 cfg3 cfg5; do
  bash tools/pmc_kernels.sh $c $O/pmc_$c > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $O/pmc_$c.log; exit 1; }
  cp $R/profiles/pmc_$c.json $O/pmc_$c.json
  python -c "
import json;d=json.load(open('$O/pmc_$c.json'));k=d['dominant_kernel'];v=d['kernels'][k];print('$c', k, round(v['duration_ms'],3), 'hbm', v['hbm_bytes'], 'call', d['seal_call_hbm_bytes'])"
done
