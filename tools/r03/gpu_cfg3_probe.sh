#!/bin/bash
# timing-only probes of the pipelined cfg3 step: MAC without its plaintext loads (noload),
# no MAC compressions at all (nomac); plus the product GPU suite after the A/B pruning
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_cfg3probe
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_bench.sh $O cfg3 2 base noload nomac || exit 1
bash tools/ab_bench.sh $O cfg2 2 base nomac || exit 1
