#!/bin/bash
# cfg2 pipeline: the MAC stream idles from the end of MAC(k+1) to the end of cipher(k) in the trace;
# more workspaces (ws4, ws6) and no workspace-reuse wait at all (nowait, timing only) vs base;
# rocprofv3 kernel trace of each for the overlap
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=gpurun_out/r03_pipews
mkdir -p $O
bash tools/ab_bench.sh $O cfg2 2 base ws4 ws6 nowait || exit 1
cd /tmp && export TMPDIR=/tmp
for v in base nowait; do
  if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof_$v -o run -- \
      python3 $R/bench.py --config cfg2 --no-check --no-cpu --no-host-inclusive --no-open --no-derive --steps 10 --warmup 1 > $R/$O/prof_$v.json 2>&1 || exit 1
done
