#!/bin/bash
# r02s: host pipeline stream placement: high-priority copy streams (base), CU-masked
# streams (cumask), all normal priority (normprio); with and without torch's stream pools.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s
mkdir -p $O
cd $R
for v in base cumask normprio; do
  for tp in none torchpool; do
    if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
    echo "$v $tp: $(timeout -k 10 120 python tools/hostpipe_one.py 64 3 $tp 2> $O/${v}_$tp.err | tr '\n' ' ')" || exit 1
  done
done
