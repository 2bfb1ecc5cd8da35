#!/bin/bash
# Build experiment variants of libtlsgpu.so (same sources, one compile-time switch
# each; see the TG_AB_* list in tlslite_amd/csrc/tg_aes3.h) into tools/ab/<name>/.
# The product library (tlslite_amd/lib) is never an A/B build.
#   bash tools/build_ab.sh name1=-DFLAG1 name2=-DFLAG2 ...   (CPU box; hipcc cross-compiles)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  python "$R/tlslite_amd/build.py" --out "$R/tools/ab/$name" ${flags//,/ } > /dev/null &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la "$R"/tools/ab/*/libtlsgpu.so
