#!/bin/bash
# Experiment builds of libtlsgpu.so: the product sources with tools/ab_overlay/tg_config.h in
# place of tlslite_amd/csrc/tg_config.h (the tuning constants, each overridable with a -D
# flag, e.g. -DTG_AB_PAIR_G1=4), one build per spec into tools/ab/<name>/.  The product
# library (tlslite_amd/lib) is never an experiment build.
#   bash tools/build_ab.sh name1=-DFLAG1 name2=-DFLAG2,-DFLAG3 ...   (CPU box; hipcc cross-compiles)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  [ "$flags" = "$spec" ] && flags=""
  python "$R/tlslite_amd/build.py" --force --out "$R/tools/ab/$name" --overlay "$R/tools/ab_overlay" ${flags//,/ } > /dev/null &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la "$R"/tools/ab/*/libtlsgpu.so
