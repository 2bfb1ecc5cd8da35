#!/bin/bash
# Same-call A/B of library builds under rocprofv3 --kernel-trace --stats (cfg bench,
# pipelined): per variant the bench line and the per-kernel average durations.
#   bash tools/ab_prof.sh <outdir> <config> <variant> [<variant> ...]   (base = product lib)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; CFG=$2
shift 2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = base ]; then unset TLSGPU_LIB; else export TLSGPU_LIB=$R/tools/ab/$v/libtlsgpu.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- \
      python3 $R/bench.py --config $CFG --no-check --no-cpu --no-host-inclusive --no-open --no-derive --steps 30 \
      > $O/$v.json 2> $O/$v.err || { echo "rocprof $v failed"; tail -20 $O/$v.err; exit 1; }
  python3 - "$O/$v" "$O/$v.json" "$v" <<'PY'
import csv, glob, json, sys
d = json.load(open(sys.argv[2]))
stats = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
ks = {}
for f in stats:
    for r in csv.DictReader(open(f)):
        n = r["Name"].split("(")[0].replace("void ", "")
        ks[n] = float(r["AverageNs"]) / 1e6
print(sys.argv[3], d["value"], d["ms_per_step"], " ".join("%s=%.3f" % (k, v) for k, v in sorted(ks.items()) if v > 0.05))
PY
done
unset TLSGPU_LIB
