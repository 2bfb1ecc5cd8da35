"""Summarize tools/pmc_kernels.sh passes: per kernel (name stem), the median
over full-size dispatches of every counter, the kernel's median duration,
and the per-seal-call HBM traffic -> profiles/pmc_<cfg>.json.

FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads 1/2 of the
bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM), so HBM bytes =
(2*FETCH_SIZE + WRITE_SIZE)*1024, the raw sum recorded beside it.  SQ cycle
counters (SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_*) count quad-cycles."""
import csv
import glob
import json
import os
import re
import statistics
import sys

out, cfg = sys.argv[1], sys.argv[2]


def stem(name):
    m = re.search(r"tg::(\w+)(<[^>]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name.split("(")[0][:60]


counters = {}   # stem -> counter -> {dispatch: value}
durations = {}  # stem -> [ns]
for f in glob.glob(os.path.join(out, "g*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = stem(r["Kernel_Name"])
        d = counters.setdefault(k, {}).setdefault(r["Counter_Name"], {})
        key = (f, r["Dispatch_Id"])
        d[key] = d.get(key, 0.0) + float(r["Counter_Value"])
for f in glob.glob(os.path.join(out, "g*", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        durations.setdefault(stem(r["Kernel_Name"]), []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))

res = {"config": cfg, "kernels": {}}
for k, cs in counters.items():
    row = {}
    for c, vals in cs.items():
        v = list(vals.values())
        top = max(v) if v else 0
        v = [x for x in v if x >= 0.5 * top]  # full-batch dispatches only
        row[c] = statistics.median(v) if v else 0
    ds = durations.get(k, [])
    if ds:
        top = max(ds)
        row["duration_ms"] = statistics.median([x for x in ds if x >= 0.3 * top]) / 1e6
    res["kernels"][k] = row
tf = sum(r.get("FETCH_SIZE", 0) for r in res["kernels"].values())
tw = sum(r.get("WRITE_SIZE", 0) for r in res["kernels"].values())
res["fetch_kib_raw"] = tf
res["write_kib"] = tw
res["hbm_bytes_per_launch_raw"] = int((tf + tw) * 1024)
res["hbm_bytes_per_launch"] = int((2 * tf + tw) * 1024)
res["note"] = ("per seal call (sum over its kernels); hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 "
               "(gfx950 FETCH_SIZE halves wide reads)")
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with open(os.path.join(root, "profiles", "pmc_%s.json" % cfg), "w") as fh:
    json.dump(res, fh, indent=1)
print(json.dumps(res, indent=1))
