"""Summarize FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh into
profiles/pmc_traffic_<cfg>.json (per-launch HBM bytes of the seal kernel).

FETCH_SIZE and WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reads 1/2 of the
bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM); both the raw and
the x2-corrected read figure are recorded."""
import csv
import glob
import json
import os
import statistics
import sys

out, cfg = sys.argv[1], sys.argv[2]


def per_dispatch(counter):
    files = glob.glob(os.path.join(out, counter, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        rows += [r for r in csv.DictReader(open(f)) if "seal" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    vals = {}
    for r in rows:
        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    top = max(vals.values())  # full-batch launches only (sub-batch launches are far smaller)
    return [v for v in vals.values() if v > 0.5 * top]


f = per_dispatch("FETCH_SIZE")
w = per_dispatch("WRITE_SIZE")
fk, wk = statistics.median(f), statistics.median(w)
res = {"config": cfg, "dispatches": [len(f), len(w)],
       "fetch_kib_raw": fk, "write_kib": wk,
       "hbm_bytes_per_launch_raw": int((fk + wk) * 1024),
       "hbm_bytes_per_launch": int((2 * fk + wk) * 1024),
       "note": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halves wide reads)"}
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with open(os.path.join(root, "profiles", "pmc_traffic_%s.json" % cfg), "w") as fh:
    json.dump(res, fh, indent=1)
print(json.dumps(res))
