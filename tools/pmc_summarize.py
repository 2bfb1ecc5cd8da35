"""Summarize tools/pmc_kernels.sh passes: per kernel (name stem), the median
over full-size dispatches of every counter, the kernel's median duration,
and its HBM traffic -> profiles/pmc_<cfg>.json.

FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reads 1/2 of the
bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM), so HBM bytes =
(2*FETCH_SIZE + WRITE_SIZE)*1024, the raw sum recorded beside it.  SQ cycle
counters (SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_*) count quad-cycles.

`hbm_bytes_per_launch` is the dominant kernel's traffic (the kernel whose
roofline bench.py reports); `seal_call_hbm_bytes` sums the kernels of one seal
call.  The bench's set-up kernels (synthetic plaintext fill, buffer zeroing)
are listed but excluded from both."""
import csv
import glob
import json
import os
import re
import statistics
import sys

out, cfg = sys.argv[1], sys.argv[2]
name = sys.argv[3] if len(sys.argv) > 3 else "pmc_%s" % cfg  # profiles/<name>.json
NCU = 256
# bench set-up: synthetic plaintext fill, buffer zeroing, state resets and the copy-rate
# measurement (d2d copies) -- not the seal call
SETUP = ("fill_kernel", "__amd_rocclr_fillBuffer", "__amd_rocclr_copyBuffer")
DOMINANT = ("cbc_pair_kernel", "cbc_kernel", "rc4_seal_kernel", "tdes4_kernel")
OPEN = ("open_", "rc4_open_kernel")  # the open path's kernels (bench.py --open): summed apart


def stem(name):
    m = re.search(r"tg::(\w+)(<[^>]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name.split("(")[0][:60]


def read_bytes(row):
    """HBM read bytes: exact from the request-size counters when collected, else the
    FETCH_SIZE doubling calibrated for wide streaming reads."""
    if "TCC_EA0_RDREQ_128B_sum" in row:
        return int(32 * row.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * row.get("TCC_EA0_RDREQ_64B_sum", 0)
                   + 128 * row["TCC_EA0_RDREQ_128B_sum"])
    return int(2 * row.get("FETCH_SIZE", 0) * 1024)


def hbm_bytes(row):
    return read_bytes(row) + int(row.get("WRITE_SIZE", 0) * 1024)


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
# the workload the passes sealed (bench.py's JSON line in each pass's log): bench.py attaches
# this file's traffic only to runs of the same workload and record count
for f in sorted(glob.glob(os.path.join(out, "g*.log"))):
    for line in open(f, errors="replace"):
        if line.startswith("{"):
            try:
                d = json.loads(line)
            except ValueError:
                continue
            res["workload"] = d["config"]["workload"]
            res["records"] = d["config"]["records_per_gpu"]
    if "workload" in res:
        break
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
    if "FETCH_SIZE" in row or "WRITE_SIZE" in row:
        row["hbm_bytes"] = hbm_bytes(row)
        row["read_bytes"] = read_bytes(row)
        row["read_bytes_2xfetch"] = int(2 * row.get("FETCH_SIZE", 0) * 1024)
    if row.get("duration_ms") and row.get("GRBM_GUI_ACTIVE"):
        cyc = row["GRBM_GUI_ACTIVE"] / 8  # per XCD
        row["clock_ghz"] = round(cyc / (row["duration_ms"] * 1e6), 3)
        # SQ_LDS_IDX_ACTIVE: LDS-array cycles summed over CUs (2 per conflict-free ds_read_b32)
        row["lds_busy"] = round(row.get("SQ_LDS_IDX_ACTIVE", 0) / NCU / cyc, 3)
        # wave64 VALU instructions per SIMD per cycle (x 2.5-4.2 cycles each = VALU busy)
        row["valu_inst_per_simd_cycle"] = round(row.get("SQ_INSTS_VALU", 0) / (4 * NCU) / cyc, 4)
    res["kernels"][k] = row

seal = {k: r for k, r in res["kernels"].items() if not k.startswith(SETUP) and not k.startswith(OPEN)}
opn = {k: r for k, r in res["kernels"].items() if k.startswith(OPEN)}
dom = [k for k in seal if k.startswith(DOMINANT)]
dom = max(dom, key=lambda k: seal[k].get("duration_ms", 0)) if dom else None
res["dominant_kernel"] = dom
res["hbm_bytes_per_launch"] = seal[dom].get("hbm_bytes") if dom else None
res["hbm_bytes_per_launch_raw"] = (int((seal[dom].get("FETCH_SIZE", 0) + seal[dom].get("WRITE_SIZE", 0)) * 1024)
                                   if dom else None)
res["seal_call_hbm_bytes"] = sum(r.get("hbm_bytes", 0) for r in seal.values())
if opn:
    res["open_call_hbm_bytes"] = sum(r.get("hbm_bytes", 0) for r in opn.values())
res["note"] = ("hbm_bytes_per_launch: the dominant kernel's HBM bytes per launch = reads from the "
               "request-size counters (32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B) + WRITE_SIZE*1024 "
               "(read_bytes_2xfetch: the FETCH_SIZE doubling, exact only for wide streaming reads); "
               "seal_call_hbm_bytes: sum over the seal call's kernels; set-up kernels (%s) excluded; "
               "clock = GRBM_GUI_ACTIVE / 8 XCDs / duration" % ", ".join(SETUP))
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with open(os.path.join(root, "profiles", name + ".json"), "w") as fh:
    json.dump(res, fh, indent=1)
print(json.dumps(res, indent=1))
