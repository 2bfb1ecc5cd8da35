"""Print the GPU timeline (kernels + memory copies) of the last `window` ms of a
rocprofv3 trace directory (diagnostic tool): start offset, duration, kind, name."""
import csv
import glob
import sys

d, window = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:40], r.get("Queue_Id", "")))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", "?"), ""))
ev.sort()
end = max(e[1] for e in ev)
t0 = end - window * 1e6
sel = [e for e in ev if e[1] >= t0]
base = sel[0][0]
for s, e, k, n, q in sel:
    print("%9.3f %8.3f %s %-42s %s" % ((s - base) / 1e6, (e - s) / 1e6, k, n, q))
