"""Gaps between consecutive launches of one kernel in a rocprofv3 kernel trace (diagnostic
tool): for the kernel whose name contains <substr>, the median duration, the median gap from
one launch's end to the next one's start, and what else ran in the gaps.
  python tools/trace_gaps.py <trace dir> <substr>"""
import csv
import glob
import statistics
import sys

d, sub = sys.argv[1], sys.argv[2]
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
ev.sort()
mine = [e for e in ev if sub in e[2]]
mine = mine[len(mine) // 4:]  # steady state: drop the first quarter (set-up, warmup)
durs = [(e - s) / 1e6 for s, e, _ in mine]
gaps = [(mine[i + 1][0] - mine[i][1]) / 1e6 for i in range(len(mine) - 1)]
print("%s: %d launches, duration median %.4f ms, gap median %.4f ms (min %.4f max %.4f)"
      % (sub, len(mine), statistics.median(durs), statistics.median(gaps), min(gaps), max(gaps)))
# other kernels overlapping each gap
inside = {}
for i in range(len(mine) - 1):
    a, b = mine[i][1], mine[i + 1][0]
    for s, e, n in ev:
        if s < b and e > a and sub not in n:
            k = n.split("(")[0][-50:]
            inside[k] = inside.get(k, 0) + 1
for k, v in sorted(inside.items(), key=lambda t: -t[1])[:8]:
    print("   in gaps: %4d x %s" % (v, k))
