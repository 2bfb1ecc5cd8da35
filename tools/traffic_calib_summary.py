"""Per kernel of tools/traffic_calib.hip: FETCH_SIZE / WRITE_SIZE (KiB) of the last dispatch
against the payload bytes (diagnostic tool).  Usage: traffic_calib_summary.py <dir> <payload>"""
import csv
import glob
import os
import re
import sys

d, payload = sys.argv[1], int(sys.argv[2])
vals = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"])
        key = (k, r["Counter_Name"])
        vals.setdefault(key, {})
        vals[key][r["Dispatch_Id"]] = vals[key].get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
for (k, c), per in sorted(vals.items()):
    last = per[max(per, key=int)]
    print("%-10s %-10s %14.0f KiB  = %.3f x payload" % (k, c, last, last * 1024 / payload))
