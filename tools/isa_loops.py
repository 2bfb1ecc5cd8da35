"""Instruction mix of the loops of one kernel in a --save-temps .s file (diagnostic tool):
for every backward branch, the instruction counts of the block range it closes.
  python tools/isa_loops.py <file.s> <symbol-prefix>"""
import re
import sys

src, sym = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sym) and l.rstrip().endswith(sym.split(":")[0]) is False
             or (l.startswith(sym) and ":" in l))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("s_endpgm"))
body = lines[start:end + 1]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(body):
    m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        cnt, ops = {}, {}
        for x in body[labels[m.group(1)]:i + 1]:
            x = x.strip()
            if not x or x[0] in ";." or x.endswith(":"):
                continue
            op = x.split()[0]
            k = ("ds" if op.startswith("ds_") else "valu" if op.startswith("v_") else "salu" if op.startswith("s_")
                 else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other")
            cnt[k] = cnt.get(k, 0) + 1
            ops[op] = ops.get(op, 0) + 1
        top = sorted(ops.items(), key=lambda t: -t[1])[:14]
        print("%s (%d-%d): %s\n   %s" % (m.group(1), labels[m.group(1)], i, cnt, " ".join("%s:%d" % t for t in top)))
