"""Mean kernel durations from a rocprofv3 kernel_trace.csv, grouped by kernel
name and grid size (skips each group's first 3 launches as warm-up).
usage: python tools/trace_by_grid.py <kernel_trace.csv> [name-substring]"""
import collections
import csv
import re
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if len(sys.argv) > 2 and sys.argv[2] not in n:
        continue
    m = re.search(r"(\w+(<[^>]*>)?)\(", n.replace("(anonymous namespace)::", ""))
    k = m.group(1) if m else n[:40]
    d[(k, r["Grid_Size_X"], r["Grid_Size_Y"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    t = v[3:] if len(v) > 5 else v
    print(f"{k[0]:28s} grid {k[1]:>7s} x {k[2]:>4s}  n={len(v):4d}  {sum(t) / len(t) / 1e3:8.1f} us")
