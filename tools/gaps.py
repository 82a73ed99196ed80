"""Idle gaps between consecutive kernels per training step, from a
rocprofv3 --kernel-trace CSV (steps delimited by k_adam).
usage: python tools/gaps.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
for si in range(1, len(idx)):
    a, b = idx[si - 1], idx[si]
    prev = int(rows[a]["End_Timestamp"])
    gaps = []
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-24:]
        gaps.append(((s - prev) / 1000, name))
        prev = e
    step = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1000
    big = " ".join(f"{g:.0f}>{n}" for g, n in gaps if g > 8)
    print(f"step {si:2d} {step:8.1f} us  idle {sum(max(g, 0) for g, _ in gaps):6.1f} us  {big}")
