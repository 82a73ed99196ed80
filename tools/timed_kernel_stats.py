"""Per-kernel average duration over the last launches of a rocprofv3 kernel
trace: the bench's timed and diagnostic steps, without the spin-up launches
that run while the GPU clock ramps (rocprofv3 --stats averages over all).
usage: python tools/timed_kernel_stats.py <run_kernel_trace.csv> <last_n_launches_of_blend_bwd>"""
import collections
import csv
import re
import sys


def main():
    path, last = sys.argv[1], int(sys.argv[2])
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the timed region starts at the last_n-th from last blend backward launch
    # minus one step: take launches from the (last)-th from last k_blend_fwd on
    fwd = [i for i, r in enumerate(rows) if "k_blend_fwd" in r["Kernel_Name"]]
    start = fwd[-last] if len(fwd) >= last else 0
    per = collections.defaultdict(list)
    for r in rows[start:]:
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:60]
        per[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print(f"# {path}: launches from the {last}-th last k_blend_fwd on")
    print(f"{'kernel':44s} {'calls':>5s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s}")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:44s} {len(v):5d} {sum(v) / len(v):9.1f} {min(v):9.1f} {max(v):9.1f}")


if __name__ == "__main__":
    main()
