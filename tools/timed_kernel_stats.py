"""Per-kernel average duration over the last launches of a rocprofv3 kernel
trace: the bench's timed and diagnostic steps, without the spin-up launches
that run while the GPU clock ramps (rocprofv3 --stats averages over all).
usage: python tools/timed_kernel_stats.py <run_kernel_trace.csv> <last_n> [skip_last]
  the region: from the (last_n + skip_last)-th last k_blend_fwd launch up to
  the skip_last-th last one (skip_last: the frames bench.py renders after its
  timed steps, e.g. 2 with --diag-steps 0); the last line sums every kernel of
  the region per step (region / last_n) and the span from its first kernel's
  start to its last kernel's end, per step."""
import collections
import csv
import re
import sys


def main():
    path, last = sys.argv[1], int(sys.argv[2])
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the timed region starts at the last_n-th from last blend backward launch
    # minus one step: take launches from the (last)-th from last k_blend_fwd on
    fwd = [i for i, r in enumerate(rows) if "k_blend_fwd" in r["Kernel_Name"]]
    start = fwd[-(last + skip)] if len(fwd) >= last + skip else 0
    end = fwd[-skip] if skip and len(fwd) >= skip else len(rows)
    per = collections.defaultdict(list)
    for r in rows[start:end]:
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:60]
        per[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print(f"# {path}: launches from the {last + skip}-th last k_blend_fwd on" +
          (f", up to the {skip}-th last" if skip else ""))
    print(f"{'kernel':44s} {'calls':>5s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s}")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:44s} {len(v):5d} {sum(v) / len(v):9.1f} {min(v):9.1f} {max(v):9.1f}")
    reg = rows[start:end]
    busy = sum(sum(v) for v in per.values())
    span = (max(int(r["End_Timestamp"]) for r in reg) - min(int(r["Start_Timestamp"]) for r in reg)) / 1000.0
    print(f"# per step: kernels {busy / last:.1f} us, span {span / last:.1f} us (first start to last end / {last})")


if __name__ == "__main__":
    main()
