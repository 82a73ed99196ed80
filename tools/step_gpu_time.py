"""GPU busy time per step from a rocprofv3 kernel trace: over the last n
steps (counted by k_blend_fwd launches), the summed kernel durations and the
wall span from the first kernel start to the last kernel end, per step --
kernel sum close to the span: GPU-bound; far below: host-bound.
usage: python tools/step_gpu_time.py <run_kernel_trace.csv> <n_steps>"""
import csv
import sys


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    fwd = [i for i, r in enumerate(rows) if "k_blend_fwd" in r["Kernel_Name"]]
    if len(fwd) < n + 1:
        print("not enough steps")
        return
    a, b = fwd[-n - 1], fwd[-1]  # n whole steps between these forward launches
    seg = rows[a:b]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3
    span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
    print(f"{n} steps: kernels {busy / n:.1f} us/step busy, span {span / n:.1f} us/step, "
          f"{len(seg) / n:.1f} launches/step, GPU busy {busy / span:.3f}")


if __name__ == "__main__":
    main()
