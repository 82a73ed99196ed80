"""GPU busy fraction of a kernel trace window: the union of the kernels'
[start, end) intervals over the span from the first to the last kernel, for
the launches between the `skip`-th k_blend_fwd and the `last`-th from the end
(e.g. a training run: its validation renders left out).
usage: python tools/busy_fraction.py <run_kernel_trace.csv> [skip_first_fwd] [skip_last_fwd]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    a = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    b = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    fwd = [i for i, r in enumerate(rows) if "k_blend_fwd" in r["Kernel_Name"]]
    lo = fwd[a] if a < len(fwd) else 0
    hi = fwd[len(fwd) - b] if b and b <= len(fwd) else len(rows)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[lo:hi])
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    nf = len([i for i in fwd if lo <= i < hi])
    print(f"{nf} forwards, {len(iv)} kernels: span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms "
          f"({busy / span:.3f}); per forward: span {span / 1e3 / max(nf, 1):.1f} us, busy {busy / 1e3 / max(nf, 1):.1f} us")


if __name__ == "__main__":
    main()
