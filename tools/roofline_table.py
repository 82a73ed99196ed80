"""Per-kernel HBM roofline table of one step: algorithmic bytes (SURVEY 8(d)'s
per-unit models x the frame's counts), the PMC traffic of the same build
(profiles/pmc_current.txt: 2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction
of MI355X_MICROARCH.md; raw FETCH + WRITE beside it) and the timed-region
kernel durations (tools/timed_kernel_stats.py output).

The frame's counts come from a bench line (bench.py's `config`: gaussians,
visible M, tile touches T, records consumed R, live (entry, cell) pairs L,
width x height) -- not from constants (a hard-coded L of
11.54 M, two atomic requests per live pair, had overstated the gather's bytes).

usage: python tools/roofline_table.py profiles/pmc_current.txt <kernel_stats_timed.txt> <bench.log>"""
import json
import re
import sys

PEAK = 8000.0  # GB/s (HBM3E spec)
SORT_CHUNK = 2048  # radix sort block (gs_internal.h kSortBlockEntries)
ALIAS = {"k_tile_ranges4": "k_tile_ranges"}  # (four positions per thread at the default tile: the same model)


def counts_from_bench(line: dict) -> dict:
    """The counts the byte models need, from one bench JSON line."""
    c = line["config"]
    W, H = int(c["width"]), int(c["height"])
    return {"N": int(c["gaussians"]), "M": int(c["visible"]), "T": int(c["tile_touches"]),
            "R": int(c["records_consumed"]), "L": int(c["live_entry_cells"]), "HW": W * H,
            "TILES": ((W + 15) // 16) * ((H + 15) // 16)}


def bench_line(path: str) -> dict:
    """The last JSON line of a bench log."""
    for ln in reversed(open(path).read().strip().splitlines()):
        ln = ln.strip()
        if ln.startswith("{"):
            return json.loads(ln)
    raise ValueError(f"no bench JSON line in {path}")


def model(k: dict, fused_adam: bool = False) -> dict:
    """kernel -> (launches per step, algorithmic bytes per step, model text).
    fused_adam: the replayed step's projection backward applies the Adam update
    itself (gs_project_backward_adam): no gradient written or re-read, the
    moments and the updated parameters moved there, no k_adam launch."""
    N, M, T, R, L, HW, TILES = (k[x] for x in ("N", "M", "T", "R", "L", "HW", "TILES"))
    nb_n, nb_t = -(-N // SORT_CHUNK), -(-T // SORT_CHUNK)
    return {
        "k_project_fwd": (1, (56 + 85) * N, "56 B/G read + 85 B/G write"),
        "k_radix_hist": (3, 4 * N + 2 * 4 * T, "4 B/key: depth MSD pass on N, 2 tile passes on T"),
        "k_radix_scan": (3, 8 * (256 * nb_n + 64 * nb_t + 128 * nb_t), "per-block digit counts, read + write"),
        "k_radix_scatter": (3, 12 * N + 2 * 16 * T, "depth: 4 read + 8 write per key; tile: 8 + 8 per entry, 2 passes"),
        "k_msd_bucket_sort": (1, 16 * N, "8 B/G read + 8 B/G write"),
        "k_bin_partials": (1, 33 * N, "ids 4 + gathered rects 8 + own rects 8 + vis 1 read, rects 8 + offsets 4 "
                                      "written, per G"),
        "k_bin_scan_partials": (1, 20 * -(-N // 1024), "5 words per 1024-G block"),
        "k_bin_emit": (1, 24 * N + 8 * T, "16 B/G read + 8 B/G written, 8 B/entry written"),
        "k_tile_ranges": (1, 8 * T + 8 * TILES, "4 B/entry keys read + 4 B/entry slot flags zeroed + 8 B/tile"),
        "k_blend_fwd": (1, 44 * R + 8 * TILES + 28 * HW, "44 R + 8 tiles + 28 HW"),
        "k_blend_bwd": (1, 44 * R + 36 * HW + 40 * M, "44 R + 36 HW + 40 M"),
        "k_gather_slots": (1, 40 * L + 4 * T + 40 * N, "40 B per live (entry, cell) L + 4 B/slot flags read, "
                                                      "40 B/G written"),
        "k_project_bwd": (1, 196 * N, "40 B/G sums + ~100 B/G read, 56 B/G written"),
        "k_adam": (1, 392 * N, "14 floats/G x (param, m, v, grad read + param, m, v written)"),
        "k_project_bwd_adam": (1, 420 * N, "40 B/G sums + ~100 B/G read; Adam fused: 14 floats/G x (m, v read + "
                                           "param, m, v written)"),
    } if not fused_adam else {k: v for k, v in model(k, False).items() if k not in ("k_project_bwd", "k_adam")} | {
        "k_project_bwd_adam": model(k, False)["k_project_bwd_adam"]}


def pmc(path):
    out, cur = {}, None
    for line in open(path):
        if line.startswith("#"):
            continue
        if not line.startswith(" "):
            cur = ALIAS.get(line.strip(), line.strip())
            out[cur] = {}
        elif cur:
            k, v = line.split()
            out[cur][k] = float(v)
    return out


def timed(path):
    out = {}
    for line in open(path):
        m = re.match(r"(k_\w+)(<[^>]*>)?\s+(\d+)\s+([\d.]+)", line)
        if m:
            k = m.group(1)
            if k == "k_project_bwd" and (m.group(2) or "").replace(" ", "") == "<true,true>":
                k = "k_project_bwd_adam"  # (the projection backward with the Adam update fused in)
            k = ALIAS.get(k, k)
            calls, avg = int(m.group(3)), float(m.group(4))
            tot = out.get(k, (0, 0.0))
            out[k] = (tot[0] + calls, tot[1] + calls * avg)
    return {k: v[1] / v[0] for k, v in out.items()}


def table(p: dict, t: dict, counts: dict) -> str:
    lines = [f"# counts (from the bench line): " + ", ".join(f"{k}={v:,}" for k, v in counts.items()),
             f"{'kernel':20s} {'launch/step':>11s} {'us/step':>8s} {'alg MB':>8s} {'PMC MB':>8s} {'raw MB':>8s} "
             f"{'alg GB/s':>9s} {'frac':>6s} {'PMC/alg':>7s}  model"]
    tot_us = tot_alg = 0.0
    fused = "k_project_bwd_adam" in t  # (the replayed step with the optimizer in the backward)
    for k, (n, alg, text) in model(counts, fused).items():
        if k not in t or k not in p:
            continue
        us = t[k] * n
        c = p[k]
        traffic = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 * n
        raw = (c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 * n
        gbs = alg / (us * 1e-6) / 1e9
        tot_us += us
        tot_alg += alg
        lines.append(f"{k:20s} {n:11d} {us:8.1f} {alg / 1e6:8.1f} {traffic / 1e6:8.1f} {raw / 1e6:8.1f} {gbs:9.0f} "
                     f"{gbs / PEAK:6.3f} {traffic / alg:7.2f}  {text}")
    if tot_us:
        lines.append(f"{'all of the above':20s} {'':11s} {tot_us:8.1f} {tot_alg / 1e6:8.1f} {'':8s} {'':8s} "
                     f"{tot_alg / (tot_us * 1e-6) / 1e9:9.0f} {tot_alg / (tot_us * 1e-6) / 1e9 / PEAK:6.3f}")
    return "\n".join(lines)


def main():
    print(table(pmc(sys.argv[1]), timed(sys.argv[2]), counts_from_bench(bench_line(sys.argv[3]))))


if __name__ == "__main__":
    main()
