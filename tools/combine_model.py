"""Model the blend backward's cell-combine options on a dumped C3 frame
(tools/live_dump.py): per (tile, entry) which of the tile's four 8x8 cells
replay the entry (the forward's liveness bits, cut at each cell's last
evaluated entry), then

  * the partials written per live entry today (one per live (entry, cell))
    against an ideal per-entry combine;
  * an opportunistic in-LDS combine of a tile's four cell waves in one
    workgroup, with a ring of R entry slots and no waiting: each wave's time
    is its own work (phase A per live entry, phase B per chunk of 8); an
    entry combines if its last live cell finishes it before any cell of the
    tile needs its ring slot for entry e + R (else its pieces spill as
    per-cell partials);
  * the workgroup's duration (the slowest of its four waves) against the
    waves' own durations -- what holding a 4-wave workgroup's slot costs.

    python tools/combine_model.py gpurun_out/live_c3.npz
"""
import sys

import numpy as np


def cell_lists(d):
    """Per tile: list length, per cell the sorted positions of its live entries."""
    live = d["live_bits"].view(np.uint64)
    ranges = d["ranges"].astype(np.int64)
    W, H = int(d["W"]), int(d["H"])
    neval = d["neval"].reshape(H, W)
    tx_n = (W + 15) // 16
    ty_n = (H + 15) // 16
    pad = np.zeros((ty_n * 16, tx_n * 16), np.int64)
    pad[:H, :W] = neval
    # per (tile, cell): the cell's last evaluated entry (max n_eval)
    cells = pad.reshape(ty_n, 2, 8, tx_n, 2, 8).max(axis=(2, 5))  # [ty, qy, tx, qx]
    out = []
    for t in range(tx_n * ty_n):
        s, e = ranges[t]
        n = e - s
        ty, tx = divmod(t, tx_n)
        lists = []
        for q in range(4):
            qy, qx = divmod(q, 2)
            wstop = int(cells[ty, qy, tx, qx])
            if wstop == 0 or n == 0:
                lists.append(np.zeros(0, np.int64))
                continue
            nw = (wstop + 63) // 64
            base = s // 64 + t
            words = live[q, base:base + nw]
            bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:wstop]
            lists.append(np.nonzero(bits)[0].astype(np.int64))
        out.append((n, lists))
    return out


def times(pos, a=1.0, b=4.0, word=0.5):
    """Finish time of each live entry of one cell wave: a per live entry
    (phase A), b per phase-B chunk (<= 8 live entries of one 64-entry word),
    `word` per word visited.  An entry is done when its chunk's phase B is."""
    if len(pos) == 0:
        return pos.astype(float)
    w = pos // 64
    fin = np.empty(len(pos))
    t = 0.0
    i = 0
    lastw = -1
    while i < len(pos):
        if w[i] != lastw:
            t += word
            lastw = w[i]
        j = i
        while j < len(pos) and j - i < 8 and w[j] == w[i]:
            j += 1
        t += a * (j - i) + b
        fin[i:j] = t
        i = j
    return fin


def main(path):
    d = np.load(path)
    tl = cell_lists(d)
    tot_live_pairs = sum(sum(len(l) for l in ls) for _, ls in tl)
    tot_entries = sum(n for n, _ in tl)
    uni = 0
    hist = np.zeros(5, np.int64)
    for n, ls in tl:
        cnt = np.zeros(n, np.int64)
        for l in ls:
            cnt[l] += 1
        hist += np.bincount(cnt, minlength=5)[:5]
        uni += int((cnt > 0).sum())
    print(f"tiles {len(tl)}  entries T {tot_entries}  live (entry, cell) {tot_live_pairs}  "
          f"live entries (any cell) {uni}  cells per live entry {tot_live_pairs / max(uni, 1):.3f}")
    print("entries by live cells 0..4:", hist.tolist())
    print(f"partials: per (entry, cell) {tot_live_pairs * 40 / 1e6:.1f} MB, per entry {uni * 40 / 1e6:.1f} MB, "
          f"pair (cells 0+1, 2+3) combine {sum_pairs(tl) * 40 / 1e6:.1f} MB")
    for R in (16, 32, 64, 128, 256, 1 << 20):
        parts, wg, own = 0, 0.0, 0.0
        for n, ls in tl:
            fins = [times(l) for l in ls]
            dur = [f[-1] if len(f) else 0.0 for f in fins]
            wg += max(dur)
            own += sum(dur)
            parts += ring_partials(n, ls, fins, R)
        print(f"ring R={R:>7}: partials {parts} ({parts * 40 / 1e6:.1f} MB, {parts / tot_live_pairs:.3f} of today)")
    print(f"4-wave workgroup: sum of slowest-wave durations x4 / sum of own durations = {4 * wg / own:.3f}")


def sum_pairs(tl):
    n_out = 0
    for n, ls in tl:
        for a, b in ((0, 1), (2, 3)):
            m = np.zeros(n, bool)
            m[ls[a]] = True
            m[ls[b]] = True
            n_out += int(m.sum())
    return n_out


def ring_partials(n, ls, fins, R):
    """Partials written with an R-slot ring and no waiting."""
    if n == 0:
        return 0
    last = np.full(n, -1.0)
    cnt = np.zeros(n, np.int64)
    for l, f in zip(ls, fins):
        last[l] = np.maximum(last[l], f)
        cnt[l] += 1
    # earliest time any cell finishes an entry at position >= e + R (needs e's slot)
    need = np.full(n, np.inf)
    for l, f in zip(ls, fins):
        if len(l) == 0:
            continue
        # for each e: first live entry of this cell at position >= e + R
        idx = np.searchsorted(l, np.arange(n) + R)
        ok = idx < len(l)
        t = np.full(n, np.inf)
        # the slot is needed when that entry's chunk starts writing: its finish time
        t[ok] = f[idx[ok]]
        need = np.minimum(need, t)
    live = cnt > 0
    combined = live & (last <= need)
    return int(combined.sum() + cnt[live & ~combined].sum())


if __name__ == "__main__" and len(sys.argv) == 2:
    main(sys.argv[1])


def chunks_of(pos, a=1.0, b=4.0, word=0.5):
    """(chunk index per live entry, chunk costs) of one cell wave."""
    if len(pos) == 0:
        return np.zeros(0, np.int64), np.zeros(0)
    w = pos // 64
    cid = np.empty(len(pos), np.int64)
    costs = []
    i, lastw = 0, -1
    while i < len(pos):
        c = 0.0
        if w[i] != lastw:
            c += word
            lastw = w[i]
        j = i
        while j < len(pos) and j - i < 8 and w[j] == w[i]:
            j += 1
        cid[i:j] = len(costs)
        costs.append(c + a * (j - i) + b)
        i = j
    return cid, np.array(costs)


def ring_wait(n, ls, R, iters=60):
    """4 cell waves of one workgroup, ring of R slots, waiting (no spills):
    an entry live in >= 2 cells occupies slot e mod R from its first
    deposit until its last; a deposit into a slot still held by an older
    entry waits for that entry's last deposit; a chunk ends when its last
    entry's deposit is done.  Returns (workgroup time, own times)."""
    cnt = np.zeros(n, np.int64)
    for l in ls:
        cnt[l] += 1
    ring = cnt >= 2
    # previous ring occupant of each entry's slot
    prev = np.full(n, -1, np.int64)
    lastocc = {}
    for e in np.nonzero(ring)[0]:
        prev[e] = lastocc.get(e % R, -1)
        lastocc[e % R] = e
    cc = [chunks_of(l) for l in ls]
    own = [float(c.sum()) if len(c) else 0.0 for _, c in cc]
    rel = np.zeros(n)  # release time of each ring entry
    dep = [np.zeros(len(l)) for l in ls]
    for _ in range(iters):
        new_rel = np.zeros(n)
        for q, l in enumerate(ls):
            cid, costs = cc[q]
            if len(l) == 0:
                continue
            need = np.where(ring[l] & (prev[l] >= 0), rel[np.maximum(prev[l], 0)], 0.0)
            t = 0.0
            d = dep[q]
            k0 = 0
            for k in range(len(costs)):
                k1 = k0
                while k1 < len(cid) and cid[k1] == k:
                    k1 += 1
                r = t + costs[k]
                dk = np.maximum(r, need[k0:k1])
                d[k0:k1] = dk
                t = float(dk.max())
                k0 = k1
            np.maximum.at(new_rel, l, d)
        if np.array_equal(new_rel, rel):
            break
        rel = new_rel
    ends = [float(d.max()) if len(d) else 0.0 for d in dep]
    return max(ends), own, ends


def wait_report(path, Rs=(8, 16, 24, 32, 64)):
    d = np.load(path)
    tl = cell_lists(d)
    rng = np.random.default_rng(0)
    sample = rng.choice(len(tl), size=min(1500, len(tl)), replace=False)
    for R in Rs:
        wg = own_sum = end_sum = maxown = 0.0
        for t in sample:
            n, ls = tl[t]
            if n == 0:
                continue
            m, own, ends = ring_wait(n, ls, R)
            wg += m
            own_sum += sum(own)
            end_sum += sum(ends)
            maxown += max(own)
        print(f"wait R={R:3d}: waves' end / own work {end_sum / own_sum:.3f}; workgroup (slowest wave) "
              f"{wg / maxown:.3f} x the slowest wave's own work; 4 x workgroup / own work {4 * wg / own_sum:.3f}")


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "wait":
    wait_report(sys.argv[1])
