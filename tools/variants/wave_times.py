"""Per-workgroup timing of the blend kernels on the C3 frame (GPU tool).

Needs a library built with -DGS_WAVE_TIMES (tools/build_variant.sh wt
-DGS_WAVE_TIMES): every k_blend_fwd / k_blend_bwd workgroup records its start
and end on the 100 MHz real-time clock and the XCD it ran on.  Reports, per
kernel, the occupancy over the launch (how many workgroups were resident),
the tail (the time the launch spends below 90 % of its peak residency), and
list-scheduling estimates of the makespan for other dispatch orders (the
workgroup durations replayed on the measured number of slots per XCD).

    GS_LIB_PATH=ab/wt.so python tools/wave_times.py
"""
from __future__ import annotations

import ctypes as C
import heapq
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

TICK_US = 0.01  # s_memrealtime: 100 MHz


def simulate(durations, order, slots):
    """Greedy list scheduling: workgroups start in `order` on the first free
    slot; returns the makespan."""
    free = [0.0] * slots
    heapq.heapify(free)
    end = 0.0
    for i in order:
        t = heapq.heappop(free)
        t1 = t + durations[i]
        end = max(end, t1)
        heapq.heappush(free, t1)
    return end


def analyse(name, t, nblk, tiles, ncell, extra_orders):
    t0 = t[:nblk, 0].astype(np.int64)
    t1 = t[:nblk, 1].astype(np.int64)
    xcc = (t[:nblk, 2] >> np.uint64(32)).astype(np.int64) & 0xF
    ran = t1 > 0
    base = t0[ran].min()
    s = (t0 - base) * TICK_US
    e = (t1 - base) * TICK_US
    d = e - s
    span = e[ran].max()
    print(f"== {name}: {ran.sum()} workgroups, span {span:.1f} us, duration mean {d[ran].mean():.2f} "
          f"p50 {np.median(d[ran]):.2f} p99 {np.percentile(d[ran], 99):.2f} max {d[ran].max():.2f} us")
    ev = np.concatenate([np.stack([s[ran], np.ones(ran.sum())], 1), np.stack([e[ran], -np.ones(ran.sum())], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    peak = conc.max()
    dt = np.diff(ev[:, 0], append=ev[-1, 0])
    avg = (conc * dt).sum() / span
    below = conc < 0.9 * peak
    # the tail: from the last time residency was >= 90 % of peak to the end
    last_full = ev[:, 0][~below].max() if (~below).any() else 0.0
    print(f"   residency: peak {peak:.0f}, mean {avg:.0f} ({avg / peak:.3f} of peak); "
          f"tail below 90 % of peak: {span - last_full:.1f} us; "
          f"work / (peak x span) = {d[ran].sum() / (peak * span):.3f}")
    per_x = [(e[ran & (xcc == x)].max() if (ran & (xcc == x)).any() else 0.0) for x in range(8)]
    print("   per-XCD end (us): " + " ".join(f"{v:.1f}" for v in per_x))
    # list scheduling per XCD (workgroup b on XCD b % 8), slots = peak / 8
    slots = max(1, int(round(peak / 8)))
    idx = np.arange(nblk)
    def mk(order):
        return max(simulate(d, [i for i in order if i % 8 == x], slots) for x in range(8))
    sim_id = mk(idx)
    print(f"   list-scheduling model, {slots} slots per XCD: dispatch order {sim_id:.1f} us (measured {span:.1f})")
    lpt = idx[np.argsort(-d, kind="stable")]
    # LPT within each XCD queue (the dispatcher's XCD of a block stays b % 8)
    print(f"   ideal LPT per XCD: {max(simulate(d, sorted([i for i in idx if i % 8 == x], key=lambda i: -d[i]), slots) for x in range(8)):.1f} us; "
          f"lower bound (work / slots): {max(d[idx % 8 == x].sum() / slots for x in range(8)):.1f} us")
    for label, order in extra_orders(d):
        print(f"   {label}: {mk(order):.1f} us")
    return d


def main():
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from stubs import Cam
    dev = torch.device("cuda", 0)
    W, H = 1920, 1080
    sc = pkg.synthetic.make_scene(1_000_000, W, H, seed=0)
    m = pkg.synthetic.to_model(sc, pkg.GaussianModel, dev)
    g = torch.Generator().manual_seed(1)
    cot = [(torch.rand(s, generator=g) * 2 - 1).to(dev) for s in ((3, H, W), (1, H, W), (1, H, W))]
    for _ in range(4):
        for p in m.grad_parameters():
            p.grad = None
        out = pkg.GaussianRenderer().render(Cam(W, H, sc.fovx, sc.fovy), m, pkg.RenderSettings(H, W, torch.zeros(3)))
        torch.autograd.backward([out["image"], out["alpha"], out["depth"]], cot)
    torch.cuda.synchronize()
    lib = pkg._native.load()
    tiles_x, tiles_y = (W + 15) // 16, (H + 15) // 16
    tiles = tiles_x * tiles_y
    ncell = 4
    nblk = ((tiles + 7) // 8) * 8 * ncell
    buf = (C.c_ulonglong * (nblk * 3))()
    res = {}
    for which, name in ((0, "k_blend_fwd"), (1, "k_blend_bwd")):
        assert lib.gs_debug_wave_times(which, buf, C.c_size_t(nblk * 24)) == 0
        res[name] = np.frombuffer(buf, dtype=np.uint64).reshape(nblk, 3).copy()

    def blk_tile(b):
        grp = b >> 3
        return (grp // ncell) * 8 + (b & 7), grp % ncell

    b = np.arange(nblk)
    tile_of, cell_of = blk_tile(b)

    def tile_orders(d):
        # keep the b -> XCD rule (b % 8) and the tile's cells together; order
        # the tiles of each XCD by their cells' summed time, longest first
        tsum = np.zeros(((tiles + 7) // 8) * 8)
        np.add.at(tsum, tile_of, d)
        out = []
        order = []
        for x in range(8):
            tx = np.arange(x, len(tsum), 8)
            tx = tx[np.argsort(-tsum[tx], kind="stable")]
            order.append(tx)
        # rebuild a block order: group k of XCD x = its k-th heaviest tile's cells
        blocks = []
        for k in range(len(order[0])):
            for c in range(ncell):
                for x in range(8):
                    t = order[x][k]
                    # the block that renders (tile t, cell c) in the launch
                    blocks.append(((t // 8) * ncell + c) * 8 + (t & 7))
        out.append(("tiles heaviest first (per XCD)", np.array(blocks)))
        return out

    fr = analyse("k_blend_fwd", res["k_blend_fwd"], nblk, tiles, ncell, tile_orders)
    bk = analyse("k_blend_bwd", res["k_blend_bwd"], nblk, tiles, ncell, tile_orders)
    ok = (fr > 0) & (bk > 0)
    print(f"correlation of a cell's fwd and bwd durations: {np.corrcoef(fr[ok], bk[ok])[0, 1]:.3f}")
    # what the forward could hand the backward as a predictor: per cell, its fwd time
    out_path = os.path.join(ROOT, "gpurun_out", "wave_times.npz")
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    np.savez_compressed(out_path, fwd=res["k_blend_fwd"], bwd=res["k_blend_bwd"])
    print("saved", out_path)


if __name__ == "__main__":
    main()
