"""Model of VERDICT r05 item 2: hide the gradient gather and the projection
backward in k_blend_bwd's launch tail, band by band of tile rows.

Inputs (CPU only):
  * the measured per-workgroup start / end of one C3 blend backward
    (gpurun_out/wave_times.npz of round 3, tools/variants/wave_times.py; the
    summary is profiles/r03/wave_times_order0.log);
  * the C3 frame's tile rectangles (the oracle's projection of the bench
    scene, oracle/ -- the checker, used here only as a calculator).

Scheme modelled: the blend backward counts finished workgroups per tile row;
once every workgroup of the launch has started (so nothing the gather waits
for still needs a slot), a gather + projection-backward kernel on a second
stream fills the slots the blend's tail leaves idle, taking the Gaussians in
the order their last tile row completes (a Gaussian is final once every row
its rectangle touches is done).  Fluid approximation: the tail kernels
progress at the idle fraction of the GPU (1 - resident / peak) while the blend
runs and at full rate after; their total cost is their measured duration alone
(work_us, both kernels), spread evenly over the visible Gaussians.

Prints the step time saved against running them after the blend backward.
usage: python tools/band_overlap_model.py [work_us ...]"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
TICK_US = 0.01
W, H, N_G, TILE = 1920, 1080, 1_000_000, 16
TX, TY = (W + TILE - 1) // TILE, (H + TILE - 1) // TILE


def blend_rows(npz_path):
    t = np.load(npz_path)["bwd"]
    t0, t1 = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    ran = t1 > 0
    base = t0[ran].min()
    s, e = (t0 - base) * TICK_US, (t1 - base) * TICK_US
    b = np.arange(len(t))
    grp = b >> 3
    tile = (grp // 4) * 8 + (b & 7)
    row = np.where(tile < TX * TY, tile // TX, -1)
    row_done = np.zeros(TY)
    for r in range(TY):
        m = ran & (row == r)
        row_done[r] = e[m].max() if m.any() else 0.0
    # residency over time (1 us grid)
    span = e[ran].max()
    grid = np.arange(0.0, span + 1.0, 0.5)
    res = np.zeros_like(grid)
    ss, ee = np.sort(s[ran]), np.sort(e[ran])
    res = np.searchsorted(ss, grid, side="right") - np.searchsorted(ee, grid, side="right")
    return row_done, grid, res, res.max(), span, s[ran].max()


def rects():
    import torch
    sys.path.insert(0, os.path.join(ROOT, "mini-3d-gaussian-splatting_amd"))
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from oracle import oracle as orc
    sc = pkg.synthetic.make_scene(N_G, W, H, seed=0)
    cov = orc.covariance(sc.scaling.numpy(), sc.rotation.numpy())
    s = orc.Scene(xyz=sc.xyz.numpy(), cov3d=cov, color_logits=sc.features_dc[:, 0].numpy(),
                  opacity=torch.sigmoid(sc.opacity[:, 0]).numpy(), wv=np.eye(4), width=W, height=H,
                  fovx=sc.fovx, fovy=sc.fovy, bg=np.zeros(3, np.float32))
    o = orc.render_forward(s, nthreads=os.cpu_count())
    m, rad, vis = o["means2d"], o["radii"], o["vis"].astype(bool)
    r = rad.astype(np.int64)  # int() of a positive radius
    cy = np.trunc(m[:, 1]).astype(np.int64)
    y0, y1 = np.maximum(cy - r, 0), np.minimum(cy + 1 + r, H)
    ok = vis & (y1 > y0)
    return (y0[ok] // TILE), ((y1[ok] - 1) // TILE)


def model(row_done, grid, res, peak, span, all_started, ty0, ty1, work_us):
    # a Gaussian is final when the last-completing row of its rectangle is
    cummax = np.maximum.accumulate(row_done)  # (rows finish nearly in order; exact max below)
    ready = np.array([row_done[a:b + 1].max() for a, b in zip(ty0, ty1)]) if len(ty0) < 200_000 else None
    if ready is None:  # vectorised: sparse table over rows
        lo, hi = ty0, ty1
        best = np.zeros(len(lo))
        for r in range(TY):
            inr = (lo <= r) & (r <= hi)
            best = np.where(inr, np.maximum(best, row_done[r]), best)
        ready = best
    ready = np.maximum(ready, all_started)
    w = work_us / len(ready)  # GPU-us per Gaussian
    order = np.sort(ready)
    dt = grid[1] - grid[0]
    t, done, i = 0.0, 0.0, 0
    n = len(order)
    cap_at = lambda tt: 1.0 if tt >= span else 1.0 - res[min(int(tt / dt), len(res) - 1)] / peak
    backlog_done = 0.0
    while backlog_done < n:
        avail = np.searchsorted(order, t, side="right")
        can = cap_at(t) * dt / w
        backlog_done = min(avail, backlog_done + can) if avail > backlog_done else backlog_done
        t += dt
        if t > span + 10 * work_us:
            break
    return t, span + work_us, cummax


def main():
    # each argument: work_us, or serial_us:overlapped_us (the tail kernels'
    # cost in index order after the blend, and in band order during it)
    works = [tuple(float(v) for v in x.split(":")) if ":" in x else (float(x), float(x)) for x in sys.argv[1:]] \
        or [(141.6, 141.6)]
    npz = os.path.join(ROOT, "gpurun_out", "wave_times.npz")
    row_done, grid, res, peak, span, all_started = blend_rows(npz)
    ty0, ty1 = rects()
    print(f"blend backward: span {span:.1f} us, peak residency {peak}, every workgroup started by "
          f"{all_started:.1f} us; rows done (us): first {row_done.min():.1f}, median {np.median(row_done):.1f}, "
          f"last {row_done.max():.1f}; rows out of order: {(np.diff(row_done) < 0).sum()} of {TY - 1}")
    idle = np.clip(1.0 - res / peak, 0, 1)
    dt = grid[1] - grid[0]
    after = grid >= all_started
    print(f"idle GPU after every workgroup started: {(idle[after] * dt).sum():.1f} us x GPU "
          f"(of which before the last row completes: {(idle[after & (grid < row_done.max())] * dt).sum():.1f})")
    print(f"visible Gaussians with a rectangle: {len(ty0):,}; last row median {np.median(ty1):.0f}")
    for ws, wo in works:
        t_overlap, _, _ = model(row_done, grid, res, peak, span, all_started, ty0, ty1, wo)
        t_serial = span + ws
        print(f"tail work {ws:.1f} us after the blend (index order) vs {wo:.1f} us overlapped (band order): "
              f"serial end {t_serial:.1f} us, overlapped end {t_overlap:.1f} us, saved {t_serial - t_overlap:.1f} us "
              f"(before the band lists' own cost)")


if __name__ == "__main__":
    main()
