"""Phase-A lane efficiency of the blend backward at a bench config
(gs_blend_backward_lane_stats), and a model of one
compaction scheme on its per-(tile, cell) counts.

Per replayed (entry, cell) the kernel's counting instantiation records the
lanes still running into the entry (transmittance not terminated) and the
lanes whose pair contributes (weight > 0); per workgroup (tile, cell) the
replays and the replays entered with >= 32 running lanes.  Running lanes
only ever drop along a cell's replay, so a cell's replays with < 32 running
lanes are a suffix of it: its "tail".

The modeled scheme (the review's example): once two cells of a tile both run
with < 32 lanes, one wave takes over the surviving pixels of both and replays
the rest of both lists.  Its best case per tile (the four cells' tails t1 >=
t2 >= t3 >= t4 paired (1,2), (3,4), the merged wave replaying max(t_a, t_b)
entries: the two tails' lists coincide) saves t2 + t4 replays.  The
saving is priced at phase A's per-replay cost: phase A is ~65 % of the
kernel (round 2 ablation, DESIGN.md section 4: 318 of 493 us without phase
B); phase B (one partial per (entry, cell)) does not shrink, since a merged
wave still writes each cell's partial.

usage: python tools/lane_stats.py [config]   (C1 / C2 / C3; default C3)"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

PHASE_A_SHARE = 318.0 / 493.0


def run(config="C3", seed=0):
    import __graft_entry__ as ge
    import bench
    pkg = ge.load_package()
    N = pkg._native
    from mini3dgs_amd import rasterizer as RZ
    from stubs import Cam
    n, W, H = bench.CONFIGS[config]
    dev = torch.device("cuda", 0)
    sc = pkg.synthetic.make_scene(n, W, H, seed=seed)
    m = pkg.synthetic.to_model(sc, pkg.GaussianModel, dev)
    camp = pkg.camera_params(Cam(W, H, sc.fovx, sc.fovy), pkg.RenderSettings(H, W, torch.zeros(3)))
    g = torch.Generator().manual_seed(1)
    gi, ga, gd = [(torch.rand(s, generator=g) * 2 - 1).to(dev) for s in ((3, H, W), (1, H, W), (1, H, W))]
    lib = N.load()
    saved, RZ._FRAME_CALLS = RZ._FRAME_CALLS, False
    try:
        pair_counts = torch.zeros((H * W,), dtype=torch.int32, device=dev)
        out = RZ.forward_pipeline(camp, m._xyz, None, m._scaling, m._rotation, m._features_dc, m._opacity,
                                  opacity_is_logit=True, pair_counts=pair_counts, need_grad=True)
    finally:
        RZ._FRAME_CALLS = saved
    image, alpha, depth = out[:3]
    fr = out[7]
    T, G = fr.T, fr.groups
    live = fr.live_bits

    def args(pg, sl):
        return N.GsBlendBwdArgs(camp.to_struct(), camp.tiles_x, camp.tiles_y, N.ptr(fr.ranges),
                                N.ptr(fr.sorted_gauss), N.ptr(fr.records), N.ptr(image), N.ptr(alpha), N.ptr(depth),
                                N.ptr(fr.pix_flags), N.ptr(fr.cell_neval), N.ptr(gi), N.ptr(ga), N.ptr(gd), N.ptr(live), 0 if live is None else live.shape[1],
                                N.ptr(pg), N.ptr(sl), T, 0, 0)
    s = N.stream_ptr()
    pg0 = torch.zeros((T * G, N.GS_PARTIAL_STRIDE), dtype=torch.float32, device=dev)
    sl0 = torch.zeros((T * G,), dtype=torch.uint8, device=dev)
    a0 = args(pg0, sl0)
    N.check(lib.gs_blend_backward(C.byref(a0), s), "gs_blend_backward")
    pg1 = torch.zeros_like(pg0)
    sl1 = torch.zeros_like(sl0)
    a1 = args(pg1, sl1)
    ng = int(lib.gs_blend_backward_groups(camp.tiles_x, camp.tiles_y, 4))
    hist = torch.zeros((2, 65), dtype=torch.int64, device=dev)
    per = torch.empty((ng, 4), dtype=torch.int32, device=dev)
    N.check(lib.gs_blend_backward_lane_stats(C.byref(a1), N.ptr(hist), N.ptr(per), s), "lane stats")
    torch.cuda.synchronize()
    same = bool(torch.equal(pg0.view(torch.int32), pg1.view(torch.int32)) and torch.equal(sl0, sl1))
    return {"config": config, "n": n, "W": W, "H": H, "T": T, "hist": hist.cpu().numpy(),
            "per": per.cpu().numpy().astype(np.int64), "tiles": camp.tiles_x * camp.tiles_y,
            "contributing_fwd": int(pair_counts.to(torch.int64).sum()), "same_partials": same}


def model(r):
    per, tiles = r["per"], r["tiles"]
    ng = per.shape[0]
    b = np.arange(ng)
    grp = b >> 3
    tile = (grp // 4) * 8 + (b & 7)
    ok = tile < tiles
    rep, rep32 = per[:, 0], per[:, 1]
    tails = np.zeros((tiles, 4), np.int64)
    tails[tile[ok], (grp % 4)[ok]] = (rep - rep32)[ok]
    ts = -np.sort(-tails, axis=1)
    saved = int((ts[:, 1] + ts[:, 3]).sum())
    return {"replays": int(rep.sum()), "replays_ge32": int(rep32.sum()), "tail_replays": int((rep - rep32).sum()),
            "saved_replays_best_case": saved}


def report(r, out=sys.stdout):
    h = r["hist"]
    reps = int(h[0].sum())
    run_l = int((h[0] * np.arange(65)).sum())
    con_l = int((h[1] * np.arange(65)).sum())
    md = model(r)
    p = lambda *a: print(*a, file=out)  # noqa: E731
    p(f"# phase-A lane statistics, {r['config']}: {r['n']:,} Gaussians {r['W']}x{r['H']}, T = {r['T']:,} "
      f"(gs_blend_backward_lane_stats; tools/lane_stats.py)")
    p(f"stats instantiation writes the product kernel's partials: {r['same_partials']}")
    p(f"replayed (entry, cell) pairs: {reps:,}   lane-replays (x64): {64 * reps:,}")
    p(f"running lanes summed: {run_l:,} ({run_l / max(1, 64 * reps):.3f} of lane-replays)")
    p(f"contributing lanes summed: {con_l:,} ({con_l / max(1, 64 * reps):.3f} of lane-replays); "
      f"the forward's contributing pairs: {r['contributing_fwd']:,}")
    p(f"per-workgroup sums agree with the histogram: {md['replays'] == reps}")
    p("")
    p("lanes  replays_entered_with_this_many_running  replays_with_this_many_contributing")
    for k in range(65):
        p(f"{k:5d}  {int(h[0][k]):14,d}  {int(h[1][k]):14,d}")
    p("")
    frac = md["saved_replays_best_case"] / max(1, reps)
    p("model: pair the surviving pixels of two cells of a tile once both run with < 32 lanes")
    p(f"  replays entered with >= 32 running lanes: {md['replays_ge32']:,}; tails (< 32): {md['tail_replays']:,} "
      f"({md['tail_replays'] / max(1, reps):.3f})")
    p(f"  best-case replays saved (tails paired t1+t2, t3+t4 per tile, merged lists coinciding): "
      f"{md['saved_replays_best_case']:,} = {frac:.3f} of replays")
    p(f"  priced at phase A's share of the kernel ({PHASE_A_SHARE:.2f}): <= {frac * PHASE_A_SHARE:.3f} of "
      f"k_blend_bwd's time")
    return md


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    r = run(cfg)
    report(r)


if __name__ == "__main__":
    main()
