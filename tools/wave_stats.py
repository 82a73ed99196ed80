"""Per-wave work statistics of the blend kernels on the C3 frame (GPU tool).

For every (tile, list entry, 8x8 wave quadrant) it counts
  processed  entries a wave walks (up to its deepest lane's last evaluated entry)
  live       processed entries where some lane has s <= 23.1 (exp(-s/2) >= 1e-5)
  bbox       processed entries whose s<=L ellipse bounding box (L = 23.1 * 1.001)
             overlaps the quadrant's pixel centres
so that wave-level culling can be priced before it is written.
    python tools/wave_stats.py [--gaussians N]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from mini3dgs_amd import rasterizer as RZ
    dev = torch.device("cuda", 0)
    W, H = a.width, a.height
    scene = pkg.synthetic.make_scene(a.gaussians, W, H, seed=0)
    model = pkg.synthetic.to_model(scene, pkg.GaussianModel, dev)

    class Cam:
        _width, _height, _FoVx, _FoVy = W, H, scene.fovx, scene.fovy

        def world_view_transform(self):
            return torch.eye(4)

    settings = pkg.RenderSettings(image_height=H, image_width=W, bg_color=torch.zeros(3))
    camp = pkg.camera_params(Cam(), settings)
    with torch.no_grad():
        pn = torch.empty((H * W,), dtype=torch.int32, device=dev)
        *_, fr = RZ.forward_pipeline(camp, model._xyz, None, model._scaling, model._rotation,
                                     model._features_dc[:, 0, :], torch.sigmoid(model._opacity).squeeze(1),
                                     pix_neval=pn)
    tx_n, ty_n = camp.tiles_x, camp.tiles_y
    ranges = fr.ranges.view(-1, 2).long().cpu()
    neval = pn.view(H, W).long()
    pad = torch.zeros(ty_n * 16, tx_n * 16, dtype=torch.long, device=dev)
    pad[:H, :W] = neval
    # per (tile, quadrant) deepest lane
    qmax = pad.view(ty_n, 2, 8, tx_n, 2, 8).amax(dim=(2, 5))  # [ty, qy, tx, qx]
    qmax = qmax.permute(0, 2, 1, 3).reshape(ty_n * tx_n, 4)    # quadrant q = qx + 2 qy
    L = 23.1 * 1.001
    tot = {k: torch.zeros((), dtype=torch.long, device=dev)
           for k in ("processed", "live", "bbox", "live_notbbox", "bwd_lockstep", "bwd_max", "bwd_sum",
                     "bwd_entries", "bwd_entries_live", "bwd_live_max", "bwd_live_sum",
                     "h_processed", "h_live", "v_processed", "v_live", "lanes_live", "h_bwd_max", "h_bwd_sum")}
    ys, xs = torch.meshgrid(torch.arange(8, device=dev), torch.arange(8, device=dev), indexing="ij")
    ys, xs = ys.reshape(-1).float(), xs.reshape(-1).float()
    num_tiles = tx_n * ty_n
    for t0 in range(0, num_tiles, 256):
        t1 = min(num_tiles, t0 + 256)
        for t in range(t0, t1):
            s0, e0 = int(ranges[t, 0]), int(ranges[t, 1])
            if e0 <= s0:
                continue
            gid = fr.sorted_gauss[s0:e0].long()
            rec = fr.records[gid]  # [n,12]
            n = rec.shape[0]
            tx, ty = t % tx_n, t // tx_n
            mx, my, q00, q11, qo = rec[:, 0:1], rec[:, 1:2], rec[:, 2:3], rec[:, 3:4], rec[:, 4:5]
            det = q00 * q11 - 0.25 * qo * qo
            sxx, syy = q11 / det, q00 / det
            hx, hy = torch.sqrt(L * sxx), torch.sqrt(L * syy)
            qx = torch.tensor([0., 8., 0., 8.], device=dev)
            qy = torch.tensor([0., 0., 8., 8.], device=dev)
            px = tx * 16 + qx[:, None] + xs[None, :]   # [4,64]
            py = ty * 16 + qy[:, None] + ys[None, :]
            dx = px[None] - mx[:, :, None]
            dy = py[None] - my[:, :, None]
            sq = dx * dx * q00[:, :, None] + qo[:, :, None] * dx * dy + dy * dy * q11[:, :, None]
            proc = torch.arange(n, device=dev)[:, None] < qmax[t][None, :]     # [n,4]
            live = proc & (sq <= 23.1).any(dim=2)
            x0, y0 = tx * 16 + qx, ty * 16 + qy
            bb = ((mx + hx >= x0[None]) & (mx - hx <= x0[None] + 7) &
                  (my + hy >= y0[None]) & (my - hy <= y0[None] + 7))
            # halves: rows (top/bottom 16x8: quadrants {0,1},{2,3}) and
            # columns (left/right 8x16: {0,2},{1,3}); a half processes an entry
            # up to its deepest lane, and is live if some lane of it is
            lvq = (sq <= 23.1)                                                  # [n,4,64]
            for key, pairs in (("h", ((0, 1), (2, 3))), ("v", ((0, 2), (1, 3)))):
                for a_, b_ in pairs:
                    ph = torch.arange(n, device=dev) < torch.maximum(qmax[t][a_], qmax[t][b_])
                    tot[key + "_processed"] += ph.sum()
                    tot[key + "_live"] += (ph & (lvq[:, a_].any(1) | lvq[:, b_].any(1))).sum()
            tot["lanes_live"] += (lvq & proc[:, :, None]).sum()
            hstop = int(qmax[t].max())
            if hstop > 0:
                hl = torch.stack([live[:hstop, 0] | live[:hstop, 1], live[:hstop, 2] | live[:hstop, 3]], 1).float()
                nbh = (hstop + 15) // 16
                hp = torch.zeros(nbh * 16, 2, device=dev)
                hp[:hstop] = hl
                perh = hp.view(nbh, 16, 2).sum(1)
                tot["h_bwd_max"] += (2 * perh.max(1).values).sum().long()
                tot["h_bwd_sum"] += perh.sum().long()
            tot["processed"] += proc.sum()
            tot["live"] += live.sum()
            tot["bbox"] += (proc & bb).sum()
            tot["live_notbbox"] += (live & ~bb).sum()
            # backward: batches of 16 up to the tile's deepest entry; per batch
            # a lockstep block pays 16 entries in every wave (no culling), the
            # culled block the busiest wave's count, decoupled waves their own
            stop = int(qmax[t].max())
            if stop > 0:
                work = (proc & bb)[:stop].float()                     # [stop, 4]
                nb = (stop + 15) // 16
                wpad = torch.zeros(nb * 16, 4, device=dev)
                wpad[:stop] = work
                per = wpad.view(nb, 16, 4).sum(1)                     # [nb, 4]
                tot["bwd_lockstep"] += 4 * stop
                tot["bwd_max"] += (4 * per.max(1).values).sum().long()
                tot["bwd_sum"] += per.sum().long()
                # exact liveness (what the forward's bitmap holds), and batches
                # formed from entries with at least one live quadrant
                lv = live[:stop]
                anyq = lv.any(1)
                tot["bwd_entries"] += stop
                tot["bwd_entries_live"] += anyq.sum()
                lvc = lv[anyq].float()
                nl = lvc.shape[0]
                if nl:
                    nb2 = (nl + 15) // 16
                    lpad = torch.zeros(nb2 * 16, 4, device=dev)
                    lpad[:nl] = lvc
                    per2 = lpad.view(nb2, 16, 4).sum(1)
                    tot["bwd_live_max"] += (4 * per2.max(1).values).sum().long()
                    tot["bwd_live_sum"] += per2.sum().long()
    tot = {k: int(v) for k, v in tot.items()}
    print(tot)
    print(f"backward phase-A wave-entries: lockstep {tot['bwd_lockstep']}, culled+barrier {tot['bwd_max']}, "
          f"decoupled {tot['bwd_sum']}")
    print(f"backward entries up to the tile stop {tot['bwd_entries']}, with a live quadrant {tot['bwd_entries_live']}; "
          f"compacted batches: busiest-wave {tot['bwd_live_max']}, decoupled {tot['bwd_live_sum']}")
    p = tot["processed"]
    print(f"halves: rows live/processed {tot['h_live']}/{tot['h_processed']}, cols {tot['v_live']}/{tot['v_processed']}; "
          f"quadrant live wave-entries {tot['live']} -> half (rows) {tot['h_live']} "
          f"(x2 pixels/lane: {2 * tot['h_live'] / max(1, tot['live']):.3f} of the quadrant cost per entry-pixel-lane); "
          f"lane efficiency in live quadrant wave-entries {tot['lanes_live'] / max(1, 64 * tot['live']):.3f}; "
          f"bwd phase-A halves busiest-wave {tot['h_bwd_max']} decoupled {tot['h_bwd_sum']}")
    print(f"live/processed = {tot['live'] / p:.3f}, bbox/processed = {tot['bbox'] / p:.3f}, "
          f"evaluated pairs (E) = {int(neval.sum())}, processed lane-pairs = {64 * p}")


if __name__ == "__main__":
    main()
