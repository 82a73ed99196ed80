"""Debug the blend backward's ring combine (GPU tool): render a random
scene, run the backward with the per-entry partials, and report NaN
(timed-out, poisoned) partials by tile and list position, the kernel time,
and the gradient sums against a per-cell (GS_BWD_RING=0) library.
    python tools/ring_debug.py [n W H]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from stubs import Cam
    RZ = pkg.rasterizer
    N = pkg._native
    syn = pkg.synthetic
    dev = torch.device("cuda", 0)
    n, W, H = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (3000, 200, 152)
    sc = syn.make_scene(n, W, H, seed=21, sigma_range=(0.005, 0.03))
    m = syn.to_model(sc, pkg.GaussianModel, dev)
    cam = pkg.camera_params(Cam(W, H, sc.fovx, sc.fovy), pkg.RenderSettings(H, W, torch.zeros(3)))
    image, alpha, depth, means2d, conics, radii, vis, fr = RZ.forward_pipeline(
        cam, m._xyz.detach(), None, m._scaling.detach(), m._rotation.detach(), m._features_dc.detach()[:, 0, :],
        torch.sigmoid(m._opacity.detach()).squeeze(1), need_grad=True)
    torch.cuda.synchronize()
    print("T", fr.T, "groups", fr.groups, "cells", cam.cells, flush=True)
    lib = N.load()
    G = fr.groups
    pair_grads = torch.full((fr.T * G, 10), -7.0, dtype=torch.float32, device=dev)
    slot_live = fr.slot_live
    g = torch.Generator().manual_seed(1)
    gi = (torch.rand((3, H, W), generator=g) * 2 - 1).to(dev)
    ba = N.GsBlendBwdArgs(cam.to_struct(), cam.tiles_x, cam.tiles_y, N.ptr(fr.ranges), N.ptr(fr.sorted_gauss),
                          N.ptr(fr.records), N.ptr(image), N.ptr(alpha), N.ptr(depth), N.ptr(fr.pix_flags),
                          N.ptr(fr.cell_neval), N.ptr(gi), 0, 0,
                          N.ptr(fr.live_bits), fr.live_bits.shape[1], N.ptr(pair_grads), N.ptr(slot_live), fr.T, 0, 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    import ctypes as C
    N.check(lib.gs_blend_backward(C.byref(ba), N.stream_ptr()), "bwd")
    e1.record()
    torch.cuda.synchronize()
    print("blend bwd ms", e0.elapsed_time(e1), flush=True)
    pg = pair_grads.cpu().numpy()
    fl = slot_live.cpu().numpy()
    nan = np.isnan(pg).any(axis=1)
    print("flagged slots", int(fl.sum()), "nan slots", int(nan.sum()), "untouched flagged",
          int(((pg[:, 0] == -7.0) & (fl > 0)).sum()), flush=True)
    if nan.any():
        # map slots back to (tile, position)
        ranges = fr.ranges.cpu().numpy()
        sg = fr.sorted_gauss.cpu().numpy()
        rec = fr.records.cpu().numpy().view(np.uint32)
        off = rec[:, 10]
        info = rec[:, 11]
        bad = set(np.nonzero(nan)[0].tolist())
        shown = 0
        for t in range(ranges.shape[0]):
            s0, s1 = ranges[t]
            ty, tx = divmod(t, cam.tiles_x)
            for p in range(s0, s1):
                gid = sg[p]
                slot = off[gid] + (ty - ((info[gid] >> 12) & 0xFFF)) * ((info[gid] >> 24) + 1) + (tx - (info[gid] & 0xFFF))
                if slot in bad and shown < 30:
                    print("nan: tile", t, "pos", p - s0, "of", s1 - s0, "gid", gid, flush=True)
                    shown += 1


if __name__ == "__main__":
    main()
