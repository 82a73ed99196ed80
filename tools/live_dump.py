"""Render the C3 frame (forward only) and save the blend's per-(entry, cell)
liveness bitmap, the tile ranges and the per-pixel n_eval to an .npz, for
modelling backward schedules offline (tools/combine_model.py).  GPU tool.
    python tools/live_dump.py <out.npz> [--gaussians N --width W --height H]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from mini3dgs_amd import rasterizer as RZ
    from stubs import Cam
    dev = torch.device("cuda", 0)
    W, H = a.width, a.height
    sc = pkg.synthetic.make_scene(a.gaussians, W, H, seed=0)
    m = pkg.synthetic.to_model(sc, pkg.GaussianModel, dev)
    camp = pkg.camera_params(Cam(W, H, sc.fovx, sc.fovy), pkg.RenderSettings(H, W, torch.zeros(3)))
    pc = torch.empty((H * W,), dtype=torch.int32, device=dev)
    pn = torch.empty_like(pc)
    with torch.no_grad():
        for _ in range(2):  # (the second frame takes the depth-key window path, as the bench's)
            image, alpha, depth, *_, fr = RZ.forward_pipeline(
                camp, m._xyz, None, m._scaling, m._rotation, m._features_dc[:, 0, :],
                torch.sigmoid(m._opacity).squeeze(1), pair_counts=pc, need_grad=True, pix_neval=pn)
    torch.cuda.synchronize()
    np.savez_compressed(a.out, live_bits=fr.live_bits.cpu().numpy(), ranges=fr.ranges.cpu().numpy(),
                        neval=pn.cpu().numpy(),
                        contrib=pc.cpu().numpy(), W=W, H=H, T=fr.T, M=fr.M)
    print("saved", a.out, "T", fr.T, "live words", fr.live_bits.shape)


if __name__ == "__main__":
    main()
