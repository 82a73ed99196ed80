"""Render the C3 frame (forward only) and save image/alpha/neval/ranges to an .npz (debug tool)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(out):
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from mini3dgs_amd import rasterizer as RZ
    from stubs import Cam
    dev = torch.device("cuda", 0)
    W, H = 1920, 1080
    sc = pkg.synthetic.make_scene(1_000_000, W, H, seed=0)
    m = pkg.synthetic.to_model(sc, pkg.GaussianModel, dev)
    camp = pkg.camera_params(Cam(W, H, sc.fovx, sc.fovy), pkg.RenderSettings(H, W, torch.zeros(3)))
    with torch.no_grad():
        pn = torch.empty((camp.image_width * camp.image_height,), dtype=torch.int32, device=m._xyz.device)
        image, alpha, depth, *_, fr = RZ.forward_pipeline(camp, m._xyz, None, m._scaling, m._rotation,
                                                          m._features_dc[:, 0, :], torch.sigmoid(m._opacity).squeeze(1),
                                                          pix_neval=pn)
    np.savez(out, image=image.cpu().numpy(), alpha=alpha.cpu().numpy(),
             neval=pn.cpu().numpy(), ranges=fr.ranges.cpu().numpy())


if __name__ == "__main__":
    main(sys.argv[1])
