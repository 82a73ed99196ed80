"""Dump the forward's saved per-pixel state (diagnostics)."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
import __graft_entry__ as ge
pkg = ge.load_package()
from mini3dgs_amd import rasterizer as RZ
W, H = 1920, 1080
sc = pkg.synthetic.make_scene(1_000_000, W, H, seed=0)
m = pkg.synthetic.to_model(sc, pkg.GaussianModel, torch.device('cuda'))
class Cam:
    _width, _height, _FoVx, _FoVy = W, H, sc.fovx, sc.fovy
    def world_view_transform(self): return torch.eye(4)
camp = pkg.camera_params(Cam(), pkg.RenderSettings(H, W, torch.zeros(3)))
pn = torch.empty((camp.image_width * camp.image_height,), dtype=torch.int32, device=m._xyz.device)
out = RZ.forward_pipeline(camp, m._xyz, None, m._scaling, m._rotation, m._features_dc[:, 0, :],
                          torch.sigmoid(m._opacity).squeeze(1), pix_neval=pn)
neval = pn.cpu().numpy()
np.savez_compressed(sys.argv[1], A=out[1].cpu().numpy().reshape(-1), neval=neval, img=out[0].cpu().numpy())
print(sys.argv[1], 'neval sum', neval.astype(np.int64).sum())
