"""Cell-shape study (not product code): how many (entry, cell) visits the
blend makes at C3 with 8x8 cells versus 8x16 "tall" cells (two pixels per
lane), from the projected means / conics / radii of one render and the
cell_hit box test of gsplat_mi355x.hip.  usage: python tools/cell_shape_stats.py"""
import importlib
import math
import sys

import torch

sys.path.insert(0, ".")
pkg = importlib.import_module("mini-3d-gaussian-splatting_amd")
syn = pkg.synthetic
from tests.stubs import Cam  # noqa: E402

W, H, TILE = 1920, 1080, 16
sc = syn.make_scene(1_000_000, W, H, seed=0)
dev = "cuda"
m = syn.to_model(sc, pkg.GaussianModel, dev)
with torch.no_grad():
    out = pkg.GaussianRenderer().render(Cam(W, H, sc.fovx, sc.fovy), m, pkg.RenderSettings(H, W, torch.zeros(3)))
mu = out["viewspace_points"].detach()
con = out["conics"].detach().reshape(-1, 4)
r = out["radii"].detach()
vis = out["visibility_filter"]
mu, con, r = mu[vis], con[vis], r[vis]
q00, q01, q11 = con[:, 0], con[:, 1], con[:, 3]
det = q00 * q11 - q01 * q01
L = 23.1 * 1.01
hx = torch.sqrt(L * q11 / det)
hy = torch.sqrt(L * q00 / det)
tx0 = torch.clamp(torch.floor((mu[:, 0] - r) / TILE), 0, (W + TILE - 1) // TILE - 1)
tx1 = torch.clamp(torch.floor((mu[:, 0] + r) / TILE), 0, (W + TILE - 1) // TILE - 1)
ty0 = torch.clamp(torch.floor((mu[:, 1] - r) / TILE), 0, (H + TILE - 1) // TILE - 1)
ty1 = torch.clamp(torch.floor((mu[:, 1] + r) / TILE), 0, (H + TILE - 1) // TILE - 1)


def count(lo_px, hi_px, c, h, size):
    """# of `size`-px bands inside [lo_px, hi_px) whose pixel centres [b, b + size - 1] meet [c - h, c + h]"""
    first = torch.maximum(lo_px, torch.ceil((c - h - (size - 1)) / size) * size)
    last = torch.minimum(hi_px - size, torch.floor((c + h) / size) * size)
    return torch.clamp((last - first) / size + 1, min=0)


x_lo, x_hi = tx0 * TILE, (tx1 + 1) * TILE
y_lo, y_hi = ty0 * TILE, (ty1 + 1) * TILE
c8 = count(x_lo, x_hi, mu[:, 0], hx, 8)
r8 = count(y_lo, y_hi, mu[:, 1], hy, 8)
r16 = count(y_lo, y_hi, mu[:, 1], hy, 16)
c16 = count(x_lo, x_hi, mu[:, 0], hx, 16)
T = ((tx1 - tx0 + 1) * (ty1 - ty0 + 1)).sum().item()
v8 = (c8 * r8).sum().item()
vt = (c8 * r16).sum().item()
v16 = (c16 * r16).sum().item()
print(f"visible {int(vis.sum())}  T {T:.4g}  (entry, cell) pairs 8x8: {4 * T:.4g}")
print(f"visits 8x8 cells: {v8:.4g} ({v8 / (4 * T):.3f} of pairs)")
print(f"visits 8x16 tall cells: {vt:.4g} ({vt / (2 * T):.3f} of pairs); lane-pixel slots {128 * vt:.4g} vs {64 * v8:.4g}")
print(f"visits 16x16 (whole tile per wave, 4 px/lane): {v16:.4g}; lane-pixel slots {256 * v16:.4g}")
