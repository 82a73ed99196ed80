"""Bitwise comparison of two library builds on the C3 frame (GPU tool).

    GS_LIB_PATH=ab/base.so python tools/bitcmp.py dump gpurun_out/a.npz
    python tools/bitcmp.py dump gpurun_out/b.npz          # in-tree library
    python tools/bitcmp.py cmp gpurun_out/a.npz gpurun_out/b.npz

A refactor claimed bit-identical (same fp32 operations, reordered or
re-encoded) must show zero differing elements here: forward outputs and
every gradient of a fixed random cotangent."""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(path, n=1_000_000, W=1920, H=1080):
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    dev = torch.device("cuda", 0)
    scene = pkg.synthetic.make_scene(n, W, H, seed=0)
    m = pkg.synthetic.to_model(scene, pkg.GaussianModel, dev)

    class Cam:
        _width, _height, _FoVx, _FoVy = W, H, scene.fovx, scene.fovy

        def world_view_transform(self):
            return torch.eye(4)
    out = pkg.GaussianRenderer().render(Cam(), m, pkg.RenderSettings(H, W, torch.tensor([0.1, 0.2, 0.3])))
    g = torch.Generator().manual_seed(1)
    cot = [(torch.rand(s, generator=g) * 2 - 1).to(dev) for s in ((3, H, W), (1, H, W), (1, H, W))]
    torch.autograd.backward([out["image"], out["alpha"], out["depth"]], cot)
    res = {k: out[k].detach().cpu().numpy() for k in ("image", "alpha", "depth", "viewspace_points", "conics")}
    for k in ("_xyz", "_features_dc", "_scaling", "_rotation", "_opacity"):
        res["grad" + k] = getattr(m, k).grad.cpu().numpy()
    np.savez(path, **res)


def cmp(pa, pb):
    a, b = np.load(pa), np.load(pb)
    bad = 0
    for k in a.files:
        x, y = a[k], b[k]
        nd = int(np.sum(x.view(np.uint32) != y.view(np.uint32)))
        mx = float(np.nanmax(np.abs(x - y))) if x.size else 0.0
        print(f"{k:22s} differing {nd:9d} / {x.size:9d}  max|diff| {mx:.3e}")
        bad += nd
    print("BIT-IDENTICAL" if bad == 0 else f"DIFFERENT ({bad} elements)")


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
