"""Bitwise-repeat check of the render backward at several tile sizes,
localising a difference to the blend backward's partials, the gather's sums
or the projection backward (GPU debug tool).
    python tools/det_debug.py [tile ...]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from stubs import Cam
    RZ = pkg.rasterizer
    syn = pkg.synthetic
    dev = torch.device("cuda", 0)
    tiles = [int(t) for t in sys.argv[1:]] or [16, 32, 64, 300]
    for tile in tiles:
        sc = syn.make_scene(8000, 480, 270, seed=5, sigma_range=(0.002, 0.02))
        runs = []
        for rep in range(3):
            m = syn.to_model(sc, pkg.GaussianModel, dev)
            out = pkg.GaussianRenderer(tile_size=tile).render(Cam(480, 270, sc.fovx, sc.fovy), m,
                                                              pkg.RenderSettings(270, 480, torch.zeros(3)))
            fr_holder = {}
            bp = RZ.backward_pipeline

            def hook(cam, fr, *a, **k):
                r = bp(cam, fr, *a, **k)
                torch.cuda.synchronize()
                fr_holder["fr"] = fr
                return r
            RZ.backward_pipeline = hook
            try:
                (out["image"].sum() + out["depth"].mean()).backward()
            finally:
                RZ.backward_pipeline = bp
            torch.cuda.synchronize()
            fr = fr_holder["fr"]
            runs.append(dict(xyz=m._xyz.grad.clone(), op=m._opacity.grad.clone(),
                             pix=fr.pix_flags.int(), T=fr.T, groups=fr.groups))
        for k in ("xyz", "op", "pix"):
            same = [torch.equal(runs[0][k], r[k]) for r in runs[1:]]
            diff = [float((runs[0][k] - r[k]).abs().max()) for r in runs[1:]]
            nd = [int((runs[0][k] != r[k]).sum()) for r in runs[1:]]
            print(f"tile {tile} T {runs[0]['T']} groups {runs[0]['groups']} {k}: equal {same} maxdiff {diff} ndiff {nd}",
                  flush=True)


if __name__ == "__main__":
    main()
