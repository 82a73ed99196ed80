"""Gradient-parity diagnostics (not product code): for a scene checked against
the oracle, list the Gaussians with the largest gradient differences with
their 2D conic condition number, screen radius, depth and whether their
footprint covers a knife-edge pixel (any margin) or a flipped one.
usage: python tools/grad_diag.py c3|odd1x33|c2"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_io as G  # noqa: E402
from stubs import Cam  # noqa: E402


def main(which):
    import __graft_entry__ as ge
    pkg = ge.load_package()
    cuda = torch.device("cuda", 0)
    syn = pkg.synthetic
    if which == "c3":
        W, H, bg, seed = 1920, 1080, (0.0, 0.0, 0.0), 1
        sc = syn.make_scene(1_000_000, W, H, seed=0)
    elif which == "odd1x33":
        W, H, bg, seed = 1, 33, (0.2, 0.1, 0.0), 1
        sc = syn.make_scene(400, W, H, seed=40 + W + H, sigma_range=(0.01, 0.2))
    else:
        W, H, bg, seed = 800, 800, (0.2, 0.3, 0.4), 3
        sc = syn.make_scene(100_000, W, H, seed=2)
    m = syn.to_model(sc, pkg.GaussianModel, cuda)
    out = pkg.GaussianRenderer().render(Cam(W, H, sc.fovx, sc.fovy), m, pkg.RenderSettings(H, W, torch.tensor(bg)))
    rng = np.random.default_rng(seed)
    gi, ga, gd = (rng.uniform(-1, 1, s).astype(np.float32) for s in ((3, H, W), (1, H, W), (1, H, W)))
    L = sum((out[k] * torch.tensor(v, device=cuda)).sum() for k, v in (("image", gi), ("alpha", ga), ("depth", gd)))
    L.backward()
    o = G.oracle()
    cov = o.covariance(sc.scaling.numpy(), sc.rotation.numpy())
    osc = o.Scene(xyz=sc.xyz.numpy(), cov3d=cov, color_logits=sc.features_dc[:, 0].numpy(),
                  opacity=torch.sigmoid(sc.opacity[:, 0]).numpy(), wv=np.eye(4), width=W, height=H,
                  fovx=sc.fovx, fovy=sc.fovy, bg=np.asarray(bg, np.float32))
    ref = o.render_backward(osc, gi, ga, gd, nthreads=16, margins=True)
    ds, dr = o.covariance_backward(sc.scaling.numpy(), sc.rotation.numpy(), ref["grads"]["cov3d"])
    edge = G.knife_edge(ref["margin"])
    img = out["image"].detach().cpu().numpy()
    alpha = out["alpha"].detach().cpu().numpy()
    flipped = edge & ((np.abs(img - ref["image"]).max(0) > 1e-5) | (np.abs(alpha - ref["alpha"])[0] > 1e-6))
    means = out["viewspace_points"].detach().cpu().numpy()
    con = out["conics"].detach().cpu().numpy().reshape(-1, 4).astype(np.float64)
    vis = out["visibility_filter"].cpu().numpy()
    t_edge = G.touching_gaussians(means, con, vis, list(zip(*np.nonzero(edge)))) if edge.sum() < 20000 else None
    t_flip = G.touching_gaussians(means, con, vis, list(zip(*np.nonzero(flipped))))
    hm, hd = 0.5 * (con[:, 0] + con[:, 3]), np.sqrt((0.5 * (con[:, 0] - con[:, 3])) ** 2 + con[:, 1] * con[:, 2])
    cond = (hm + hd) / np.maximum(hm - hd, 1e-30)
    radii = out["radii"].detach().cpu().numpy()
    print(f"{which}: knife-edge px {int(edge.sum())}, flipped px {int(flipped.sum())}, "
          f"Gaussians touching flipped {int(t_flip.sum())}")
    for name, d, r in (("scaling", m._scaling.grad.cpu().numpy(), ds), ("rotation", m._rotation.grad.cpu().numpy(), dr),
                       ("xyz", m._xyz.grad.cpu().numpy(), ref["grads"]["xyz"])):
        scale = np.abs(r).max()
        e = np.abs(d - r).max(1) / scale
        order = np.argsort(-e)[:8]
        print(f"  {name}: scale {scale:.3g}; max rel err {e.max():.3g}; off flipped {e[~t_flip].max():.3g}; "
              f"off flipped and cond<1e3 {e[~t_flip & (cond < 1e3)].max():.3g}")
        for i in order:
            print(f"    g {i}: err {e[i]:.3g} |ref| {np.abs(r[i]).max() / scale:.3g} cond {cond[i]:.3g} radius {radii[i]:.3g} "
                  f"z {sc.xyz[i, 2].item():.3g} flip {bool(t_flip[i])} edge {None if t_edge is None else bool(t_edge[i])}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "c3")
