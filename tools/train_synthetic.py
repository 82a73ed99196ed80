"""Config C4 stand-in (the NeRF-synthetic lego scene is not available
offline): a Blender-format scene whose ground truth is rendered from a known
Gaussian set at 800x800, then the full GaussianTrainer loop from a random
init.  Prints one JSON line: iterations/s, test PSNR, Gaussian count.
    python tools/train_synthetic.py [--iters 7000] [--views 100] [--size 800]"""
import argparse
import json
import math
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def build_scene(pkg, views=100, size=800, gt_gaussians=200_000, device=None):
    """The C4 stand-in dataset: `views` cameras on a sphere of radius 4 around
    a ball of `gt_gaussians` random Gaussians, each image rendered from them
    at size x size (NeRF-synthetic layout, composited on black).  Returns the
    loaded NeRFSyntheticDataset with 1/8 of the views held out as test views."""
    from test_training_cpu import look_at_c2w_gl, _png
    dev = device if device is not None else torch.device("cuda", 0)
    tmp = tempfile.mkdtemp()
    os.makedirs(os.path.join(tmp, "train"))
    frames, rng = [], np.random.default_rng(0)
    for i in range(views):
        th, ph = 2 * math.pi * rng.random(), math.asin(2 * rng.random() - 1) * 0.8
        C = 4.0 * np.array([math.cos(th) * math.cos(ph), math.sin(th) * math.cos(ph), math.sin(ph)])
        frames.append({"file_path": f"./train/r_{i}", "transform_matrix": look_at_c2w_gl(C).tolist()})
    _png(os.path.join(tmp, "train", "blank.png"), 4, 4, np.zeros((4, 4, 4), np.uint8))
    for f in frames:
        os.link(os.path.join(tmp, "train", "blank.png"), os.path.join(tmp, f["file_path"][2:] + ".png"))
    with open(os.path.join(tmp, "transforms_train.json"), "w") as fh:
        json.dump({"camera_angle_x": 0.6911, "frames": frames}, fh)
    ds = pkg.NeRFSyntheticDataset(tmp, device=dev)
    ds.load_cameras()
    g = torch.Generator().manual_seed(3)
    n = gt_gaussians
    d = torch.randn(n, 3, generator=g)
    xyz = d / d.norm(dim=1, keepdim=True) * torch.rand(n, 1, generator=g) ** (1 / 3)
    gt = pkg.GaussianModel()
    gt._set(xyz.to(dev), (torch.rand(n, 1, 3, generator=g) * 4 - 2).to(dev), torch.zeros(n, 15, 3, device=dev),
            torch.log(0.005 + 0.02 * torch.rand(n, 3, generator=g)).to(dev),
            torch.nn.functional.normalize(torch.randn(n, 4, generator=g), dim=-1).to(dev), torch.full((n, 1), 1.0).to(dev))
    r = pkg.GaussianRenderer()
    with torch.no_grad():
        for cam in ds.cameras:
            cam._width = cam._height = size
            cam._FoVy = cam._FoVx
            cam._image = r.render(cam, gt, pkg.RenderSettings(size, size, torch.zeros(3)))["image"].clone()
    ds.split_train_test(0.125)
    ds.root = tmp
    return ds


def make_trainer(pkg, ds, iters=7000):
    cfg = pkg.TrainingConfig(iterations=iters, num_random_points=100_000, log_interval=500,
                             densify_until_iter=min(15000, iters // 2), output_path=os.path.join(ds.root, "out"))
    tr = pkg.GaussianTrainer(cfg, ds)
    tr.setup()
    return tr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=7000)
    ap.add_argument("--views", type=int, default=100)
    ap.add_argument("--size", type=int, default=800)
    ap.add_argument("--gt-gaussians", type=int, default=200_000)
    ap.add_argument("--profile-iters", type=int, default=0,
                    help="host profile (cProfile) of this many iterations after 100 warm ones, then exit")
    a = ap.parse_args()
    import __graft_entry__ as ge
    pkg = ge.load_package()
    ds = build_scene(pkg, a.views, a.size, a.gt_gaussians)
    n = a.gt_gaussians
    tr = make_trainer(pkg, ds, a.iters)
    if a.profile_iters:
        import cProfile
        import pstats
        tr.train(100)
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        tr.train(a.profile_iters)
        torch.cuda.synchronize()
        pr.disable()
        dt = time.perf_counter() - t0
        print(f"{a.profile_iters} iterations: {1e3 * dt / a.profile_iters:.3f} ms each (with the profiler)")
        pstats.Stats(pr).sort_stats("tottime").print_stats(30)
        return
    p0 = tr.validate()["psnr"]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    v = tr.validate()
    print(json.dumps({"workload": f"C4 stand-in: synthetic Blender-format scene, {a.views} views {a.size}x{a.size}, "
                                  f"GT {n} Gaussians, random init 100k", "iterations": a.iters,
                      "it_per_s": round(a.iters / dt, 1), "train_s": round(dt, 2), "psnr_init": round(p0, 2),
                      "psnr_test": round(v["psnr"], 2), "gaussians": v["num_gaussians"],
                      "losses": [round(x, 4) for x in tr.train_losses]}), flush=True)


if __name__ == "__main__":
    main()
