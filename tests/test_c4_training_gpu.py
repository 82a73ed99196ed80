"""Config C4 on the GPU, as a test (round-3 review item 4): the full
GaussianTrainer loop (render -> fused L1 + D-SSIM -> backward -> FusedAdam ->
densify / prune) for 7,000 iterations at 800x800 on 100 views, from a random
init of 100k Gaussians.

The NeRF-synthetic lego scene BASELINE.json names is not in the container (no
network) and the reference's trainer and dataset are stubs
(/root/reference/src/train/trainer.py:32-89, src/data/dataset.py:30-61), so
C4 is PARITY UNPINNED: there is no reference PSNR to match.  The scene is
tools/train_synthetic.py's stand-in: a Blender-format dataset whose images
are rendered from a known set of 200k Gaussians.  Asserted: the held-out
views' PSNR clears a floor (round 3 measured 37.3 dB), density control ran,
and the depth-key window stopped missing after the first frames (a miss
re-renders a frame).  Prints iterations/s."""
import json
import os
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

PSNR_FLOOR = 33.0
WARM_FRAMES = 200  # frames (train + validation renders) before which a window miss is allowed


def test_c4_synthetic_training_7k(pkg, cuda):
    import train_synthetic as ts
    ds = ts.build_scene(pkg, views=100, size=800, gt_gaussians=200_000, device=cuda)
    tr = ts.make_trainer(pkg, ds, iters=7000)
    RZ = pkg.rasterizer
    RZ._WINDOW_STATE.pop(cuda, None)
    RZ._DEPTH_HIST.pop(cuda, None)
    p0 = tr.validate()["psnr"]
    n0 = tr.gaussians.get_num_points()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ws = RZ.depth_window_stats(cuda)
    v = tr.validate()
    line = {"workload": "C4 stand-in (parity unpinned): 100 views 800x800, GT 200k Gaussians, random init 100k",
            "iterations": 7000, "it_per_s": round(7000 / dt, 1), "train_s": round(dt, 2), "psnr_init": round(p0, 2),
            "psnr_test": round(v["psnr"], 2), "gaussians": v["num_gaussians"], "window": ws}
    print(json.dumps(line))
    assert v["psnr"] >= PSNR_FLOOR, line
    assert v["psnr"] > p0 + 10.0
    assert v["num_gaussians"] != n0  # density control ran
    assert ws["frame"] >= 7000
    assert ws["last_miss"] is None or ws["last_miss"] < WARM_FRAMES, line
