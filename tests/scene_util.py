"""A NeRF-synthetic-format training scene whose ground-truth images are
rendered from a known Gaussian set (no dataset is available offline;
BASELINE config C4 names the lego scene).  Shared by the GPU training tests
and the data-parallel worker (tests/dp_worker.py)."""
import json
import math

import numpy as np
import torch

from test_training_cpu import _png, look_at_c2w_gl


def write_scene_files(root, n_views=12, size=64):
    """transforms_train.json + blank RGBA frames (the images are replaced by
    renders of the ground-truth set in load_scene)."""
    (root / "train").mkdir(parents=True, exist_ok=True)
    frames = []
    rng = np.random.default_rng(0)
    for i in range(n_views):
        th, ph = 2 * math.pi * i / n_views, 0.3 + 0.4 * rng.random()
        C = 4.0 * np.array([math.cos(th) * math.cos(ph), math.sin(th) * math.cos(ph), math.sin(ph)])
        _png(root / "train" / f"r_{i}.png", size, size, np.zeros((size, size, 4), np.uint8))
        frames.append({"file_path": f"./train/r_{i}", "transform_matrix": look_at_c2w_gl(C).tolist()})
    (root / "transforms_train.json").write_text(json.dumps({"camera_angle_x": 0.69, "frames": frames}))


def load_scene(pkg, root, cuda, size=64, split=True):
    ds = pkg.NeRFSyntheticDataset(str(root), device=cuda)
    ds.load_cameras()
    # ground truth: 1500 Gaussians in a ball of radius 0.7
    g = torch.Generator().manual_seed(3)
    n = 1500
    d = torch.randn(n, 3, generator=g)
    xyz = d / d.norm(dim=1, keepdim=True) * 0.7 * torch.rand(n, 1, generator=g) ** (1 / 3)
    gt = pkg.GaussianModel()
    gt._set(xyz.to(cuda), (torch.rand(n, 1, 3, generator=g) * 4 - 2).to(cuda), torch.zeros(n, 15, 3, device=cuda),
            torch.log(0.03 + 0.05 * torch.rand(n, 3, generator=g)).to(cuda),
            torch.nn.functional.normalize(torch.randn(n, 4, generator=g), dim=-1).to(cuda),
            torch.full((n, 1), 1.5).to(cuda))
    r = pkg.GaussianRenderer()
    with torch.no_grad():
        for cam in ds.get_train_cameras():
            cam._image = r.render(cam, gt, pkg.RenderSettings(size, size, torch.zeros(3)))["image"].clone()
    if split:
        ds.split_train_test(0.25)
    return ds


def dp_config(pkg, out):
    """Three iterations with one densification (iteration 2)."""
    return pkg.TrainingConfig(iterations=3, densify_from_iter=2, densify_until_iter=2, densify_interval=2,
                              densify_grad_threshold=2e-5, num_random_points=3000, log_interval=1,
                              output_path=str(out), position_lr_init=1.6e-3, position_lr_final=1.6e-5)
