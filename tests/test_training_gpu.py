"""End-to-end training on the GPU: a NeRF-synthetic-format scene whose
ground-truth images are rendered from a known Gaussian set (no dataset is
available offline; BASELINE config C4 names the lego scene), then
GaussianTrainer (render -> fused L1+D-SSIM -> backward -> FusedAdam ->
densify) from a random init.  Checks the PSNR rises and checkpoints
round-trip."""
import json
import math

import numpy as np
import pytest
import torch

from test_training_cpu import look_at_c2w_gl, _png

pytestmark = pytest.mark.gpu


def _scene(pkg, tmp_path, cuda, n_views=12, size=64):
    (tmp_path / "train").mkdir()
    frames = []
    rng = np.random.default_rng(0)
    for i in range(n_views):
        th, ph = 2 * math.pi * i / n_views, 0.3 + 0.4 * rng.random()
        C = 4.0 * np.array([math.cos(th) * math.cos(ph), math.sin(th) * math.cos(ph), math.sin(ph)])
        _png(tmp_path / "train" / f"r_{i}.png", size, size, np.zeros((size, size, 4), np.uint8))
        frames.append({"file_path": f"./train/r_{i}", "transform_matrix": look_at_c2w_gl(C).tolist()})
    (tmp_path / "transforms_train.json").write_text(json.dumps({"camera_angle_x": 0.69, "frames": frames}))
    ds = pkg.NeRFSyntheticDataset(str(tmp_path), device=cuda)
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
    ds.split_train_test(0.25)
    return ds


def test_trainer_learns_and_checkpoints(pkg, cuda, tmp_path):
    ds = _scene(pkg, tmp_path, cuda)
    cfg = pkg.TrainingConfig(iterations=600, densify_from_iter=100, densify_until_iter=400, densify_interval=100,
                             num_random_points=4000, log_interval=100, output_path=str(tmp_path / "out"),
                             position_lr_init=1.6e-3, position_lr_final=1.6e-5)
    tr = pkg.GaussianTrainer(cfg, ds)
    tr.setup()
    before = tr.validate()
    n0 = tr.gaussians.get_num_points()
    tr.train()
    after = tr.validate()
    print(f"PSNR {before['psnr']:.2f} -> {after['psnr']:.2f} dB; Gaussians {n0} -> {after['num_gaussians']}")
    assert after["psnr"] > before["psnr"] + 5.0
    assert after["num_gaussians"] != n0  # density control ran
    assert len(tr.train_losses) == 6 and tr.train_losses[-1] < tr.train_losses[0]
    path = tr.save_checkpoint(tr.iteration)
    tr2 = pkg.GaussianTrainer(cfg, ds)
    tr2.load_checkpoint(tr.iteration)
    for a, b in zip(tr.gaussians.parameter_list(), tr2.gaussians.parameter_list()):
        assert torch.equal(a.detach(), b.detach())
    assert tr2.iteration == tr.iteration and path.endswith(".safetensors")
    assert math.isclose(tr2.validate()["psnr"], after["psnr"], rel_tol=1e-6)
    # resuming trains on: the run state (cameras, scene extent) is rebuilt by
    # load_checkpoint, and the resumed run takes the same steps as the original
    assert tr2.scene_extent == tr.scene_extent and tr2._perm is not None
    tr.train(5)
    tr2.train(5)
    assert tr2.iteration == tr.iteration
    for a, b in zip(tr.gaussians.parameter_list(), tr2.gaussians.parameter_list()):
        assert torch.equal(a.detach(), b.detach())
