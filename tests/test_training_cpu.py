"""Host-side training pieces on CPU: config, dataset loaders and their pose
conventions (renderer.py:150-162: +Z forward, Y up), LR schedule."""
import json
import math

import numpy as np
import pytest
import torch


def look_at_c2w_gl(C, target=(0.0, 0.0, 0.0), up=(0.0, 0.0, 1.0)):
    """Blender / OpenGL camera-to-world: columns right, up, back (camera looks down -Z)."""
    C, target, up = (np.asarray(v, np.float64) for v in (C, target, up))
    back = C - target
    back /= np.linalg.norm(back)
    right = np.cross(up, back)
    right /= np.linalg.norm(right)
    upv = np.cross(back, right)
    m = np.eye(4)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = right, upv, back, C
    return m


def _png(path, h, w, rgba):
    from PIL import Image
    Image.fromarray(rgba.astype(np.uint8), "RGBA").save(path)


def test_config_defaults_and_yaml(pkg, tmp_path):
    c = pkg.TrainingConfig()
    # config/config.py:33-67 defaults
    assert (c.iterations, c.position_lr_init, c.position_lr_final, c.feature_lr, c.opacity_lr, c.scaling_lr,
            c.rotation_lr, c.densify_from_iter, c.densify_until_iter, c.densify_grad_threshold,
            c.densify_interval) == (30000, 0.00016, 0.0000016, 0.0025, 0.05, 0.005, 0.001, 500, 15000, 0.0002, 100)
    c.iterations = 7000
    p = tmp_path / "c.yaml"
    pkg.ConfigManager.save(c, str(p))
    assert pkg.ConfigManager.load(str(p)) == c
    p.write_text("bogus_key: 1\n")
    with pytest.raises(KeyError):
        pkg.ConfigManager.load(str(p))


def test_nerf_synthetic_loader(pkg, tmp_path):
    frames = []
    (tmp_path / "train").mkdir()
    for i, C in enumerate([(0, -4, 0), (4, 0, 1)]):
        rgba = np.zeros((6, 8, 4), np.uint8)
        rgba[..., 0], rgba[..., 3] = 200, 128  # red at half alpha
        _png(tmp_path / "train" / f"r_{i}.png", 6, 8, rgba)
        frames.append({"file_path": f"./train/r_{i}", "transform_matrix": look_at_c2w_gl(C).tolist()})
    (tmp_path / "transforms_train.json").write_text(json.dumps({"camera_angle_x": 0.7, "frames": frames}))
    ds = pkg.NeRFSyntheticDataset(str(tmp_path))
    ds.load_cameras()
    cams = ds.get_train_cameras()
    assert len(cams) == 2 and ds.get_test_cameras() == []
    cam = cams[0]
    assert (cam._width, cam._height) == (8, 6)
    assert math.isclose(cam._FoVy, 2 * math.atan(math.tan(0.35) * 6 / 8), rel_tol=1e-9)
    img = cam._image
    assert img.shape == (3, 6, 8)
    assert abs(img[0, 0, 0].item() - 200 / 255 * 128 / 255) < 1e-6 and img[1].abs().max() == 0  # over black
    wv = cam.world_view_transform().double()
    origin_cam = wv[:3, :3] @ torch.zeros(3, dtype=torch.float64) + wv[:3, 3]
    assert origin_cam[2] > 3.9 and abs(origin_cam[0]) < 1e-5 and abs(origin_cam[1]) < 1e-5  # in front, centred
    above = wv[:3, :3] @ torch.tensor([0, 0, 1.0], dtype=torch.float64) + wv[:3, 3]
    assert above[1] > 0.5  # world up is camera +Y (renderer draws it at the top)
    info = ds.get_scene_info()
    assert info["num_train"] == 2 and info["radius"] > 0


def test_colmap_loader(pkg, tmp_path):
    sp = tmp_path / "sparse" / "0"
    sp.mkdir(parents=True)
    (tmp_path / "images").mkdir()
    (sp / "cameras.txt").write_text("# comment\n1 PINHOLE 8 6 10 11 4 3\n2 SIMPLE_PINHOLE 8 6 9 4 3\n")
    # identity rotation, camera at the origin looking down COLMAP +Z (Y down)
    (sp / "images.txt").write_text("# header\n1 1 0 0 0 0 0 0 1 a.png\n1 2 -1\n2 1 0 0 0 0 0 -2 2 b.png\n\n")
    (sp / "points3D.txt").write_text("1 0 -1 5 255 0 0 0.1 1 0\n2 1 1 5 0 255 0 0.1\n")
    for name in ("a.png", "b.png"):
        _png(tmp_path / "images" / name, 6, 8, np.full((6, 8, 4), 255, np.uint8))
    ds = pkg.COLMAPDataset(str(tmp_path), test_every=0)
    ds.load_cameras()
    assert len(ds.cameras) == 2 and len(ds.get_train_cameras()) == 2
    a = ds.cameras[0]
    assert math.isclose(a._FoVx, 2 * math.atan(8 / 20), rel_tol=1e-9)
    assert math.isclose(a._FoVy, 2 * math.atan(6 / 22), rel_tol=1e-9)
    wv = a.world_view_transform().double()
    p = wv[:3, :3] @ torch.tensor([0, -1.0, 5.0], dtype=torch.float64) + wv[:3, 3]  # COLMAP: above (Y down)
    assert p[2] > 4.9 and p[1] > 0.9  # ours: in front, Y up
    assert ds.points.shape == (2, 3) and np.allclose(ds.colors[0], [1, 0, 0])
    b = ds.cameras[1]
    assert np.allclose(b.camera_center.numpy(), [0, 0, 2])  # t = -R C with C = (0,0,2) (Y flip leaves z)


def test_lr_schedule(pkg):
    s = pkg.optim.LearningRateScheduler(1e-3, 1e-5, 0, 1.0, 100)
    assert math.isclose(s.get_lr(0), 1e-3) and math.isclose(s.get_lr(100), 1e-5) and math.isclose(s.get_lr(500), 1e-5)
    assert math.isclose(s.get_lr(50), 1e-5 + (1e-3 - 1e-5) * 0.5, rel_tol=1e-12)
    d = pkg.optim.LearningRateScheduler(1e-3, 1e-3, 10, 0.1, 100)
    assert math.isclose(d.get_lr(0), 1e-4) and math.isclose(d.get_lr(10), 1e-3)
    dc = pkg.optim.DensityController(pkg.TrainingConfig())
    assert dc.should_densify(500) and dc.should_densify(15000) and not dc.should_densify(550)
    assert not dc.should_densify(400) and not dc.should_densify(15100)


def test_reference_api_names(pkg, tmp_path):
    """Reference entry points kept under their names: ConfigManager
    load_from_yaml / save_to_yaml / get_default_config (config.py:69-95),
    GaussianModel.create_from_pcd (gaussian_model.py:42-76) over the point
    formats of IOUtils.load_point_cloud (io_utils.py:34-83), get_parameters."""
    import numpy as np
    cm = pkg.ConfigManager
    cfg = cm.get_default_config()
    cfg.iterations = 123
    cm.save_to_yaml(cfg, str(tmp_path / "sub" / "c.yaml"))
    assert cm.load_from_yaml(str(tmp_path / "sub" / "c.yaml")).iterations == 123
    pts = np.array([[0, 0, 0], [1, 2, 3], [-1, 0.5, 2]], np.float32)
    cols = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float32)
    np.savez(tmp_path / "p.npz", points=pts, colors=cols)
    np.save(tmp_path / "p.npy", np.concatenate([pts, cols], 1))
    (tmp_path / "p.txt").write_text("".join(" ".join(map(str, r)) + "\n" for r in pts))
    (tmp_path / "points3D.txt").write_text("# id x y z r g b err track\n" + "".join(
        f"{i} {p[0]} {p[1]} {p[2]} {int(c[0] * 255)} {int(c[1] * 255)} {int(c[2] * 255)} 0.1 1 2\n"
        for i, (p, c) in enumerate(zip(pts, cols))))
    for name, has_col in (("p.npz", True), ("p.npy", True), ("p.txt", False), ("points3D.txt", True)):
        m = pkg.GaussianModel()
        m.create_from_pcd(str(tmp_path / name), device="cpu")
        assert torch.allclose(m._xyz, torch.from_numpy(pts)), name
        want = torch.from_numpy(cols) if has_col else torch.ones(3, 3)
        assert torch.allclose(m._features_dc[:, 0], want), name
        assert len(m.get_parameters()) == 6
