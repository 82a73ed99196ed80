"""Host-side logic of the drop-in API (no GPU needed)."""
import math

import numpy as np
import pytest
import torch


class _Cam:
    _width, _height, _FoVx, _FoVy = 48, 32, math.radians(70), math.radians(50)

    def world_view_transform(self):
        m = torch.eye(4)
        m[:3, 3] = torch.tensor([0.1, 0.2, 0.3])
        return m


def test_camera_params_follow_reference_intrinsics(pkg):
    """renderer.py:140-152: fx = 0.5 W / tan(FoVx/2) from the CAMERA size,
    image size from the SETTINGS."""
    st = pkg.RenderSettings(image_height=20, image_width=30, bg_color=torch.tensor([0.1, 0.2, 0.3]))
    c = pkg.camera_params(_Cam(), st)
    assert (c.image_width, c.image_height) == (30, 20)
    assert c.fx == pytest.approx(0.5 * 48 / math.tan(math.radians(35)))
    assert c.fy == pytest.approx(0.5 * 32 / math.tan(math.radians(25)))
    assert (c.cx, c.cy) == (24.0, 16.0)
    assert c.view[3] == pytest.approx(0.1) and c.view[7] == pytest.approx(0.2) and c.view[11] == pytest.approx(0.3)
    assert c.tiles_x == 2 and c.tiles_y == 2
    assert c.bg == pytest.approx((0.1, 0.2, 0.3))


def test_world_view_as_tensor_attribute(pkg):
    class Cam2(_Cam):
        pass
    cam = Cam2()
    cam.world_view_transform = torch.eye(4)
    c = pkg.camera_params(cam, pkg.RenderSettings(8, 8, torch.zeros(3)))
    assert c.view == tuple([1.0, 0, 0, 0, 0, 1.0, 0, 0, 0, 0, 1.0, 0])


def test_no_cpu_fallback(pkg):
    """The product path must fail loudly without a HIP device tensor."""
    m = pkg.GaussianModel()
    m.create_from_random(10)
    with pytest.raises(RuntimeError, match="HIP device"):
        pkg.GaussianRenderer().render(_Cam(), m, pkg.RenderSettings(8, 8, torch.zeros(3)))


def test_renderer_constructor_range(pkg):
    """GaussianRenderer(tile_size, radius_min, radius_max) (renderer.py:24-28):
    any tile edge >= 1 (the reference takes any int; 0 divides by zero there)
    and finite radii are taken as given.  The kernels' edge is the tile_size,
    or max(W, H) when it is larger (one tile holds the image either way:
    effective_tile); tiles of many cells replay them in batches within a
    memory budget (rasterizer.cell_batch)."""
    for t in (1, 8, 12, 16, 32, 256, 257, 1000, 10 ** 6):
        r = pkg.GaussianRenderer(tile_size=t, radius_max=80.0)
        assert r.tile_size == t and r.radius_max == 80.0
    c = pkg.camera_params(_Cam(), pkg.RenderSettings(20, 30, torch.zeros(3)), tile_size=8)
    assert (c.tiles_x, c.tiles_y, c.cells) == (4, 3, 1)
    assert pkg.camera_params(_Cam(), pkg.RenderSettings(20, 30, torch.zeros(3)), tile_size=32).cells == 16
    # a tile above the image: one tile of max(W, H) = 30 px
    for t in (31, 1000, 10 ** 9):
        c = pkg.camera_params(_Cam(), pkg.RenderSettings(20, 30, torch.zeros(3)), tile_size=t)
        assert (c.tile_size, c.tiles_x, c.tiles_y) == (30, 1, 1)
    big = pkg.RenderSettings(4000, 4000, torch.zeros(3))
    assert pkg.camera_params(_Cam(), big, tile_size=300).groups == 1444  # one partial per 8x8 cell
    assert pkg.camera_params(_Cam(), big, tile_size=256).groups == 1024
    # tiles above 4096 px (round 6; ABI 21 stopped at 4096): a 5000-px image as
    # one tile, or in 2 x 2 tiles of 4500 px
    assert pkg._native.GS_MAX_TILE == 16384
    c = pkg.camera_params(_Cam(), pkg.RenderSettings(5000, 5000, torch.zeros(3)), tile_size=10 ** 6)
    assert (c.tile_size, c.tiles_x, c.tiles_y, c.cells) == (5000, 1, 1, 625 ** 2)
    c = pkg.camera_params(_Cam(), pkg.RenderSettings(5000, 5000, torch.zeros(3)), tile_size=4500)
    assert (c.tile_size, c.tiles_x, c.tiles_y) == (4500, 2, 2)
    # an image wider than GS_MAX_TILE cannot be one tile: a tile edge that would
    # cover it raises, where the reference renders it as one tile
    with pytest.raises(ValueError):
        pkg.camera_params(_Cam(), pkg.RenderSettings(100, 40000, torch.zeros(3)), tile_size=10 ** 6)
    with pytest.raises(ValueError):  # a 70000-px image in tiles above 16384 px that do not cover it
        pkg.camera_params(_Cam(), pkg.RenderSettings(100, 70000, torch.zeros(3)), tile_size=35000)
    for bad in (dict(tile_size=0), dict(tile_size=-3), dict(tile_size=8.5), dict(radius_max=float("inf")),
                dict(radius_min=3.0, radius_max=2.0)):
        with pytest.raises(ValueError):
            pkg.GaussianRenderer(**bad)


def test_cell_batches_and_bitmap_budget(pkg):
    """Bounded memory at any tile size: the backward's partials
    [T, G] and the forward's liveness bitmap stay within their budgets; the
    default tile's four cells never batch (the performance path), whatever T."""
    RZ = pkg.rasterizer
    lib = pkg._native.load()
    B = RZ.PARTIAL_BUDGET_BYTES
    assert RZ.cell_batch(4, 10 ** 9) == 4
    assert RZ.cell_batch(16, 10 ** 5) == 16
    for cells, T in ((1444, 1_050_000), (57_600, 1_000_000), (262_144, 4_000_000), (1024, 50_000_000)):
        g = RZ.cell_batch(cells, T)
        assert 1 <= g <= cells and (g == 1 or 41 * T * g <= B)
    # ADVICE r04's case: 1080p, one 1920-px tile (57,600 cells), 1M entries: ~7 GB of bitmap -> none
    assert RZ.live_bitmap_bytes(lib, 57_600, 1_000_000, 1) == 0
    assert RZ.live_bitmap_bytes(lib, 4, 4_411_397, 8160) == 8 * 4 * (4_411_397 // 64 + 8160 + 2)
    small = RZ.live_bitmap_bytes(lib, 1444, 3000, 6)
    assert 0 < small <= RZ.LIVE_BUDGET_BYTES


def test_gaussian_model_layout(pkg):
    """test_gaussian_model.py:35-72 restated for this package's model."""
    m = pkg.GaussianModel()
    m.create_from_random(64, 1.0, generator=torch.Generator().manual_seed(0))
    assert m._xyz.shape == (64, 3) and m._features_dc.shape == (64, 1, 3)
    assert m._features_rest.shape == (64, 15, 3) and m._scaling.shape == (64, 3)
    assert m._rotation.shape == (64, 4) and m._opacity.shape == (64, 1)
    assert m.get_features.shape == (64, 16, 3)
    assert torch.all(m.get_scaling > 0)
    assert torch.allclose(m.get_rotation.norm(dim=-1), torch.ones(64), atol=1e-5)
    a = m.get_opacity
    assert torch.all(a > 0) and torch.all(a < 1)


def test_covariance_property_works(pkg):
    """Reference get_covariance is broken (gaussian_model.py:127); ours equals
    compute_3d_covariance and the oracle's restatement."""
    import golden_io as G
    m = pkg.GaussianModel()
    m.create_from_random(32, generator=torch.Generator().manual_seed(1))
    cov = m.get_covariance.detach().numpy()
    ref = G.oracle().covariance(m._scaling.detach().numpy(), m._rotation.detach().numpy())
    assert np.allclose(cov, ref, atol=1e-6, rtol=1e-5)


def test_camera_world_view_matches_reference_producer(pkg):
    """CameraUtils.build_world_view_matrix (camera.py:80-141): C2W -> W2C."""
    ang = 0.4
    R = np.array([[math.cos(ang), -math.sin(ang), 0], [math.sin(ang), math.cos(ang), 0], [0, 0, 1]], np.float32)
    C = np.array([1.0, -2.0, 0.5], np.float32)
    cam = pkg.Camera(0, R, C, 1.0, 1.0, None, "x", 16, 16)
    wv = cam.world_view_transform().numpy()
    assert np.allclose(wv[:3, :3], R.T, atol=1e-6)
    assert np.allclose(wv[:3, 3], -R.T @ C, atol=1e-6)
    assert np.allclose(cam.camera_center.numpy(), C, atol=1e-5)


def test_synthetic_scene_distribution(pkg):
    sc = pkg.synthetic.make_scene(5000, 192, 108, seed=0)
    z = sc.xyz[:, 2]
    assert z.min() >= 2 and z.max() <= 6
    s = sc.scaling.exp()
    assert s.min() >= 0.002 - 1e-6 and s.max() <= 0.01 + 1e-6
    assert torch.allclose(sc.rotation.norm(dim=1), torch.ones(5000), atol=1e-5)
    sc2 = pkg.synthetic.make_scene(5000, 192, 108, seed=0)
    assert torch.equal(sc.xyz, sc2.xyz)


def test_depth_window_choice(pkg):
    """rasterizer.depth_window: a window of key bits around the previous
    frame's visible fp32 depth bits, widened by 1/8 of the range each side;
    None when the range needs all 32 bits.  Visible keys stay below
    255 << (bits - 8): the MSD depth sort's top bucket is the culled sentinel's."""
    import struct
    RZ = pkg.rasterizer
    bits = lambda z: struct.unpack("<I", struct.pack("<f", z))[0]
    w = RZ.depth_window(bits(2.0), bits(6.0))  # the C3 distribution: 24 bits, 3 passes
    assert w is not None and w[1] <= 24
    assert RZ.window_holds(w, bits(2.0), bits(6.0)) and RZ.window_holds(w, bits(2.1), bits(5.5))
    assert not RZ.window_holds(w, bits(0.5), bits(6.0)) and not RZ.window_holds(w, bits(2.0), bits(60.0))
    w = RZ.depth_window(bits(0.01), bits(1000.0))  # 28 bits: no LSD pass saved, but the MSD sort's
    assert w is not None and 24 < w[1] < 32 and RZ.window_holds(w, bits(0.01), bits(1000.0))
    assert RZ.depth_window(bits(1e-38), bits(3e38)) is None  # all 32 bits
    assert RZ.depth_window(0xFFFFFFFF, 0) is None  # nothing visible
    assert RZ.window_holds(None, bits(0.01), bits(1e30))
    base, nb = RZ.depth_window(bits(3.0), bits(3.0))  # a single depth
    assert nb >= 1 and RZ.window_holds((base, nb), bits(3.0), bits(3.0))


def test_render_input_validation(pkg, monkeypatch):
    """Inputs the kernels would misread raise before any launch: wrong row
    counts or shapes, non-float dtypes, a missing covariance; other float
    dtypes are cast to fp32 (on the autograd tape)."""
    import sys
    R = sys.modules[pkg.__name__ + ".rasterizer"]
    monkeypatch.setattr(R, "_check_inputs", lambda x: None)  # (no HIP device here)
    n = 4

    def call(**kw):
        a = dict(xyz=torch.zeros(n, 3), cov3d=torch.zeros(n, 3, 3), scaling=None, rotation=None,
                 logits=torch.zeros(n, 3), opacity=torch.zeros(n))
        a.update(kw)
        R.rasterize(None, a["xyz"], a["cov3d"], a["scaling"], a["rotation"], a["logits"], a["opacity"])

    with pytest.raises(ValueError, match="opacity"):
        call(opacity=torch.zeros(n + 1))
    with pytest.raises(ValueError, match="cov3d"):
        call(cov3d=torch.zeros(n, 3))
    with pytest.raises(ValueError, match="xyz"):
        call(xyz=torch.zeros(n, 2))
    with pytest.raises(TypeError, match="colour"):
        call(logits=torch.zeros(n, 3, dtype=torch.int32))
    with pytest.raises(ValueError, match="covariance"):
        call(cov3d=None)
    with pytest.raises(ValueError, match="rotation"):
        call(cov3d=None, scaling=torch.zeros(n, 3), rotation=torch.zeros(n, 3))
    # fp64 passes validation (cast), then reaches the launch path (camera None here)
    with pytest.raises(AttributeError):
        call(logits=torch.zeros(n, 3, dtype=torch.float64))


def test_host_scalars_and_struct_caches(pkg):
    """camera_params reads the view and background as fp32 values from any
    tensor / sequence form; the ABI structs cached by value
    (CameraParams.to_struct, rasterizer._gaussians_struct) follow every
    change of what they hold."""
    import torch
    R, RZ = pkg.renderer, pkg.rasterizer
    wv = torch.arange(16, dtype=torch.float64).reshape(4, 4) / 7
    want = [float(v) for v in wv.float().reshape(-1)]
    assert R._host_f32(wv, 16) == want
    assert R._host_f32(wv.float(), 16) == want
    assert R._host_f32(wv.float().reshape(-1), 16) == want
    assert R._host_f32([0.1, 0.2, 0.3], 3) == [float(v) for v in torch.tensor([0.1, 0.2, 0.3])]
    with pytest.raises(ValueError):
        R._host_f32(torch.zeros(3, 3), 16)
    cp = RZ.CameraParams(64, 48, 50.0, 50.0, 32.0, 24.0, tuple(range(12)), (0.0, 0.5, 1.0))
    a = cp.to_struct()
    assert a is cp.to_struct() and (a.image_width, a.image_height, a.bg[1]) == (64, 48, 0.5)
    cp2 = RZ.CameraParams(64, 48, 50.0, 50.0, 32.0, 24.0, tuple(range(12)), (0.0, 0.25, 1.0))
    assert cp2.to_struct().bg[1] == 0.25 and a.bg[1] == 0.5
    xyz, sc, rot = torch.zeros(5, 3), torch.zeros(5, 3), torch.zeros(5, 4)
    col, op = torch.zeros(5, 1, 3), torch.zeros(5, 1)
    g = RZ._gaussians_struct(5, xyz, None, sc, rot, col, op, True)
    assert g is RZ._gaussians_struct(5, xyz, None, sc, rot, col, op, True)
    assert (g.xyz, g.color_logits, g.color_stride, g.opacity_is_logit) == (xyz.data_ptr(), col.data_ptr(), 3, 1)
    g2 = RZ._gaussians_struct(5, xyz, None, sc, rot, col, op, False)
    assert g2.opacity_is_logit == 0 and g.opacity_is_logit == 1
    xyz2 = torch.zeros(5, 3)
    assert RZ._gaussians_struct(5, xyz2, None, sc, rot, col, op, True).xyz == xyz2.data_ptr()


def test_fused_adam_runs_step_hooks(pkg):
    """torch.optim.Optimizer's step pre / post hooks (per optimizer
    and global) run around FusedAdam.step and step_ranges, in torch's order;
    a pre hook may rewrite the arguments.  (No gradients: nothing launches.)"""
    import torch
    from torch.optim.optimizer import register_optimizer_step_post_hook
    p = torch.nn.Parameter(torch.zeros(3))
    opt = pkg.optim.FusedAdam([p])
    calls = []
    h1 = opt.register_step_pre_hook(lambda o, a, k: calls.append(("pre", a)))
    h2 = opt.register_step_post_hook(lambda o, a, k: calls.append(("post", a)))
    h3 = register_optimizer_step_post_hook(lambda o, a, k: calls.append(("global_post", a)))
    try:
        assert opt.step() is None
        opt.step_ranges([(0, 3)])
    finally:
        h1.remove(), h2.remove(), h3.remove()
    assert [c[0] for c in calls] == ["pre", "post", "global_post"] * 2
    assert calls[0][1] == (None,) and calls[3][1] == ([(0, 3)], None)
    calls.clear()
    opt.step()
    assert calls == []
