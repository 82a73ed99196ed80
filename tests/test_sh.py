"""SH colour (behind RenderSettings.sh_degree / the model's
active_sh_degree): degree 0 is the reference's DC-only render bit for bit;
degrees 1..3 match a torch fp32 statement of the SH logits
(tests/sh_reference.py) composed with the already parity-checked DC path --
forward images and the gradients to features_rest, features_dc and xyz
(whose view-direction term goes through the SH)."""
import ctypes as C
import math

import pytest
import torch

from sh_reference import sh_basis, sh_logits


def _posed_view():
    a, b = 0.3, -0.2
    Ry = torch.tensor([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    Rx = torch.tensor([[1, 0, 0], [0, math.cos(b), -math.sin(b)], [0, math.sin(b), math.cos(b)]])
    wv = torch.eye(4)
    wv[:3, :3] = Rx @ Ry
    wv[:3, 3] = torch.tensor([0.3, -0.2, 0.5])
    return wv


def test_campos_is_camera_centre(pkg):
    from mini3dgs_amd.rasterizer import CameraParams
    wv = _posed_view()
    cam = CameraParams(64, 48, 50.0, 50.0, 32.0, 24.0, tuple(wv[:3, :].reshape(-1).tolist()), (0, 0, 0))
    c = torch.tensor(cam.campos)
    # the camera centre maps to the view-space origin
    assert torch.allclose(wv[:3, :3] @ c + wv[:3, 3], torch.zeros(3), atol=1e-6)


def test_sh_reference_degree0_and_basis_norm():
    g = torch.Generator().manual_seed(0)
    xyz, dc, rest = torch.randn(50, 3, generator=g), torch.randn(50, 3, generator=g), torch.randn(50, 15, 3, generator=g)
    assert torch.equal(sh_logits(xyz, dc, rest, torch.zeros(3), 0), dc)
    # real SH are orthonormal on the sphere: Monte-Carlo Gram matrix ~ I / (4 pi)
    d = torch.randn(200000, 3, generator=g, dtype=torch.float64)
    d = d / d.norm(dim=1, keepdim=True)
    Y = sh_basis(d)
    gram = (Y.T @ Y) / d.shape[0] * 4 * math.pi
    assert torch.allclose(gram, torch.eye(15, dtype=torch.float64), atol=0.03)


def test_sh_degree_is_validated(pkg):
    N = pkg._native
    lib = N.load()
    a = N.GsProjectArgs()
    a.cam.tile_size, a.cam.image_width, a.cam.image_height = 16, 8, 8
    a.g.n = 4
    fake = C.c_void_p(16)
    for f in ("xyz", "color_logits", "opacity", "cov3d"):
        setattr(a.g, f, fake)
    for f in ("means2d", "conics", "radii", "vis", "records", "rects", "depth_keys", "key_minmax"):
        setattr(a, f, fake)
    a.key_bits = 32
    a.g.sh_degree = 4
    assert lib.gs_project_forward(C.byref(a), None) == 1
    assert b"sh_degree" in lib.gs_last_error()
    a.g.sh_degree = 2  # without sh_rest
    assert lib.gs_project_forward(C.byref(a), None) == 1


def _scene(pkg, cuda, n=6000, W=96, H=72, seed=5):
    scene = pkg.synthetic.make_scene(n, W, H, seed=seed, sigma_range=(0.01, 0.05))
    m = pkg.synthetic.to_model(scene, pkg.GaussianModel, cuda)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        m._features_rest.copy_((0.4 * torch.randn(n, 15, 3, generator=g)).to(cuda))
        m._features_dc.copy_((torch.rand(n, 1, 3, generator=g) * 4 - 2).to(cuda))
    wv = _posed_view()

    class Cam:
        _width, _height, _FoVx, _FoVy = W, H, scene.fovx, scene.fovy

        def world_view_transform(self):
            return wv
    return m, Cam(), W, H


@pytest.mark.gpu
def test_sh_degree0_is_the_reference_render(pkg, cuda):
    m, cam, W, H = _scene(pkg, cuda)
    r = pkg.GaussianRenderer()
    a = r.render(cam, m, pkg.RenderSettings(H, W, torch.zeros(3)))
    b = r.render(cam, m, pkg.RenderSettings(H, W, torch.zeros(3), sh_degree=0))
    assert torch.equal(a["image"], b["image"])


@pytest.mark.gpu
@pytest.mark.parametrize("degree", [1, 2, 3])
def test_sh_matches_torch_statement(pkg, cuda, degree):
    from mini3dgs_amd.rasterizer import rasterize
    m, cam, W, H = _scene(pkg, cuda)
    r = pkg.GaussianRenderer()
    st = pkg.RenderSettings(H, W, torch.tensor([0.1, 0.2, 0.3]), sh_degree=degree)
    g = torch.Generator().manual_seed(9)
    cot = (torch.rand(3, H, W, generator=g) * 2 - 1).to(cuda)

    out = r.render(cam, m, st)
    (out["image"] * cot).sum().backward()
    got = {k: getattr(m, k).grad.clone() for k in ("_xyz", "_features_dc", "_features_rest")}
    img = out["image"].detach()
    for p in m.parameters():
        p.grad = None

    # reference composition: torch SH logits -> the (parity-checked) DC path
    camp = pkg.camera_params(cam, st)
    campos = torch.tensor(camp.campos, device=cuda)
    logits = sh_logits(m._xyz, m._features_dc[:, 0, :], m._features_rest, campos, degree)
    ref = rasterize(camp, m._xyz, None, m._scaling, m._rotation, logits, m._opacity.squeeze(1),
                    opacity_is_logit=True)
    (ref[0] * cot).sum().backward()
    exp = {k: getattr(m, k).grad.clone() for k in ("_xyz", "_features_dc", "_features_rest")}

    assert int(ref[6].sum()) > 1000
    assert (img - ref[0].detach()).abs().max().item() <= 1e-5
    nb = (degree + 1) ** 2 - 1
    assert torch.count_nonzero(got["_features_rest"][:, nb:]) == 0
    for k, v in exp.items():
        scale = v.abs().max().item()
        assert scale > 0, k
        err = (got[k] - v).abs().max().item()
        assert err <= 1e-4 * scale + 1e-7, (k, err, scale)
