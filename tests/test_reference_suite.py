"""The reference's own unit tests for the hot path, restated against this
package: the same classes, test names, inputs and expectations as
/root/reference/tests/test_renderer.py (TestRenderer, :93-161) and
tests/test_gaussian_model.py (TestGaussianModel, :33-140), so a reference user
finds their checks passing here.  Differences, each forced by the build:
  * the renderer runs on a HIP device (the reference's fixture says "cpu";
    this package has no CPU render path), so TestRenderer is `gpu`;
  * densification is one GPU pass here, so test_densify_operations is `gpu`,
    and needs none of the reference test's monkeypatches (its helpers exist);
  * tests/test_math_utils.py is three `pass` bodies and tests/test_camera.py
    checks the camera's projection matrices, which the render path never
    reads (only world_view_transform is on it): not restated.
"""
import math

import pytest
import torch


@pytest.fixture(scope="module")
def pkg():
    import __graft_entry__ as ge
    return ge.load_package()


def _stub_camera(width, height, fov_deg, device):
    """A duck-typed camera: the four attributes and the world_view_transform()
    method the renderer reads (renderer.py:140-150)."""
    cam = type("StubCamera", (), {})()
    cam._width, cam._height = width, height
    cam._FoVx = cam._FoVy = math.radians(fov_deg)
    wv = torch.eye(4, device=device)
    cam.world_view_transform = lambda: wv
    return cam


class _StubGaussians:
    """Axis-aligned Gaussians exposing get_xyz / get_opacity / get_features
    ([N,16,3], DC in slot 0) / get_covariance = diag(sigma^2), the accessors
    the reference's renderer reads."""

    def __init__(self, xyz, sigmas, colors_dc, opacities, device):
        f = lambda v: torch.as_tensor(v, dtype=torch.float32, device=device)
        self._xyz, sig = f(xyz), f(sigmas)
        n = self._xyz.shape[0]
        self._features = torch.zeros((n, 16, 3), device=device)
        self._features[:, 0, :] = f(colors_dc)
        self._opacity = f(opacities).view(-1, 1)
        self._cov = torch.diag_embed(sig * sig)

    get_xyz = property(lambda self: self._xyz)
    get_opacity = property(lambda self: self._opacity)
    get_features = property(lambda self: self._features)
    get_covariance = property(lambda self: self._cov)


@pytest.mark.gpu
class TestRenderer:
    def setup_method(self):
        self.device = "cuda"
        self.H = self.W = 64

    def _render(self, pkg, gs, size=None, debug=True):
        w = h = size or self.W
        cam = _stub_camera(w, h, 60.0, self.device)
        settings = pkg.RenderSettings(image_height=self.H, image_width=self.W,
                                      bg_color=torch.zeros(3, device=self.device), scale_modifier=1.0,
                                      debug=debug)
        self.settings = settings
        return pkg.GaussianRenderer(tile_size=16, radius_min=0.01, radius_max=50.0).render(cam, gs, settings)

    def test_shapes_and_types(self, pkg):
        gs = _StubGaussians([[0.0, 0.0, 1.0]], [[0.01] * 3], [[1.0, 1.0, 1.0]], [0.8], self.device)
        out = self._render(pkg, gs)
        assert out["image"].shape == (3, self.H, self.W)
        assert out["alpha"].shape == (1, self.H, self.W)
        assert out["depth"].shape == (1, self.H, self.W)
        assert out["viewspace_points"].shape[1] == 2
        assert out["visibility_filter"].dtype == torch.bool
        assert out["radii"].ndim == 1
        assert out["conics"].shape[-2:] == (2, 2)

    def test_culling_all_behind(self, pkg):
        # a 32x32 camera with the 64x64 settings, as the reference test has it
        gs = _StubGaussians([[0.0, 0.0, -1.0], [0.0, 0.0, -2.0]], [[0.01] * 3] * 2,
                            [[1.0, 0.0, 0.0], [0.0, 1.0, 0.0]], [0.5, 0.5], self.device)
        out = self._render(pkg, gs, size=32)
        bg = self.settings.bg_color.view(3, 1, 1).repeat(1, self.H, self.W)
        assert torch.allclose(out["image"], bg)
        assert torch.count_nonzero(out["alpha"]) == 0

    def test_front_to_back_blending_center_pixel(self, pkg):
        # two Gaussians on the optical axis (pixel (32, 32)) at Z = 1 (red) and
        # Z = 2 (green), opacity 0.5 each: A = 0.5 + 0.5 * 0.5 = 0.75,
        # rgb = 0.5 sigmoid(red) + 0.25 sigmoid(green), depth = (0.5 + 0.5) / 0.75
        gs = _StubGaussians([[0.0, 0.0, 1.0], [0.0, 0.0, 2.0]], [[0.01] * 3] * 2,
                            [[1.0, 0.0, 0.0], [0.0, 1.0, 0.0]], [0.5, 0.5], self.device)
        out = self._render(pkg, gs)
        cx, cy = self.W // 2, self.H // 2
        rgb, a, d = out["image"][:, cy, cx], out["alpha"][0, cy, cx], out["depth"][0, cy, cx]
        assert torch.allclose(a, torch.tensor(0.75, device=self.device), atol=1e-3)
        s0 = torch.sigmoid(torch.tensor([1.0, 0.0, 0.0], device=self.device))
        s1 = torch.sigmoid(torch.tensor([0.0, 1.0, 0.0], device=self.device))
        assert torch.allclose(rgb, 0.5 * s0 + 0.25 * s1, atol=1e-3)
        assert torch.allclose(d, torch.tensor(4 / 3, device=self.device), atol=2e-2)


def _quat_to_mat(q):
    """[w, x, y, z] -> R, restated from the rotation formula
    (math_utils.py:20-24) for the covariance check."""
    q = torch.nn.functional.normalize(q, dim=-1)
    w, x, y, z = q.unbind(-1)
    rows = [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
            2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
            2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]
    return torch.stack(rows, -1).view(-1, 3, 3)


def _make_model(pkg, n, extent=1.0, device="cpu"):
    m = pkg.GaussianModel(pkg.TrainingConfig())
    m.create_from_random(n, extent, device=device)
    return m


class TestGaussianModel:
    def test_parameter_initialization(self, pkg):
        n = 256
        m = _make_model(pkg, n)
        assert m.get_xyz.shape == (n, 3)
        assert m._features_dc.shape == (n, 1, 3)
        assert m._features_rest.shape == (n, 15, 3)
        assert m._scaling.shape == (n, 3)
        assert m._rotation.shape == (n, 4)
        assert m._opacity.shape == (n, 1)
        assert m.xyz_gradient_accum.shape == (n, 3)
        assert m.denom.shape == (n, 1)
        assert m.max_radii2D.shape[0] == n

    def test_property_access(self, pkg):
        n = 64
        m = _make_model(pkg, n)
        sigma = m.get_scaling
        assert sigma.shape == (n, 3) and torch.all(sigma > 0)
        qn = torch.linalg.norm(m.get_rotation, dim=-1)
        assert torch.allclose(qn, torch.ones_like(qn), atol=1e-5)
        a = m.get_opacity
        assert torch.all(a > 0) and torch.all(a < 1)
        feats = m.get_features
        assert feats.shape == (n, 16, 3)
        assert torch.allclose(feats, torch.cat([m._features_dc, m._features_rest], dim=1))

    def test_covariance_computation(self, pkg):
        n = 32
        m = _make_model(pkg, n)
        cov = m.compute_3d_covariance()
        assert cov.shape == (n, 3, 3)
        R = _quat_to_mat(m.get_rotation)
        want = R @ torch.diag_embed(m.get_scaling ** 2) @ R.transpose(-1, -2)
        assert torch.allclose(cov, want, atol=1e-5, rtol=1e-5)
        assert torch.all(torch.linalg.eigvalsh(cov) > -1e-6)
        # get_covariance is the working accessor here (the reference's calls a
        # missing attribute, gaussian_model.py:127)
        assert torch.allclose(m.get_covariance, cov)

    @pytest.mark.gpu
    def test_densify_operations(self, pkg):
        n, extent, k = 64, 1.0, 8
        m = _make_model(pkg, n, extent, device="cuda")
        m._xyz.grad = torch.ones_like(m._xyz)  # every Gaussian above the gradient threshold
        with torch.no_grad():
            m._scaling[:k] = math.log(0.06 * extent)        # > 0.03 extent: split
            m._scaling[k:2 * k] = math.log(0.005 * extent)  # <= 0.01 extent: clone
        n0 = m.get_num_points()
        m.density_and_split(grad_threshold=0.5, scene_extent=extent)
        assert m.get_num_points() == n0 + k  # k originals replaced by 2k
        m._xyz.grad = torch.ones_like(m._xyz)
        n1 = m.get_num_points()
        m.density_and_clone(grad_threshold=0.5, scene_extent=extent)
        assert m.get_num_points() == n1 + k  # k clones, the originals stay
