"""Generate golden vectors by running the REFERENCE renderer in this container.

    python tests/golden/make_golden.py [--ref /root/reference] [--only NAME] [--skip-large]

This script is the only place that imports the reference
(/root/reference/src/core/renderer.py, gaussian_model.py, camera.py); it runs
at fixture-generation time in the build container, never on the GPU box and
never from the tests.  Each case is written as <name>.npz holding:

  inputs : xyz, cov3d, color_logits, opacity, wv, width, height, cam_width,
           cam_height, fovx, fovy, bg  (+ scaling, rotation for model cases)
  outputs: image, alpha, depth, means2d, conics, radii, vis
  grads  : d_xyz, d_cov3d (or d_scaling, d_rotation), d_color_logits,
           d_opacity for L = <g_image,image> + <g_alpha,alpha> + <g_depth,depth>
           (+ <g_means2d,viewspace_points> + <g_conics,conics>), cotangents
           stored alongside (seeded U[-1,1]).

Backward fixtures stay at <=64x64: the reference backward is autograd through
a per-pixel Python loop, O(contributing pairs x H x W).
The duck-typed camera / Gaussian stand-ins follow the contract the reference
renderer reads (renderer.py:59,88-94,135,140-150,166), the same contract its
own tests satisfy (tests/test_renderer.py:7-53).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


class StubCamera:
    """What renderer.py reads from a camera: _width/_height/_FoVx/_FoVy and a
    callable world_view_transform() (renderer.py:140-150)."""

    def __init__(self, w, h, fovx, fovy, wv):
        self._width, self._height = int(w), int(h)
        self._FoVx, self._FoVy = float(fovx), float(fovy)
        self._wv = wv

    def world_view_transform(self):
        return self._wv


class StubGaussians:
    """get_xyz / get_covariance / get_features [N,16,3] / get_opacity [N,1]
    (renderer.py:88-94,135,166); every tensor a leaf with requires_grad."""

    def __init__(self, xyz, cov3d, logits, opacity):
        n = xyz.shape[0]
        self.xyz = torch.tensor(xyz, dtype=torch.float32, requires_grad=True)
        self.cov = torch.tensor(cov3d, dtype=torch.float32, requires_grad=True)
        feats = np.zeros((n, 16, 3), np.float32)
        feats[:, 0, :] = logits
        self.feats = torch.tensor(feats, requires_grad=True)
        self.op = torch.tensor(np.asarray(opacity, np.float32).reshape(n, 1), requires_grad=True)

    @property
    def get_xyz(self):
        return self.xyz

    @property
    def get_covariance(self):
        return self.cov

    @property
    def get_features(self):
        return self.feats

    @property
    def get_opacity(self):
        return self.op


class ModelAdapter:
    """Wraps the reference GaussianModel; its own get_covariance is broken
    (gaussian_model.py:127 `self._get_rotation`), so the working
    compute_3d_covariance (:200-207) is what the adapter exposes."""

    def __init__(self, m):
        self.m = m

    @property
    def get_xyz(self):
        return self.m.get_xyz

    @property
    def get_covariance(self):
        return self.m.compute_3d_covariance()

    @property
    def get_features(self):
        return self.m.get_features

    @property
    def get_opacity(self):
        return self.m.get_opacity

    @property
    def _features_dc(self):
        return self.m._features_dc


def fov_pair(w, h, fovx_deg):
    fx = math.radians(fovx_deg)
    fy = 2.0 * math.atan(math.tan(fx / 2) * h / w)
    return fx, fy


def synth(n, w, h, rng, zlo=2.0, zhi=6.0, slo=0.002, shi=0.01, fovx_deg=60.0, full_rot=True):
    """SURVEY.md 8(d) synthetic distribution."""
    fx, fy = fov_pair(w, h, fovx_deg)
    z = rng.uniform(zlo, zhi, n)
    x = rng.uniform(-1, 1, n) * z * math.tan(fx / 2)
    y = rng.uniform(-1, 1, n) * z * math.tan(fy / 2)
    xyz = np.stack([x, y, z], 1).astype(np.float32)
    sig = np.exp(rng.uniform(math.log(slo), math.log(shi), (n, 3))).astype(np.float32)
    q = rng.standard_normal((n, 4)).astype(np.float32) if full_rot else np.tile([1, 0, 0, 0], (n, 1)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    R = quat_to_R(q)
    cov = (R * (sig ** 2)[:, None, :]) @ np.transpose(R, (0, 2, 1))
    logits = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    opac = (1.0 / (1.0 + np.exp(-rng.standard_normal(n)))).astype(np.float32)
    return xyz, cov.astype(np.float32), logits, opac, fx, fy


def quat_to_R(q):
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    return np.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], 1).reshape(-1, 3, 3)


def run_case(ref, name, xyz, cov, logits, opac, wv, W, H, fovx, fovy, bg, cam_wh=None,
             backward=True, extra_cot=False, seed=1, model=None, tile=16, radius_min=0.01, radius_max=50.0):
    from src.core.renderer import GaussianRenderer, RenderSettings
    cw, ch = cam_wh if cam_wh is not None else (W, H)
    cam = StubCamera(cw, ch, fovx, fovy, torch.tensor(np.asarray(wv, np.float32)))
    gs = ModelAdapter(model) if model is not None else StubGaussians(xyz, cov, logits, opac)
    settings = RenderSettings(image_height=H, image_width=W,
                              bg_color=torch.tensor(np.asarray(bg, np.float32)))
    # the constructor's full range (renderer.py:24-28): tile_size changes the
    # image (a pixel blends its whole tile's list), radius_max/min the binning
    rend = GaussianRenderer(tile_size=tile, radius_min=radius_min, radius_max=radius_max)
    t0 = time.time()
    out = rend.render(cam, gs, settings)
    t_fwd = time.time() - t0
    rec = dict(
        width=W, height=H, cam_width=cw, cam_height=ch, fovx=fovx, fovy=fovy,
        wv=np.asarray(wv, np.float32), bg=np.asarray(bg, np.float32),
        tile=int(tile), radius_min=float(radius_min), radius_max=float(radius_max),
        image=out["image"].detach().numpy(), alpha=out["alpha"].detach().numpy(),
        depth=out["depth"].detach().numpy(), means2d=out["viewspace_points"].detach().numpy(),
        conics=out["conics"].detach().numpy(), radii=out["radii"].detach().numpy(),
        vis=out["visibility_filter"].numpy(),
    )
    if model is not None:
        m = model
        rec.update(xyz=m._xyz.detach().numpy(), scaling=m._scaling.detach().numpy(),
                   rotation=m._rotation.detach().numpy(),
                   cov3d=m.compute_3d_covariance().detach().numpy(),
                   color_logits=m._features_dc.detach().numpy()[:, 0, :],
                   opacity_raw=m._opacity.detach().numpy()[:, 0],
                   opacity=m.get_opacity.detach().numpy()[:, 0])
    else:
        rec.update(xyz=xyz, cov3d=cov, color_logits=logits, opacity=np.asarray(opac, np.float32))
    t_bwd = 0.0
    if backward:
        g = np.random.default_rng(seed)
        n = rec["xyz"].shape[0]
        cot = dict(g_image=g.uniform(-1, 1, (3, H, W)).astype(np.float32),
                   g_alpha=g.uniform(-1, 1, (1, H, W)).astype(np.float32),
                   g_depth=g.uniform(-1, 1, (1, H, W)).astype(np.float32))
        if extra_cot:
            cot["g_means2d"] = g.uniform(-1, 1, (n, 2)).astype(np.float32)
            cot["g_conics"] = g.uniform(-1, 1, (n, 2, 2)).astype(np.float32)
        loss = (out["image"] * torch.from_numpy(cot["g_image"])).sum() \
            + (out["alpha"] * torch.from_numpy(cot["g_alpha"])).sum() \
            + (out["depth"] * torch.from_numpy(cot["g_depth"])).sum()
        if extra_cot:
            loss = loss + (out["viewspace_points"] * torch.from_numpy(cot["g_means2d"])).sum() \
                + (out["conics"] * torch.from_numpy(cot["g_conics"])).sum()
        t0 = time.time()
        loss.backward()
        t_bwd = time.time() - t0
        rec.update(cot)
        z = lambda t, shape: (t.grad.numpy() if t.grad is not None else np.zeros(shape, np.float32))
        if model is not None:
            m = model
            rec.update(d_xyz=z(m._xyz, (n, 3)), d_scaling=z(m._scaling, (n, 3)),
                       d_rotation=z(m._rotation, (n, 4)),
                       d_color_logits=z(m._features_dc, (n, 1, 3))[:, 0, :],
                       d_opacity_raw=z(m._opacity, (n, 1))[:, 0])
        else:
            rec.update(d_xyz=z(gs.xyz, (n, 3)), d_cov3d=z(gs.cov, (n, 3, 3)),
                       d_color_logits=z(gs.feats, (n, 16, 3))[:, 0, :],
                       d_opacity=z(gs.op, (n, 1))[:, 0])
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **rec)
    return dict(name=name, N=int(rec["xyz"].shape[0]), W=W, H=H, backward=backward, tile=int(tile),
                radius_max=float(radius_max),
                ref_fwd_s=round(t_fwd, 3), ref_bwd_s=round(t_bwd, 3),
                visible=int(rec["vis"].sum()))


def cases(ref, only=None, skip_large=False):
    ident = np.eye(4, dtype=np.float32)
    fov60 = math.radians(60.0)
    out = []

    def want(n):
        return only is None or n in only

    # 1. the reference's own known answer scene (test_renderer.py:127-161)
    if want("kat_two_coaxial"):
        out.append(run_case(ref, "kat_two_coaxial",
                            np.array([[0, 0, 1], [0, 0, 2]], np.float32),
                            np.stack([np.diag([1e-4] * 3)] * 2).astype(np.float32),
                            np.array([[1, 0, 0], [0, 1, 0]], np.float32), [0.5, 0.5],
                            ident, 64, 64, fov60, fov60, [0, 0, 0]))
    # 2. single Gaussian (test_shapes_and_types, :95-111)
    if want("kat_single"):
        out.append(run_case(ref, "kat_single", np.array([[0, 0, 1]], np.float32),
                            np.diag([1e-4] * 3)[None].astype(np.float32),
                            np.array([[1, 1, 1]], np.float32), [0.8], ident, 64, 64, fov60, fov60,
                            [0, 0, 0]))
    # 3. all behind the camera, camera 32x32 vs settings 64x64 (:113-125)
    if want("all_behind"):
        out.append(run_case(ref, "all_behind", np.array([[0, 0, -1], [0, 0, -2]], np.float32),
                            np.stack([np.diag([1e-4] * 3)] * 2).astype(np.float32),
                            np.array([[1, 0, 0], [0, 1, 0]], np.float32), [0.5, 0.5], ident,
                            64, 64, fov60, fov60, [0.2, 0.3, 0.4], cam_wh=(32, 32), backward=False))
    # 4. random scene, full rotations, bg != 0 (double-bg path), extra cotangents
    if want("random_bg"):
        rng = np.random.default_rng(4)
        xyz, cov, lg, op, fx, fy = synth(60, 64, 64, rng, slo=0.01, shi=0.05)
        out.append(run_case(ref, "random_bg", xyz, cov, lg, op, ident, 64, 64, fx, fy,
                            [0.2, 0.3, 0.4], extra_cot=True))
    # 5. huge Gaussians: radius clamp at 50 px, many tiles each
    if want("radius_clamp"):
        rng = np.random.default_rng(5)
        xyz, cov, lg, op, fx, fy = synth(6, 64, 64, rng, slo=0.3, shi=0.6)
        out.append(run_case(ref, "radius_clamp", xyz, cov, lg, op * 0.3, ident, 64, 64, fx, fy,
                            [0.1, 0.1, 0.1]))
    # 6. centres off-screen / negative pixel coords (int() truncation toward 0)
    if want("offscreen"):
        rng = np.random.default_rng(6)
        n = 24
        fx, fy = fov_pair(48, 48, 60.0)
        z = rng.uniform(2, 4, n)
        px = rng.uniform(-6, 54, n)
        py = rng.uniform(-6, 54, n)
        fpx = 0.5 * 48 / math.tan(fx / 2)
        x = (px - 24) * z / fpx
        y = -(py - 24) * z / fpx
        xyz = np.stack([x, y, z], 1).astype(np.float32)
        sig = np.full((n, 3), 0.03, np.float32)
        cov = np.stack([np.diag(s ** 2) for s in sig]).astype(np.float32)
        out.append(run_case(ref, "offscreen", xyz, cov, rng.uniform(-1, 1, (n, 3)).astype(np.float32),
                            rng.uniform(0.3, 0.9, n).astype(np.float32), ident, 48, 48, fx, fy,
                            [0, 0, 0]))
    # 7. dense overlap: A crosses 0.995 (termination), raw opacity > 1 (alpha clamp)
    if want("saturate"):
        rng = np.random.default_rng(7)
        n = 40
        fx, fy = fov_pair(32, 32, 60.0)
        z = np.sort(rng.uniform(2, 3, n))
        xy = rng.uniform(-0.15, 0.15, (n, 2)) * z[:, None]
        xyz = np.concatenate([xy, z[:, None]], 1).astype(np.float32)
        cov = np.stack([np.diag([0.04 ** 2] * 3)] * n).astype(np.float32)
        op = rng.uniform(0.6, 0.95, n).astype(np.float32)
        op[::9] = 1.5
        out.append(run_case(ref, "saturate", xyz, cov, rng.uniform(-2, 2, (n, 3)).astype(np.float32),
                            op, ident, 32, 32, fx, fy, [0.5, 0.5, 0.5]))
    # 8. posed camera from the reference's W2C producer, non-square image with
    #    partial tiles, camera size != image size
    if want("posed_camera"):
        from src.core.camera import CameraUtils
        rng = np.random.default_rng(8)
        ang = 0.3
        R_cw = np.array([[math.cos(ang), 0, math.sin(ang)], [0, 1, 0],
                         [-math.sin(ang), 0, math.cos(ang)]], np.float32)
        C_w = np.array([0.4, -0.2, -0.5], np.float32)
        wv = CameraUtils.build_world_view_matrix(R_cw, C_w, True).numpy().astype(np.float32)
        xyz, cov, lg, op, fx, fy = synth(50, 40, 36, rng, slo=0.01, shi=0.06)
        xyz = ((xyz - wv[:3, 3]) @ wv[:3, :3]).astype(np.float32)  # world pts seen by this camera
        out.append(run_case(ref, "posed_camera", xyz, cov, lg, op, wv, 40, 36, fx, fy,
                            [0.05, 0.1, 0.0], cam_wh=(44, 36)))
    # 9. reference GaussianModel.create_from_random path (grads to raw params)
    if want("model_random"):
        from src.core.gaussian_model import GaussianModel
        from config.config import TrainingConfig
        torch.manual_seed(9)
        m = GaussianModel(TrainingConfig())
        m.create_from_random(80, 1.0)
        with torch.no_grad():  # shift in front of the camera (SURVEY 8d, C1 variant)
            m._xyz[:, 2] += 3.0
            m._opacity.normal_()
            m._scaling.add_(torch.empty_like(m._scaling).uniform_(-0.7, 0.7))
        fx, fy = fov_pair(64, 64, 60.0)
        out.append(run_case(ref, "model_random", None, None, None, None, ident, 64, 64, fx, fy,
                            [0, 0, 0], model=m))
    # 11-14. GaussianRenderer(tile_size=..., radius_min/max=...) beyond the
    # defaults: the tile a pixel belongs to decides which Gaussians it blends
    # (pixels outside a Gaussian's AABB but inside a touched tile still blend it)
    if want("tile8"):
        rng = np.random.default_rng(11)
        xyz, cov, lg, op, fx, fy = synth(60, 64, 64, rng, slo=0.01, shi=0.05)
        out.append(run_case(ref, "tile8", xyz, cov, lg, op, ident, 64, 64, fx, fy, [0.2, 0.3, 0.4],
                            extra_cot=True, tile=8))
    if want("tile32"):
        rng = np.random.default_rng(12)
        xyz, cov, lg, op, fx, fy = synth(70, 72, 56, rng, slo=0.01, shi=0.06)
        out.append(run_case(ref, "tile32", xyz, cov, lg, op, ident, 72, 56, fx, fy, [0.1, 0.0, 0.2], tile=32))
    if want("tile12"):
        rng = np.random.default_rng(13)
        xyz, cov, lg, op, fx, fy = synth(50, 52, 44, rng, slo=0.01, shi=0.05)
        out.append(run_case(ref, "tile12", xyz, cov, lg, op, ident, 52, 44, fx, fy, [0.0, 0.1, 0.0], tile=12))
    if want("radius80_tile8"):
        # 3 sigma beyond 80 px: the clamp binds at radius_max=80, and rects span
        # 12 x 10 tiles of 8 px (more than the 8 x 8 of the default setup)
        rng = np.random.default_rng(14)
        xyz, cov, lg, op, fx, fy = synth(6, 96, 80, rng, zlo=2.0, zhi=3.0, slo=0.7, shi=1.2)
        out.append(run_case(ref, "radius80_tile8", xyz, cov, lg, op * 0.3, ident, 96, 80, fx, fy,
                            [0.1, 0.1, 0.1], tile=8, radius_min=0.6, radius_max=80.0))
    # 10. C1-shaped forward only (5k Gaussians, 256x256, SURVEY 8d distribution)
    if want("c1_forward") and not skip_large:
        rng = np.random.default_rng(0)
        xyz, cov, lg, op, fx, fy = synth(5000, 256, 256, rng)
        out.append(run_case(ref, "c1_forward", xyz, cov, lg, op, ident, 256, 256, fx, fy,
                            [0, 0, 0], backward=False))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--skip-large", action="store_true")
    a = ap.parse_args()
    sys.path.insert(0, a.ref)
    torch.set_num_threads(8)
    man_path = os.path.join(HERE, "manifest.json")
    manifest = json.load(open(man_path)) if os.path.exists(man_path) else {}
    for rec in cases(a.ref, set(a.only) if a.only else None, a.skip_large):
        manifest[rec["name"]] = rec
        print(json.dumps(rec), flush=True)
    json.dump(manifest, open(man_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
