"""Config C1 (BASELINE.json configs[0]): 5k random Gaussians, one 256x256
camera, rendered through the drop-in GaussianRenderer.

The reference's examples/simple_scene.py is an empty file (SURVEY.md section
2, row 15, leaves it to the build).  This one runs the reference's own
workflow, in the reference's names:

  1. GaussianModel.create_from_random(5000) (gaussian_model.py:78-98), moved
     in front of the camera, and a Camera built by the reference's pose
     convention (camera.py:80-141); RenderSettings + GaussianRenderer().render()
     (renderer.py:13-114); a backward through the image.
  2. The C1 scene the reference's own CPU renderer drew (tests/golden/
     c1_forward.npz, 5k Gaussians, 256x256; made by tests/golden/make_golden.py,
     ~163 s in the reference) drawn again through the duck-typed accessors the
     reference renderer reads (get_xyz / get_covariance / get_features /
     get_opacity), with the largest difference from the reference's image.

    python examples/simple_scene.py [--out simple_scene.png]

Needs a HIP device (the renderer has no CPU path).
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C1_FIXTURE = os.path.join(ROOT, "tests", "golden", "c1_forward.npz")


def _package():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    return ge.load_package()


class _Gaussians:
    """The accessors renderer.py reads (:88-94, :135, :166), over plain tensors."""

    def __init__(self, torch, xyz, cov3d, logits, opacity, device):
        t = lambda a: torch.tensor(np.asarray(a, np.float32), device=device)
        n = len(xyz)
        feats = np.zeros((n, 16, 3), np.float32)
        feats[:, 0] = logits
        self.get_xyz, self.get_covariance = t(xyz), t(np.asarray(cov3d).reshape(n, 3, 3))
        self.get_features, self.get_opacity = t(feats), t(np.asarray(opacity).reshape(n, 1))


class _Cam:
    """camera._width/_height/_FoVx/_FoVy and world_view_transform() (renderer.py:140-150)."""

    def __init__(self, torch, w, h, fovx, fovy, wv):
        self._width, self._height, self._FoVx, self._FoVy = int(w), int(h), float(fovx), float(fovy)
        self._wv = torch.as_tensor(np.asarray(wv, np.float32))

    def world_view_transform(self):
        return self._wv


def run(out_png: str | None = None, check: bool = True, verbose: bool = True) -> dict:
    import torch
    pkg = _package()
    dev = torch.device("cuda", 0)
    W = H = 256

    # 1. the reference's workflow: a random model, a posed camera, render + backward
    g = pkg.GaussianModel(pkg.TrainingConfig())
    g.create_from_random(5000, scene_extent=1.0, device=dev, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():  # (seeded: the example prints the same numbers every run)
        gen = torch.Generator().manual_seed(1)
        g._scaling.add_((torch.rand(g._scaling.shape, generator=gen) - 0.5).to(dev))
        g._opacity.copy_(torch.randn(g._opacity.shape, generator=gen).to(dev))
    cam = pkg.Camera(uid=0, R=np.eye(3, dtype=np.float32), T=np.array([0.0, 0.0, -3.0], np.float32),
                     FoVx=math.radians(60), FoVy=math.radians(60), image=None, image_name="c1",
                     width=W, height=H)  # camera centre 3 units behind the origin, looking down +z
    settings = pkg.RenderSettings(image_height=H, image_width=W, bg_color=torch.zeros(3))
    renderer = pkg.GaussianRenderer()
    out = renderer.render(cam, g, settings)
    out["image"].sum().backward()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        out = renderer.render(cam, g, settings)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 100.0
    res = {"visible": int(out["visibility_filter"].sum()), "mean_alpha": float(out["alpha"].detach().mean()),
           "render_ms": ms, "grad_xyz_finite": bool(torch.isfinite(g._xyz.grad).all())}
    if out_png:
        _write_png(out_png, out["image"].detach().clamp(0, 1).cpu().numpy())
        res["png"] = out_png

    # 2. the C1 scene the reference rendered (its own outputs, a fixture)
    if check and os.path.exists(C1_FIXTURE):
        f = np.load(C1_FIXTURE)
        gs = _Gaussians(torch, f["xyz"], f["cov3d"], f["color_logits"], f["opacity"], dev)
        c = _Cam(torch, f["cam_width"], f["cam_height"], f["fovx"], f["fovy"], f["wv"])
        st = pkg.RenderSettings(image_height=int(f["height"]), image_width=int(f["width"]),
                                bg_color=torch.tensor(np.asarray(f["bg"], np.float32)))
        o = renderer.render(c, gs, st)
        res["c1_max_abs_err_image"] = float(np.abs(o["image"].cpu().numpy() - f["image"]).max())
        res["c1_max_abs_err_alpha"] = float(np.abs(o["alpha"].cpu().numpy() - f["alpha"]).max())
        res["c1_visibility_equal"] = bool(np.array_equal(o["visibility_filter"].cpu().numpy(), f["vis"].astype(bool)))
    if verbose:
        print("simple_scene (C1):", ", ".join(f"{k}={v:.4g}" if isinstance(v, float) else f"{k}={v}"
                                             for k, v in res.items()))
    return res


def _write_png(path: str, img: np.ndarray) -> None:
    """[3,H,W] in [0,1] -> 8-bit RGB PNG (zlib only, no imaging library)."""
    import struct
    import zlib
    rgb = (np.transpose(img, (1, 2, 0)) * 255.0 + 0.5).astype(np.uint8)
    h, w, _ = rgb.shape
    raw = b"".join(b"\x00" + rgb[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
    with open(path, "wb") as fh:
        fh.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
                 chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--out", default=None, help="write the rendered image as a PNG")
    args = ap.parse_args()
    r = run(args.out)
    if "c1_max_abs_err_image" in r and not (r["c1_max_abs_err_image"] <= 1e-4 and r["c1_visibility_equal"]):
        sys.exit("C1 differs from the reference's image")
