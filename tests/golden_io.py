"""Helpers shared by the tests: fixture loading and tolerance checks.

Tolerances (north_star: outputs within 1e-4 fp32 of the reference):
  * image / alpha / means2d / radii: abs 1e-4
  * conics: rel 1e-4 (entries scale like 1/sigma_px^2)
  * depth = D / (A + 1e-6): abs 1e-4 where alpha >= 1e-2, abs 1e-4 * depth
    scale elsewhere (the division amplifies rounding for tiny A)
  * gradients: |d - d_ref| <= 2e-3 * max|d_ref| + 1e-5 per tensor
    (reference backward is autograd over a different but algebraically
    identical expression order)
"""
from __future__ import annotations

import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

IMG_ATOL = 1e-4
GRAD_RTOL = 2e-3
GRAD_ATOL = 1e-5


def oracle():
    sys.path.insert(0, ROOT)
    from oracle import oracle as o  # test infrastructure only
    return o


def fixture_names():
    return sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    return {k: z[k] for k in z.files}


def scene_of(f):
    o = oracle()
    return o.Scene(xyz=f["xyz"], cov3d=f["cov3d"], color_logits=f["color_logits"],
                   opacity=f["opacity"], wv=f["wv"], width=int(f["width"]), height=int(f["height"]),
                   fovx=float(f["fovx"]), fovy=float(f["fovy"]), bg=f["bg"],
                   cam_width=int(f["cam_width"]), cam_height=int(f["cam_height"]))


def max_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b)))


def check_image(out, ref, atol=IMG_ATOL):
    """Returns a list of failure strings (empty = pass)."""
    errs = []
    for k in ("image", "alpha"):
        e = max_err(out[k], ref[k])
        if not e <= atol:
            errs.append(f"{k}: max abs err {e:.3g} > {atol}")
    a = np.asarray(ref["alpha"], np.float64)
    d_out = np.asarray(out["depth"], np.float64)
    d_ref = np.asarray(ref["depth"], np.float64)
    scale = max(1.0, float(np.max(np.abs(d_ref))) if d_ref.size else 1.0)
    tol = np.where(a >= 1e-2, atol * scale, atol * scale * 100)
    bad = np.abs(d_out - d_ref) > tol
    if bad.any():
        errs.append(f"depth: {int(bad.sum())} px over tol, max err {max_err(d_out, d_ref):.3g}")
    return errs


def check_projection(out, ref, atol=IMG_ATOL):
    errs = []
    if not np.array_equal(np.asarray(out["vis"], bool), np.asarray(ref["vis"], bool)):
        errs.append("visibility_filter differs")
    for k in ("means2d", "radii"):
        e = max_err(out[k], ref[k])
        if not e <= atol * max(1.0, float(np.max(np.abs(ref[k])))):
            errs.append(f"{k}: max abs err {e:.3g}")
    c, cr = np.asarray(out["conics"], np.float64), np.asarray(ref["conics"], np.float64)
    rel = np.abs(c - cr) / np.maximum(np.abs(cr).reshape(len(cr), -1).max(1)[:, None, None], 1e-30)
    if rel.size and rel.max() > 1e-4:
        errs.append(f"conics: max rel err {rel.max():.3g}")
    return errs


def check_grad(name, d, dref, rtol=GRAD_RTOL, atol=GRAD_ATOL):
    d = np.asarray(d, np.float64).reshape(np.shape(dref))
    dref = np.asarray(dref, np.float64)
    scale = float(np.max(np.abs(dref))) if dref.size else 0.0
    e = max_err(d, dref)
    tol = rtol * scale + atol
    if not e <= tol:
        return [f"grad {name}: max abs err {e:.3g} > tol {tol:.3g} (scale {scale:.3g})"]
    return []
