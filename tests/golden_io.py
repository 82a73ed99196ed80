"""Helpers shared by the tests: fixture loading and tolerance checks.

Tolerances (north_star: outputs within 1e-4 fp32 of the reference):
  * image / alpha / means2d / radii: abs 1e-4
  * conics: rel 1e-4 (entries scale like 1/sigma_px^2)
  * depth = D / (A + 1e-6): abs 1e-4 where alpha >= 1e-2, abs 1e-4 * depth
    scale elsewhere (the division amplifies rounding for tiny A)
  * scenes checked against the oracle (no reference run possible at that
    size) may exempt KNIFE-EDGE pixels only: pixels whose oracle replay
    came within a few ulps of a decision threshold (knife_edge below; the
    GPU's exp is ~1 ulp from glibc's, so such a pixel may decide the
    other way), each one reported
  * gradients: |d - d_ref| <= 1e-4 * max|d_ref| + 1e-7 per tensor
    (reference backward is autograd over a different but algebraically
    identical expression order).  On oracle scenes
    with knife-edge pixels that flipped, the Gaussians whose footprint
    covers such a pixel (touching_gaussians) are exempt and reported: a
    flipped termination changes every contributor's dL/dalpha there.
"""
from __future__ import annotations

import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

IMG_ATOL = 1e-4
GRAD_RTOL = 1e-4
GRAD_ATOL = 1e-7


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
                   cam_width=int(f["cam_width"]), cam_height=int(f["cam_height"]), **renderer_kwargs(f, "tile"))


def renderer_kwargs(f, tile_key="tile_size"):
    """The fixture's GaussianRenderer(tile_size, radius_min, radius_max)
    (defaults 16, 0.01, 50 for fixtures that predate the keys)."""
    return {tile_key: int(f["tile"]) if "tile" in f else 16,
            "radius_min": float(f["radius_min"]) if "radius_min" in f else 0.01,
            "radius_max": float(f["radius_max"]) if "radius_max" in f else 50.0}


def max_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b)))


# knife-edge thresholds, in ulps of the threshold value (gso_fwd_out.margin):
# the w < 1e-5 skip flips only within exp's rounding (~2 ulps of w) -- a
# flipped pair moves A by <= 1e-5 and depth by <= 1e-5 / A x its depth gap,
# and may cascade into the break; A at the 0.995 break differs by a few ulps
# when nothing but exp's rounding differs
KNIFE_W_ULPS = 4.0
KNIFE_A_ULPS = 16.0


def knife_edge(margin):
    """[H,W] bool: pixels within rounding of a blend decision."""
    return (np.asarray(margin[1]) <= KNIFE_A_ULPS) | (np.asarray(margin[0]) <= KNIFE_W_ULPS)


def pixel_errors(out, ref, atol=IMG_ATOL):
    """[H,W] bool: pixels whose image/alpha (abs atol) or depth (abs atol where
    alpha >= 1e-2, atol x depth scale x 100 elsewhere) is out of tolerance."""
    img = np.abs(np.asarray(out["image"], np.float64) - np.asarray(ref["image"], np.float64)) > atol
    bad = img.any(0) | (np.abs(np.asarray(out["alpha"], np.float64) - np.asarray(ref["alpha"], np.float64)) > atol)[0]
    a = np.asarray(ref["alpha"], np.float64)[0]
    d_out = np.asarray(out["depth"], np.float64)[0]
    d_ref = np.asarray(ref["depth"], np.float64)[0]
    scale = max(1.0, float(np.max(np.abs(d_ref))) if d_ref.size else 1.0)
    tol = np.where(a >= 1e-2, atol, atol * scale * 100)
    return bad | (np.abs(d_out - d_ref) > tol)


def check_image(out, ref, atol=IMG_ATOL, exempt=None):
    """Returns a list of failure strings (empty = pass).  exempt: optional
    [H,W] bool of knife-edge pixels (oracle scenes only)."""
    bad = pixel_errors(out, ref, atol)
    if exempt is not None:
        bad &= ~exempt
    if bad.any():
        ys, xs = np.nonzero(bad)
        return [f"{int(bad.sum())} px out of tolerance (first at y={ys[0]}, x={xs[0]}); max errs image "
                f"{max_err(out['image'], ref['image']):.3g}, alpha {max_err(out['alpha'], ref['alpha']):.3g}, "
                f"depth {max_err(out['depth'], ref['depth']):.3g}"]
    return []


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


def check_grad(name, d, dref, rtol=GRAD_RTOL, atol=GRAD_ATOL, rows=None):
    """rows: optional [N] bool, the Gaussians to check (the scale stays the
    whole tensor's max |d_ref|)."""
    d = np.asarray(d, np.float64).reshape(np.shape(dref))
    dref = np.asarray(dref, np.float64)
    scale = float(np.max(np.abs(dref))) if dref.size else 0.0
    if rows is not None:
        d, dref = d[rows], dref[rows]
    e = max_err(d, dref)
    tol = rtol * scale + atol
    print(f"  grad {name}: max err {e / max(scale, 1e-30):.3g} of scale {scale:.3g}")
    if not e <= tol:
        return [f"grad {name}: max abs err {e:.3g} > tol {tol:.3g} (scale {scale:.3g})"]
    return []


def grad_rel_err(d, dref, rows=None):
    """max |d - d_ref| over `rows` / max |d_ref| over all rows."""
    d = np.asarray(d, np.float64).reshape(np.shape(dref))
    dref = np.asarray(dref, np.float64)
    scale = max(float(np.max(np.abs(dref))) if dref.size else 0.0, 1e-30)
    if rows is not None:
        d, dref = d[rows], dref[rows]
    return max_err(d, dref) / scale


def flipped_pixels(out, ref, edge, img_tol=1e-5, alpha_tol=1e-6):
    """[H,W] bool: knife-edge pixels (`edge`) whose image or alpha differ by
    more than rounding -- a decision there went the other way."""
    img = np.abs(np.asarray(out["image"], np.float64) - np.asarray(ref["image"], np.float64)).max(0) > img_tol
    alp = (np.abs(np.asarray(out["alpha"], np.float64) - np.asarray(ref["alpha"], np.float64)) > alpha_tol)[0]
    return np.asarray(edge, bool) & (img | alp)


def touching_gaussians(means2d, conics, vis, pixels, s_max=23.1 * 1.01):
    """[N] bool: visible Gaussians whose blend footprint (s = d^T Q d <=
    s_max, the :336 skip with a 1 % margin) covers any of `pixels` [(y, x)]."""
    mu = np.asarray(means2d, np.float64)
    q = np.asarray(conics, np.float64).reshape(-1, 4)
    hit = np.zeros(len(mu), bool)
    for y, x in pixels:
        dx, dy = x - mu[:, 0], y - mu[:, 1]
        s = dx * dx * q[:, 0] + dx * dy * (q[:, 1] + q[:, 2]) + dy * dy * q[:, 3]
        hit |= ~(s > s_max)  # (NaN counts as touching)
    return hit & np.asarray(vis, bool)
