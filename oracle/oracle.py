"""ctypes wrapper around liboracle (gs_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the parity checker / CPU baseline.  The
product renderer (mini-3d-gaussian-splatting_amd) never imports this module.

The functions mirror /root/reference/src/core/renderer.py:31-367 (forward)
and its autograd backward; see gs_oracle.c for the restatement notes.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libgs_oracle.so")
_lib = None

_fp = C.POINTER(C.c_float)


class _Scene(C.Structure):
    _fields_ = [
        ("N", C.c_int), ("W", C.c_int), ("H", C.c_int), ("tile", C.c_int),
        ("cam_w", C.c_int), ("cam_h", C.c_int),
        ("fovx", C.c_double), ("fovy", C.c_double),
        ("wv", _fp), ("radius_min", C.c_float), ("radius_max", C.c_float),
        ("bg", _fp), ("xyz", _fp), ("cov3d", _fp), ("color_logits", _fp),
        ("opacity", _fp), ("force_neval", C.POINTER(C.c_int32)),
    ]


class _FwdOut(C.Structure):
    _fields_ = [
        ("means2d", _fp), ("cov2d", _fp), ("conics", _fp), ("depths", _fp),
        ("radii", _fp), ("vis", C.POINTER(C.c_uint8)),
        ("sorted_idx", C.POINTER(C.c_int32)), ("M", C.c_int32),
        ("image", _fp), ("alpha", _fp), ("depth", _fp),
        ("T", C.c_int64), ("E", C.c_int64), ("C", C.c_int64), ("margin", _fp),
    ]


class _BwdIO(C.Structure):
    _fields_ = [
        ("g_image", _fp), ("g_alpha", _fp), ("g_depth", _fp),
        ("g_means2d", _fp), ("g_conics", _fp),
        ("d_xyz", _fp), ("d_cov3d", _fp), ("d_color_logits", _fp),
        ("d_opacity", _fp), ("d_means2d", _fp), ("d_conics", _fp),
    ]


def build() -> str:
    """Compile liboracle with the committed Makefile (gcc is in the image)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "gs_oracle.c"))
        ):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _lib.gso_forward.argtypes = [C.POINTER(_Scene), C.POINTER(_FwdOut), C.c_int]
        _lib.gso_backward.argtypes = [C.POINTER(_Scene), C.POINTER(_FwdOut), C.POINTER(_BwdIO), C.c_int]
        _lib.gso_covariance.argtypes = [C.c_int, _fp, _fp, _fp]
        _lib.gso_covariance_bwd.argtypes = [C.c_int, _fp, _fp, _fp, _fp, _fp]
    return _lib


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _p(a: Optional[np.ndarray]):
    if a is None:
        return C.cast(None, _fp)
    return a.ctypes.data_as(_fp)


@dataclass
class Scene:
    """Inputs of one render() call, in the reference's duck-typed terms."""
    xyz: np.ndarray            # [N,3]  get_xyz
    cov3d: np.ndarray          # [N,3,3] get_covariance
    color_logits: np.ndarray   # [N,3]  get_features[:,0,:]
    opacity: np.ndarray        # [N]    get_opacity.squeeze(1)
    wv: np.ndarray             # [4,4]  camera.world_view_transform()
    width: int
    height: int
    fovx: float
    fovy: float
    bg: np.ndarray             # [3]
    cam_width: Optional[int] = None   # camera._width (defaults to width)
    cam_height: Optional[int] = None  # camera._height (defaults to height)
    tile: int = 16
    radius_min: float = 0.01
    radius_max: float = 50.0
    # [H,W] int32 or None: decision-forced replay -- pixel p evaluates exactly
    # its first force_neval[p] list entries, with no termination test of its
    # own (another renderer's per-pixel n_eval; gs_oracle.c gso_scene)
    force_neval: Optional[np.ndarray] = None


def _scene_struct(s: Scene, keep: list) -> _Scene:
    arrs = dict(
        wv=_f32(s.wv).reshape(16), bg=_f32(s.bg).reshape(3), xyz=_f32(s.xyz).reshape(-1, 3),
        cov3d=_f32(s.cov3d).reshape(-1, 9), color_logits=_f32(s.color_logits).reshape(-1, 3),
        opacity=_f32(s.opacity).reshape(-1),
    )
    fn = None
    if s.force_neval is not None:
        fn = np.ascontiguousarray(np.asarray(s.force_neval, dtype=np.int32).reshape(int(s.height), int(s.width)))
        arrs["force_neval"] = fn
    keep.append(arrs)
    n = arrs["xyz"].shape[0]
    cw = int(s.width if s.cam_width is None else s.cam_width)
    ch = int(s.height if s.cam_height is None else s.cam_height)
    return _Scene(n, int(s.width), int(s.height), int(s.tile), cw, ch, float(s.fovx), float(s.fovy),
                  _p(arrs["wv"]), float(s.radius_min), float(s.radius_max), _p(arrs["bg"]),
                  _p(arrs["xyz"]), _p(arrs["cov3d"]), _p(arrs["color_logits"]), _p(arrs["opacity"]),
                  C.cast(None, C.POINTER(C.c_int32)) if fn is None else fn.ctypes.data_as(C.POINTER(C.c_int32)))


def _alloc_fwd(n: int, h: int, w: int, margins: bool = False):
    o = dict(
        means2d=np.zeros((n, 2), np.float32), cov2d=np.zeros((n, 2, 2), np.float32),
        conics=np.zeros((n, 2, 2), np.float32), depths=np.zeros(n, np.float32),
        radii=np.zeros(n, np.float32), vis=np.zeros(n, np.uint8),
        sorted_idx=np.zeros(max(n, 1), np.int32), image=np.zeros((3, h, w), np.float32),
        alpha=np.zeros((1, h, w), np.float32), depth=np.zeros((1, h, w), np.float32),
    )
    st = _FwdOut(_p(o["means2d"]), _p(o["cov2d"]), _p(o["conics"]), _p(o["depths"]),
                 _p(o["radii"]), o["vis"].ctypes.data_as(C.POINTER(C.c_uint8)),
                 o["sorted_idx"].ctypes.data_as(C.POINTER(C.c_int32)), 0,
                 _p(o["image"]), _p(o["alpha"]), _p(o["depth"]), 0, 0, 0, C.cast(None, _fp))
    if margins:
        o["margin"] = np.zeros((2, h, w), np.float32)
        st.margin = _p(o["margin"])
    return o, st


def _finish_fwd(o: dict, st: _FwdOut) -> Dict[str, np.ndarray]:
    o["vis"] = o["vis"].astype(bool)
    o["sorted_idx"] = o["sorted_idx"][: st.M].copy()
    o["M"], o["T"], o["E"], o["C"] = int(st.M), int(st.T), int(st.E), int(st.C)
    return o


def render_forward(s: Scene, nthreads: int = 0, margins: bool = False) -> Dict[str, np.ndarray]:
    """Forward of renderer.py:31-114; returns numpy arrays + work counters.
    margins: also `margin` [2,H,W], each pixel's distance (ulps) to the w < 1e-5
    skip and the A >= 0.995 break (gs_oracle.c, gso_fwd_out.margin)."""
    keep: list = []
    sc = _scene_struct(s, keep)
    o, st = _alloc_fwd(sc.N, s.height, s.width, margins)
    rc = lib().gso_forward(C.byref(sc), C.byref(st), int(nthreads))
    if rc:
        raise RuntimeError(f"gso_forward failed ({rc})")
    return _finish_fwd(o, st)


def render_backward(s: Scene, g_image, g_alpha, g_depth, g_means2d=None, g_conics=None,
                    nthreads: int = 0, margins: bool = False) -> Dict[str, np.ndarray]:
    """Gradients of L = <g_image,image> + <g_alpha,alpha> + <g_depth,depth>
    (+ <g_means2d,viewspace_points> + <g_conics,conics>) w.r.t. the inputs."""
    keep: list = []
    sc = _scene_struct(s, keep)
    n, h, w = sc.N, s.height, s.width
    o, st = _alloc_fwd(n, h, w, margins)
    gi, ga, gd = _f32(g_image).reshape(3, h, w), _f32(g_alpha).reshape(h, w), _f32(g_depth).reshape(h, w)
    gm = None if g_means2d is None else _f32(g_means2d).reshape(n, 2)
    gc = None if g_conics is None else _f32(g_conics).reshape(n, 4)
    d = dict(xyz=np.zeros((n, 3), np.float32), cov3d=np.zeros((n, 3, 3), np.float32),
             color_logits=np.zeros((n, 3), np.float32), opacity=np.zeros(n, np.float32),
             means2d=np.zeros((n, 2), np.float32), conics=np.zeros((n, 2, 2), np.float32))
    io = _BwdIO(_p(gi), _p(ga), _p(gd), _p(gm), _p(gc), _p(d["xyz"]), _p(d["cov3d"]),
                _p(d["color_logits"]), _p(d["opacity"]), _p(d["means2d"]), _p(d["conics"]))
    rc = lib().gso_backward(C.byref(sc), C.byref(st), C.byref(io), int(nthreads))
    if rc:
        raise RuntimeError(f"gso_backward failed ({rc})")
    out = _finish_fwd(o, st)
    out["grads"] = d
    return out


def covariance(scaling, rotation) -> np.ndarray:
    """GaussianModel.compute_3d_covariance (gaussian_model.py:200-207)."""
    s, r = _f32(scaling).reshape(-1, 3), _f32(rotation).reshape(-1, 4)
    out = np.zeros((s.shape[0], 3, 3), np.float32)
    lib().gso_covariance(s.shape[0], _p(s), _p(r), _p(out))
    return out


def covariance_backward(scaling, rotation, dcov):
    s, r = _f32(scaling).reshape(-1, 3), _f32(rotation).reshape(-1, 4)
    g = _f32(dcov).reshape(-1, 9)
    ds = np.zeros_like(s)
    dr = np.zeros_like(r)
    lib().gso_covariance_bwd(s.shape[0], _p(s), _p(r), _p(g), _p(ds), _p(dr))
    return ds, dr
