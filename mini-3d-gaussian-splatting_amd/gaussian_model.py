"""GaussianModel with the reference's parameter layout and accessors
(src/core/gaussian_model.py:15-128, 200-216).

Parameters, activations, get_* accessors, covariance, random init, and
densification (reference :130-197) as one GPU
compaction pass (gs_densify_count / gs_densify_emit) that also remaps the
optimizer's Adam moments.

Fixes relative to the reference, each a reference bug the render path trips
over: get_covariance works (the reference calls a missing
`self._get_rotation`, :127); there is no config dependency.
"""
from __future__ import annotations

import math
from typing import Optional

import ctypes as C

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as N


def build_rotation_matrix(q: torch.Tensor) -> torch.Tensor:
    """q=[w,x,y,z] -> R (math_utils.py:10-26)."""
    q = F.normalize(q, dim=-1)
    w, x, y, z = q.unbind(-1)
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y),
    ], dim=-1)
    return R.view(-1, 3, 3)


class GaussianModel(nn.Module):
    # The renderer builds Sigma from _scaling/_rotation inside the projection
    # kernel when it sees this flag (see renderer.py).
    _gs_fused_covariance = True

    def __init__(self, config=None, max_sh_degree: int = 3):
        super().__init__()
        self.config = config
        self.max_sh_degree = max_sh_degree
        # SH degree the renderer evaluates (RenderSettings.sh_degree=None reads
        # it).  0 = the reference's DC-only colour; raised by oneup_sh_degree().
        self.active_sh_degree = 0
        self._xyz = nn.Parameter(torch.empty(0, 3))
        self._features_dc = nn.Parameter(torch.empty(0, 1, 3))
        self._features_rest = nn.Parameter(torch.empty(0, 15, 3))
        self._scaling = nn.Parameter(torch.empty(0, 3))
        self._rotation = nn.Parameter(torch.empty(0, 4))
        self._opacity = nn.Parameter(torch.empty(0, 1))
        self.register_buffer("xyz_gradient_accum", torch.zeros(0, 3))
        self.register_buffer("denom", torch.zeros(0, 1))
        self.register_buffer("max_radii2D", torch.zeros(0))
        self.scaling_activation = torch.exp
        self.scaling_inverse_activation = torch.log
        self.opacity_activation = torch.sigmoid
        self.rotation_activation = F.normalize

    def oneup_sh_degree(self) -> None:
        """Raise the rendered SH degree by one, up to max_sh_degree."""
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    # -- init -------------------------------------------------------------
    def _set(self, xyz, fdc, frest, scaling, rot, opacity):
        self._xyz = nn.Parameter(xyz.contiguous())
        self._features_dc = nn.Parameter(fdc.contiguous())
        self._features_rest = nn.Parameter(frest.contiguous())
        self._scaling = nn.Parameter(scaling.contiguous())
        self._rotation = nn.Parameter(rot.contiguous())
        self._opacity = nn.Parameter(opacity.contiguous())
        n, dev = xyz.shape[0], xyz.device
        self.xyz_gradient_accum = torch.zeros(n, 3, device=dev)
        self.denom = torch.zeros(n, 1, device=dev)
        self.max_radii2D = torch.zeros(n, device=dev)

    @torch.no_grad()
    def create_from_random(self, num_points: int, scene_extent: float = 1.0,
                           device=None, generator: Optional[torch.Generator] = None) -> None:
        """gaussian_model.py:78-98"""
        dev = device if device is not None else self._xyz.device
        kw = dict(generator=generator)
        xyz = (torch.rand(num_points, 3, **kw) - 0.5) * (2.0 * scene_extent)
        fdc = torch.rand(num_points, 1, 3, **kw)
        frest = torch.zeros(num_points, 15, 3)
        scaling = torch.full((num_points, 3), math.log(0.02 * scene_extent))
        rot = F.normalize(torch.randn(num_points, 4, **kw), dim=-1)
        opacity = torch.full((num_points, 1), -2.0)
        self._set(*(t.to(dev) for t in (xyz, fdc, frest, scaling, rot, opacity)))

    @torch.no_grad()
    def create_from_points(self, points: torch.Tensor, colors: Optional[torch.Tensor] = None,
                           spatial_lr_scale: float = 1.0) -> None:
        """create_from_pcd (gaussian_model.py:42-76) from in-memory points."""
        points = torch.as_tensor(points, dtype=torch.float32)
        n, dev = points.shape[0], points.device
        if n == 0:
            raise ValueError("No points given.")
        colors = torch.ones(n, 3, device=dev) if colors is None else torch.as_tensor(colors, dtype=torch.float32)
        extent = (points.max(0).values - points.min(0).values).mean().item()
        base = 0.01 * max(extent, 1e-2) * spatial_lr_scale
        self._set(points, colors[:, None, :], torch.zeros(n, 15, 3, device=dev),
                  torch.full((n, 3), math.log(base), device=dev),
                  F.normalize(torch.randn(n, 4, device=dev), dim=-1), torch.full((n, 1), 0.5, device=dev))

    @torch.no_grad()
    def create_from_pcd(self, pcd_path: str, spatial_lr_scale: float = 1.0, device=None) -> None:
        """gaussian_model.py:42-76: initialise from a point-cloud file (the
        formats of dataset.load_point_cloud; the reference's own loader call,
        IOUtils.load_pcd, does not exist)."""
        from .dataset import load_point_cloud
        pts, cols = load_point_cloud(pcd_path)
        if pts.shape[0] == 0:
            raise ValueError("No points found in the PCD file.")
        dev = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.create_from_points(torch.from_numpy(pts).to(dev),
                                None if cols is None else torch.from_numpy(cols).to(dev), spatial_lr_scale)

    # -- accessors (gaussian_model.py:101-128) ------------------------------
    @property
    def get_xyz(self) -> torch.Tensor:
        return self._xyz

    @property
    def get_features(self) -> torch.Tensor:
        if self._features_rest.numel() == 0:
            return self._features_dc
        return torch.cat([self._features_dc, self._features_rest], dim=1)

    @property
    def get_scaling(self) -> torch.Tensor:
        return self.scaling_activation(self._scaling)

    @property
    def get_rotation(self) -> torch.Tensor:
        return self.rotation_activation(self._rotation)

    @property
    def get_opacity(self) -> torch.Tensor:
        return self.opacity_activation(self._opacity)

    @property
    def get_covariance(self) -> torch.Tensor:
        return self.compute_3d_covariance()

    def compute_3d_covariance(self) -> torch.Tensor:
        """R diag(sigma^2) R^T (gaussian_model.py:200-207)"""
        sigma = self.get_scaling
        R = build_rotation_matrix(self.get_rotation)
        return R @ torch.diag_embed(sigma ** 2) @ R.transpose(-1, -2)

    def get_num_points(self) -> int:
        return int(self._xyz.shape[0])

    @torch.no_grad()
    def reset_opacity(self, new_opacity: float = 0.01) -> None:
        val = torch.clamp(torch.tensor(new_opacity, device=self._opacity.device), 1e-4, 1 - 1e-4)
        self._opacity.data[:] = self.inverse_sigmoid(val)

    @staticmethod
    def inverse_sigmoid(x):
        return torch.log(x / (1 - x))

    def grad_parameters(self):
        """Parameters that receive a render gradient (features_rest only while
        SH colour is on, active_sh_degree > 0)."""
        ps = [self._xyz, self._features_dc, self._scaling, self._rotation, self._opacity]
        if self.active_sh_degree > 0:
            ps.insert(2, self._features_rest)
        return ps

    def parameter_list(self):
        """The six parameters in gs_model_arrays order."""
        return [self._xyz, self._features_dc, self._features_rest, self._scaling, self._rotation, self._opacity]

    def get_parameters(self):
        """The parameter list the reference's optimizer asks for
        (optimizer.py:71, `gaussians.get_parameters()`)."""
        return self.parameter_list()

    # -- densification (gaussian_model.py:130-197, optimizer.py:34-67) --------
    @torch.no_grad()
    def densify_and_prune(self, grad_threshold: float, scene_extent: float, min_opacity: float = 0.01,
                          optimizer: Optional[torch.optim.Optimizer] = None, seed: Optional[int] = None,
                          split: bool = True, clone: bool = True, prune: bool = True,
                          xyz_grad: Optional[torch.Tensor] = None) -> dict:
        """Split large / clone small high-gradient Gaussians, then drop those
        with opacity <= min_opacity, in one GPU pass (semantics in
        include/gsplat_mi355x.h, "Densification").  With `optimizer`, its
        Adam moments follow the Gaussians (new ones start at zero) and its
        parameter references are replaced.  Returns the output counts."""
        params = self.parameter_list()
        n, dev = self.get_num_points(), self._xyz.device
        grad = xyz_grad if xyz_grad is not None else self._xyz.grad
        for p in params:
            if not (p.is_cuda and p.is_contiguous()):
                raise RuntimeError("densify needs contiguous parameters on a HIP device")
        if seed is None:
            self._densify_calls = getattr(self, "_densify_calls", 0) + 1
            seed = 0x5EED0000 + self._densify_calls
        lib = N.load()
        rest = int(self._features_rest[0].numel()) if n else 0
        flags = (N.GS_DENSIFY_SPLIT if split else 0) | (N.GS_DENSIFY_CLONE if clone else 0) | \
                (N.GS_DENSIFY_PRUNE if prune else 0)
        states = [optimizer.state.get(p, {}) if optimizer is not None else {} for p in params]

        def arrays(ts):
            return N.GsModelArrays(*[N.ptr(t) for t in ts])

        ws = torch.empty((max(int(lib.gs_densify_workspace_bytes(n)), 4),), dtype=torch.uint8, device=dev)
        counters = torch.zeros((4,), dtype=torch.int32, device=dev)
        g = None if grad is None else grad.detach().float().contiguous()
        a = N.GsDensifyArgs()
        a.n, a.rest_floats, a.in_ = n, rest, arrays(params)
        a.xyz_grad = N.ptr(g)
        a.grad_threshold, a.scene_extent = float(grad_threshold), float(scene_extent)
        a.split_size, a.clone_size, a.min_opacity = 0.03, 0.01, float(min_opacity)
        a.flags, a.seed = flags, int(seed) & 0xFFFFFFFFFFFFFFFF
        a.adam_m_in = arrays([st.get("exp_avg") for st in states])
        a.adam_v_in = arrays([st.get("exp_avg_sq") for st in states])
        a.workspace, a.workspace_bytes, a.counters = N.ptr(ws), ws.numel(), N.ptr(counters)
        stream = N.stream_ptr()
        N.check(lib.gs_densify_count(C.byref(a), stream), "gs_densify_count")
        kept, nsplit, ncl, n_out = (int(v) for v in counters.tolist())
        outs = [torch.empty((n_out,) + tuple(p.shape[1:]), dtype=p.dtype, device=dev) for p in params]
        m_out = [torch.empty_like(o) if "exp_avg" in st else None for o, st in zip(outs, states)]
        v_out = [torch.empty_like(o) if "exp_avg_sq" in st else None for o, st in zip(outs, states)]
        a.out, a.adam_m_out, a.adam_v_out = arrays(outs), arrays(m_out), arrays(v_out)
        N.check(lib.gs_densify_emit(C.byref(a), stream), "gs_densify_emit")
        new = [nn.Parameter(o) for o in outs]
        if optimizer is not None:
            remap = {id(p): (q, st, m, v) for p, q, st, m, v in zip(params, new, states, m_out, v_out)}
            for group in optimizer.param_groups:
                group["params"] = [remap[id(p)][0] if id(p) in remap else p for p in group["params"]]
            for p in params:
                if p in optimizer.state:
                    del optimizer.state[p]
            for p, q, st, m, v in zip(params, new, states, m_out, v_out):
                if st:
                    nst = dict(st)
                    if m is not None:
                        nst["exp_avg"] = m
                    if v is not None:
                        nst["exp_avg_sq"] = v
                    optimizer.state[q] = nst
        (self._xyz, self._features_dc, self._features_rest, self._scaling, self._rotation,
         self._opacity) = new
        self.xyz_gradient_accum = torch.zeros(n_out, 3, device=dev)
        self.denom = torch.zeros(n_out, 1, device=dev)
        self.max_radii2D = torch.zeros(n_out, device=dev)
        return {"kept": kept, "split": nsplit, "cloned": ncl, "n": n_out}

    def density_and_split(self, grad_threshold: float, scene_extent: float) -> None:
        """gaussian_model.py:131-157 (split only, no opacity prune)."""
        self.densify_and_prune(grad_threshold, scene_extent, split=True, clone=False, prune=False)

    def density_and_clone(self, grad_threshold: float, scene_extent: float) -> None:
        """gaussian_model.py:160-178 (clone only, no opacity prune)."""
        self.densify_and_prune(grad_threshold, scene_extent, split=False, clone=True, prune=False)

    @torch.no_grad()
    def prune_points(self, mask: torch.Tensor) -> None:
        """gaussian_model.py:181-197: keep the Gaussians where mask is True."""
        (self._xyz, self._features_dc, self._features_rest, self._scaling, self._rotation,
         self._opacity) = [nn.Parameter(p.data[mask].contiguous()) for p in self.parameter_list()]
        n, dev = self.get_num_points(), self._xyz.device
        self.xyz_gradient_accum = torch.zeros(n, 3, device=dev)
        self.denom = torch.zeros(n, 1, device=dev)
        self.max_radii2D = torch.zeros(n, device=dev)
