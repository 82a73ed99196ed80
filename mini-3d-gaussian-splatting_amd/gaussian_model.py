"""GaussianModel with the reference's parameter layout and accessors
(src/core/gaussian_model.py:15-128, 200-216).

Only what the render path reads is here: parameters, activations,
get_* accessors, covariance, random init.  Densification (reference
:130-197) is a "next" row of SURVEY.md section 8(f) and is not part of this
round's scope.

Fixes relative to the reference, each a reference bug the render path trips
over: get_covariance works (the reference calls a missing
`self._get_rotation`, :127); there is no config dependency.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


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
        """Parameters that receive a render gradient (features_rest does not)."""
        return [self._xyz, self._features_dc, self._scaling, self._rotation, self._opacity]
