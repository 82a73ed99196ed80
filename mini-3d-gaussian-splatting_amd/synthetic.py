"""Synthetic scenes of SURVEY.md 8(d) (the benchmark / parity workload).

Generated on the CPU with a seeded torch.Generator, then copied to the
device, so the GPU path and the CPU oracle see bit-identical inputs.
  camera: identity W2C, FoVx = 60 deg, FoVy = 2 atan(tan(30 deg) H/W)
  z ~ U[2,6], x ~ U[-1,1] z tan(FoVx/2), y ~ U[-1,1] z tan(FoVy/2)
  sigma per axis log-uniform in [0.002, 0.01] -> _scaling = log sigma
  _rotation = normalize(randn(4)), _opacity ~ N(0,1) (sigmoid applied),
  _features_dc ~ U[0,1], _features_rest = 0
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch


@dataclass
class SyntheticScene:
    xyz: torch.Tensor       # [N,3]
    scaling: torch.Tensor   # [N,3] raw (log sigma)
    rotation: torch.Tensor  # [N,4] raw quaternion
    features_dc: torch.Tensor  # [N,1,3]
    opacity: torch.Tensor   # [N,1] raw logit
    width: int
    height: int
    fovx: float
    fovy: float


def fov_pair(width: int, height: int, fovx_deg: float = 60.0):
    fx = math.radians(fovx_deg)
    return fx, 2.0 * math.atan(math.tan(fx / 2) * height / width)


def make_scene(n: int, width: int, height: int, seed: int = 0, sigma_range=(0.002, 0.01),
               z_range=(2.0, 6.0)) -> SyntheticScene:
    g = torch.Generator().manual_seed(seed)
    fx, fy = fov_pair(width, height)
    z = torch.rand(n, generator=g) * (z_range[1] - z_range[0]) + z_range[0]
    x = (torch.rand(n, generator=g) * 2 - 1) * z * math.tan(fx / 2)
    y = (torch.rand(n, generator=g) * 2 - 1) * z * math.tan(fy / 2)
    lo, hi = math.log(sigma_range[0]), math.log(sigma_range[1])
    scaling = torch.rand(n, 3, generator=g) * (hi - lo) + lo
    rot = torch.randn(n, 4, generator=g)
    rot = rot / rot.norm(dim=1, keepdim=True)
    opacity = torch.randn(n, 1, generator=g)
    fdc = torch.rand(n, 1, 3, generator=g)
    return SyntheticScene(torch.stack([x, y, z], 1), scaling, rot, fdc, opacity, width, height, fx, fy)


def to_model(scene: SyntheticScene, model_cls, device):
    m = model_cls()
    n = scene.xyz.shape[0]
    m._set(scene.xyz.to(device), scene.features_dc.to(device), torch.zeros(n, 15, 3, device=device),
           scene.scaling.to(device), scene.rotation.to(device), scene.opacity.to(device))
    return m
