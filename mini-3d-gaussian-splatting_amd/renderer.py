"""Drop-in GaussianRenderer / RenderSettings (reference: src/core/renderer.py).

Same class names, constructor arguments, render() signature and output
dict as the reference (renderer.py:13-114).  The four stages run as HIP
kernels (see rasterizer.py); the duck-typed inputs are read exactly where
the reference reads them:

  camera._width/_height/_FoVx/_FoVy, camera.world_view_transform()  (:140-150)
  gaussians.get_xyz (:135), get_covariance (:166), get_features or
  _features_dc (:88-92), get_opacity (:94)

Differences a caller can observe (all documented in DESIGN.md):
  * `world_view_transform` may be a method (what the reference calls) or a
    tensor/property (what the reference's own Camera defines).
  * When `gaussians` is this package's GaussianModel, covariance is built
    inside the projection kernel from the raw `_scaling`/`_rotation` (same
    math as GaussianModel.compute_3d_covariance) and colours are read from
    `_features_dc` instead of materialising get_features; gradients reach the
    same leaves, except `_features_rest`, whose gradient is identically zero
    in the reference and is left as None here.
  * `radii` and `visibility_filter` carry no gradient.
  * `settings.scale_modifier` and `settings.debug` are ignored, as in the
    reference.
  * `settings.sh_degree` (default: the model's `active_sh_degree`, else 0)
    switches on view-dependent SH colour; at 0 -- the default for the
    reference's own model and stubs -- colours are the reference's
    sigmoid(DC).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import _native as N
from .rasterizer import CameraParams, rasterize


@dataclass
class RenderSettings:
    """renderer.py:13-20"""
    image_height: int
    image_width: int
    bg_color: torch.Tensor
    scale_modifier: float = 1.0
    debug: bool = False
    # View-dependent colour (not in the reference, which renders
    # DC only): None takes `gaussians.active_sh_degree` when the model has one,
    # else 0 (the reference's behaviour).  1..3 evaluates SH of that degree from
    # get_features[:, 1:, :] (include/gsplat_mi355x.h, gs_gaussians).
    sh_degree: Optional[int] = None


def _world_view(camera) -> torch.Tensor:
    wv = camera.world_view_transform
    if callable(wv):
        wv = wv()
    return torch.as_tensor(wv)


def effective_tile(tile_size: int, width: int, height: int) -> int:
    """The tile edge the kernels use for GaussianRenderer(tile_size) on a
    width x height image: tile_size, or max(width, height) when it is larger
    -- the same image and gradients, since every tile of at least max(W, H)
    holds the whole image (renderer.py:263-298: one tile, every Gaussian whose
    rectangle meets the image, in depth order).  Edges up to GS_MAX_TILE."""
    t = int(tile_size)
    if t > max(int(width), int(height)):
        t = max(int(width), int(height), 1)
    if t > N.GS_MAX_TILE:
        raise ValueError(f"tile_size {tile_size} on a {width}x{height} image: a tile edge of {t} px (the "
                         f"smaller of tile_size and max(W, H)) is above GS_MAX_TILE = {N.GS_MAX_TILE}, "
                         f"which is not supported")
    return t


def _host_f32(t, count: int) -> list:
    """The values of `t` (a tensor or sequence of `count` numbers) rounded to
    fp32, as Python floats, row-major (a CPU fp32 tensor is read as is)."""
    if not isinstance(t, torch.Tensor) or t.device.type != "cpu" or t.dtype != torch.float32:
        t = torch.as_tensor(t).detach().to("cpu", torch.float32)
    if t.numel() != count:
        raise ValueError(f"expected {count} values, got a tensor of shape {tuple(t.shape)}")
    d = t.dim()
    if d == 1:
        return t.tolist()
    if d == 2:  # (a 4x4 view matrix: tolist and flatten, 1 us instead of reshape + tolist's 3)
        return [v for row in t.tolist() for v in row]
    return t.reshape(count).tolist()


def camera_params(camera, settings: RenderSettings, radius_min=0.01, radius_max=50.0, tile_size=16) -> CameraParams:
    """Host scalars of renderer.py:140-152 (python double -> fp32 in the ABI)."""
    W, H = camera._width, camera._height
    fx = 0.5 * W / math.tan(camera._FoVx * 0.5)
    fy = 0.5 * H / math.tan(camera._FoVy * 0.5)
    view = tuple(_host_f32(_world_view(camera), 16)[:12])
    bg = tuple(_host_f32(settings.bg_color, 3))
    tile = effective_tile(tile_size, settings.image_width, settings.image_height)
    return CameraParams(int(settings.image_width), int(settings.image_height), fx, fy, W * 0.5, H * 0.5,
                        view, bg, float(radius_min), float(radius_max), tile)


class GaussianRenderer:
    """renderer.py:22-114"""

    def __init__(self, tile_size=16, radius_min=0.01, radius_max=50.0):
        # any tile edge the reference's binning can use (renderer.py:261-298):
        # every int >= 1 (0 divides by zero in the reference); edges above
        # the image render as one tile of max(W, H) (effective_tile); radii as
        # the reference clamps them (:190)
        if int(tile_size) != tile_size or tile_size < 1:
            raise ValueError(f"tile_size must be an integer >= 1, got {tile_size!r}")
        if not (math.isfinite(radius_max) and 0 <= radius_min <= radius_max):
            raise ValueError(f"need 0 <= radius_min <= radius_max < inf, got {radius_min!r}, {radius_max!r}")
        self.tile_size = int(tile_size)
        self.radius_min = radius_min
        self.radius_max = radius_max
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")

    def render(self, camera, gaussians, settings: RenderSettings) -> Dict[str, torch.Tensor]:
        cam = camera_params(camera, settings, self.radius_min, self.radius_max, self.tile_size)
        xyz = gaussians.get_xyz
        fused = getattr(gaussians, "_gs_fused_covariance", False)
        if fused:
            # this package's GaussianModel: covariance from the raw scaling /
            # rotation and get_opacity's sigmoid are computed in the kernels;
            # the [N,1,3] / [N,1] leaves go in as they are (no view node on the
            # tape: the rasterizer reads rows by stride and returns gradients
            # in the leaves' shapes)
            cov3d, scaling, rotation = None, gaussians._scaling, gaussians._rotation
            logits = gaussians._features_dc
        else:
            cov3d, scaling, rotation = gaussians.get_covariance, None, None
            feats = gaussians.get_features  # one read: the SH rest below is a view of it
            if feats.dim() == 3 and feats.shape[1] >= 1:
                logits = feats[:, 0, :]
            else:
                logits = gaussians._features_dc.squeeze(1)
        opacity = gaussians._opacity if fused else gaussians.get_opacity.squeeze(1)
        sh_degree = settings.sh_degree
        if sh_degree is None:
            sh_degree = int(getattr(gaussians, "active_sh_degree", 0))
        sh_rest = None
        if sh_degree > 0:
            sh_rest = gaussians._features_rest if fused else feats[:, 1:, :]
        grad_dest = None
        sink = getattr(gaussians, "_gs_grad_sink", None) if fused else None
        if sink is not None:
            # data-parallel bucket (distributed.GradAllReduce.attach): the
            # gradient kernels write straight into it when it can take them
            names = ["xyz", "color", "opacity", "scaling", "rotation"]
            leaves = [gaussians._xyz, gaussians._features_dc, gaussians._opacity, gaussians._scaling,
                      gaussians._rotation]
            if sh_degree > 0:
                names.append("sh_rest")
                leaves.append(gaussians._features_rest)

            def grad_dest():
                views = sink.grad_destinations(leaves)
                if views is None:
                    return None
                d = dict(zip(names, views))
                # reduce finished ranges during the backward -- only when the
                # render writes every row of the bucket: a bucket parameter the
                # render does not reach (e.g. _features_rest with sh_degree 0
                # while the model's active degree is > 0) is filled (zero or
                # its .grad) by all_reduce_mean before its collective instead
                if hasattr(sink, "rows_ready") and getattr(sink, "covers", lambda _: False)(leaves):
                    d["_rows_ready"], d["_chunks"] = sink.rows_ready, sink.overlap_chunks()
                return d
        image, alpha, depth, means2d, conics, radii, vis = rasterize(
            cam, xyz, cov3d, scaling, rotation, logits, opacity, opacity_is_logit=fused,
            sh_rest=sh_rest, sh_degree=sh_degree, grad_dest=grad_dest)
        # the reference's output dtypes (renderer.py:74-83, :273-275, :359-367):
        # the projection outputs in the Gaussians' dtype, image in the
        # background's (out_rgb starts as bg), alpha / depth float32 (zeros of
        # the default dtype).  Computed in fp32 here either way.
        if xyz.dtype == torch.float64:
            means2d, conics, radii = means2d.double(), conics.double(), radii.double()
        if torch.as_tensor(settings.bg_color).dtype == torch.float64:
            image = image.double()
        return {
            "image": image,
            "alpha": alpha,
            "depth": depth,
            "viewspace_points": means2d,
            "visibility_filter": vis,
            "radii": radii,
            "conics": conics,
        }
