"""Photometric loss of the reference (src/core/loss.py:9-63) on MI355X:
L1 + D-SSIM fused into two HIP kernels (gs_loss_forward / gs_loss_backward,
include/gsplat_mi355x.h).

API mirrors the reference:
  SSIMLoss(window_size=11, size_average=True)(pred, target) -> D-SSIM
  GaussianLoss(lambda_dssim=0.2)(rendered, target) -> (total, {"l1", "dssim", "total_loss"})

The reference SSIMLoss.forward (loss.py:17-39) builds the SSIM map and ends
without a return; its caller uses the value as `dssim` (loss.py:57-58), so it
is defined here as 1 - mean(clamp(SSIM map, 0, 1)) over the reference's own
statistics (K-tap Gaussian window, sigma = K/6, separable, zero padding,
C1 = 0.01^2, C2 = 0.03^2).  Inputs are [C,H,W] or [B,C,H,W] fp32 on the GPU
(B*C planes, averaged together).  There is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Tuple

import torch
from torch import nn

from . import _native as N

_C1, _C2 = 0.01 ** 2, 0.03 ** 2  # loss.py:14-15


def _planes(t: torch.Tensor) -> torch.Tensor:
    if not t.is_cuda:
        raise RuntimeError("the MI355X loss needs tensors on a HIP device; there is no CPU path")
    if t.dim() == 4:
        t = t.reshape(-1, t.shape[-2], t.shape[-1])
    if t.dim() != 3:
        raise ValueError(f"expected [C,H,W] or [B,C,H,W], got {tuple(t.shape)}")
    return t.float().contiguous()


class _FusedPhotometric(torch.autograd.Function):
    """out = [total, l1, dssim]; only `total` carries a gradient (to pred)."""

    @staticmethod
    def forward(ctx, pred, target, lambda_dssim: float, window: int, need_grad: bool):
        lib = N.load()
        Cn, H, W = pred.shape
        dev = pred.device
        ws = torch.empty((int(lib.gs_loss_workspace_bytes(Cn, H, W)),), dtype=torch.uint8, device=dev)
        out = torch.empty((3,), dtype=torch.float32, device=dev)
        maps = torch.empty((3, Cn, H, W), dtype=torch.float32, device=dev) if need_grad else None
        a = N.GsLossArgs(Cn, H, W, N.ptr(pred), N.ptr(target), float(lambda_dssim), int(window), _C1, _C2,
                         N.ptr(ws), ws.numel(), N.ptr(maps), N.ptr(out), None, None)
        N.check(lib.gs_loss_forward(C.byref(a), N.stream_ptr()), "gs_loss_forward")
        ctx.save_for_backward(pred, target, maps)
        ctx.lam, ctx.window = float(lambda_dssim), int(window)
        return out

    @staticmethod
    def backward(ctx, g_out):
        pred, target, maps = ctx.saved_tensors
        if maps is None or g_out is None:
            return None, None, None, None, None
        lib = N.load()
        Cn, H, W = pred.shape
        g_total = g_out[0:1].contiguous()
        d_pred = torch.empty_like(pred)
        a = N.GsLossArgs(Cn, H, W, N.ptr(pred), N.ptr(target), ctx.lam, ctx.window, _C1, _C2,
                         None, 0, N.ptr(maps), None, N.ptr(g_total), N.ptr(d_pred))
        N.check(lib.gs_loss_backward(C.byref(a), N.stream_ptr()), "gs_loss_backward")
        return d_pred, None, None, None, None


def photometric_loss(pred: torch.Tensor, target: torch.Tensor, lambda_dssim: float = 0.2,
                     window_size: int = 11) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(total, l1, dssim) as device scalars, no host sync; total is
    differentiable w.r.t. pred (target is a constant, as in training)."""
    p, t = _planes(pred), _planes(target)
    if p.shape != t.shape:
        raise ValueError(f"pred {tuple(p.shape)} vs target {tuple(t.shape)}")
    out = _FusedPhotometric.apply(p, t.detach(), lambda_dssim, window_size, pred.requires_grad)
    return out[0], out[1].detach(), out[2].detach()


class SSIMLoss(nn.Module):
    """loss.py:9-39; returns D-SSIM = 1 - mean(clamp(SSIM, 0, 1))."""

    def __init__(self, window_size: int = 11, size_average: bool = True):
        super().__init__()
        self.window_size = window_size
        self.size_average = size_average  # (unused by the reference as well: always the mean)
        self.C1, self.C2 = _C1, _C2

    def forward(self, pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        return photometric_loss(pred, target, 1.0, self.window_size)[0]


class GaussianLoss(nn.Module):
    """loss.py:41-63: total = (1 - lambda) L1 + lambda D-SSIM."""

    def __init__(self, lambda_dssim: float = 0.2):
        super().__init__()
        self.lambda_dssim = lambda_dssim
        self.ssim_loss = SSIMLoss()

    def forward(self, rendered: torch.Tensor, target: torch.Tensor) -> Tuple[torch.Tensor, Dict[str, float]]:
        total, l1, dssim = photometric_loss(rendered, target, self.lambda_dssim, self.ssim_loss.window_size)
        vals = torch.stack([l1, dssim, total.detach()]).tolist()  # one host sync (the reference does three)
        return total, {"l1": vals[0], "dssim": vals[1], "total_loss": vals[2]}
