"""FusedAdam: torch.optim.Adam semantics, one HIP launch for up to 8 tensors.

The reference builds torch.optim.Adam over five parameter groups
(src/core/optimizer.py:100-113); torch's fused Adam then launches once per
group.  This optimizer keeps the same per-group hyper-parameters and state
layout ('step', 'exp_avg', 'exp_avg_sq' per parameter) but updates every
tensor in a single gs_adam_step launch.
Parameters without .grad are skipped, as torch does.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _native as N


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        batches = {}
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.is_contiguous()):
                    raise RuntimeError("FusedAdam needs contiguous fp32 HIP tensors")
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                t = st["step"]
                d = N.GsAdamTensor(N.ptr(p), N.ptr(st["exp_avg"]), N.ptr(st["exp_avg_sq"]), N.ptr(p.grad),
                                   p.numel(), float(group["lr"]), 1.0 - b1 ** t, (1.0 - b2 ** t) ** 0.5)
                batches.setdefault((float(b1), float(b2), float(group["eps"])), []).append(d)
        lib = N.load()
        stream = torch.cuda.current_stream().cuda_stream
        for (b1, b2, eps), ds in batches.items():
            for i in range(0, len(ds), N.GS_ADAM_MAX_TENSORS):
                chunk = ds[i:i + N.GS_ADAM_MAX_TENSORS]
                a = N.GsAdamArgs()
                a.num_tensors, a.beta1, a.beta2, a.eps = len(chunk), b1, b2, eps
                for k, d in enumerate(chunk):
                    a.t[k] = d
                N.check(lib.gs_adam_step(C.byref(a), stream), "gs_adam_step")
        return loss
