"""Data-parallel training over views: one view per GPU, one all-reduce.

SURVEY.md 8(e): each rank renders its own camera with a full replica of the
GaussianModel; the only exchange per step is the mean of the Gaussian
parameter gradients, done as ONE flat all_reduce(SUM) / world over
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X, "gloo" on CPU
for tests), issued after the last backward kernel and before
optimizer.step().  Payload: xyz 3 + features_dc 3 + scaling 3 + rotation 4 +
opacity 1 = 14 fp32 (56 B) per Gaussian; features_rest has an identically
zero render gradient and is not sent unless SH colour is on
(GaussianModel.grad_parameters: +45 fp32 per Gaussian then).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch


class GradAllReduce:
    """Mean-all-reduce of `params`' .grad through one flat bucket.

    The bucket is allocated once (re-allocated only if the parameter count
    changes, e.g. after densification) and reused every step.  A missing
    .grad counts as zeros, so ranks whose view saw none of a parameter still
    take part in the collective.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], dist=None, group=None):
        if dist is None:
            import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.params: List[torch.nn.Parameter] = list(params)
        self._flat: Optional[torch.Tensor] = None
        self._sizes: List[int] = []

    def _bucket(self) -> torch.Tensor:
        sizes = [p.numel() for p in self.params]
        if self._flat is None or sizes != self._sizes or self._flat.device != self.params[0].device:
            self._sizes = sizes
            self._flat = torch.empty(sum(sizes), dtype=torch.float32, device=self.params[0].device)
        return self._flat

    def all_reduce_mean(self) -> None:
        flat = self._bucket()
        views = torch.split(flat, self._sizes)
        for p, v in zip(self.params, views):
            if p.grad is None:
                v.zero_()
            else:
                v.copy_(p.grad.reshape(-1))
        world = self.dist.get_world_size(self.group)
        self.dist.all_reduce(flat, op=self.dist.ReduceOp.SUM, group=self.group)
        flat.div_(world)
        for p, v in zip(self.params, views):
            if p.grad is None:
                p.grad = v.view_as(p).clone()
            else:
                p.grad.copy_(v.view_as(p))
