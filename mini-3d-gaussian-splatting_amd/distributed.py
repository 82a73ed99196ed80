"""Data-parallel training over views: one view per GPU, one gradient mean.

SURVEY.md 8(e): each rank renders its own camera with a full replica of the
GaussianModel; the only exchange per step is the mean of the Gaussian
parameter gradients before the optimizer step.  Payload: xyz 3 + features_dc
3 + scaling 3 + rotation 4 + opacity 1 = 14 fp32 (56 B) per Gaussian, one
flat bucket; features_rest has an identically zero render gradient and is not
sent unless SH colour is on (GaussianModel.grad_parameters: +45 fp32 then).

Transport: backend "nccl" (= RCCL over xGMI on MI355X) goes to RCCL directly
(rccl.RcclComm: a communicator of its own, its own HIP stream, ncclAvg, per
range an event pair), because torch.distributed's per-call host time (22 us
an all-reduce, 59 us a coalesced group, 9 us an event) set the pace of the
step's tail; GS_DP_NATIVE=0 keeps torch.distributed.  gloo (CPU tests) sums,
then divides by the world size.

Pipelining: with the bucket attached (zero copy), the render backward runs
its last stage (gradient gather + projection backward) in `chunks` ranges of
Gaussians and hands each finished range to rows_ready(), which issues its
reduction asynchronously (the collective stream waits for that range's
kernels only); reduce_and_step() then queues the Adam update of range k
behind range k's reduction only (FusedAdam.step_ranges), so range k's
reduction overlaps the gather / projection backward of the ranges after it
and the Adam updates of the ranges before it.  Every rank issues the same
ranges in the same order (same N, same chunk rule), as collectives must
match.  Default: 4 ranges above one rank, 1 at world size 1
(GS_ALLREDUCE_CHUNKS overrides); the result is bit-identical for every range
count (an elementwise update of the same reduced values).
"""
from __future__ import annotations

import os
import time
from typing import Iterable, List, Optional

import torch


_NATIVE_COMMS: dict = {}
NATIVE_STATUS: dict = {}  # key -> {"native", "rccl_nranks", "self_check_err", "fallback_reason"}
_ATEXIT = False


def _agreement(dist, group, device):
    """agree(ok) -> the logical AND of `ok` over the group's ranks (one int32
    MIN all-reduce through torch.distributed on `device`)."""
    def agree(ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        return bool(int(t.item()))
    return agree


def _comm_key(dist, group, device) -> tuple:
    """The (process group, device) key of _NATIVE_COMMS / NATIVE_STATUS."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    return (id(group if group is not None else dist.group.WORLD), str(device))


def _native_comm(dist, group, factory=None, device=None):
    """The process group's RcclComm on the current device, or None -- decided
    by all ranks together (rccl.RcclComm: every construction step that can
    fail on some ranks only is followed by an all-ranks agreement, so either
    every rank drives RCCL natively or every rank falls back to
    torch.distributed; never a mix, whose collectives would not match).
    Created once per (group, device), on every rank at the same point (the
    first GradAllReduce is built at the same iteration everywhere).  The
    outcome is kept in NATIVE_STATUS for the bench line.  `factory` and
    `device` are for tests (a fake communicator over gloo on the CPU)."""
    global _ATEXIT
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = _comm_key(dist, group, device)
    if key not in _NATIVE_COMMS:
        coll_dev = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
        agree = _agreement(dist, group, coll_dev)
        comm, reason = None, None
        if factory is None:
            try:
                from .rccl import RcclComm as factory
            except Exception as e:  # noqa: BLE001 -- this rank cannot; tell the others at step 1
                reason = f"import rccl: {e}"
                agree(False)
        if factory is not None:
            try:
                comm = factory(dist, group, device=device, agree=agree, coll_device=coll_dev)
            except Exception as e:  # noqa: BLE001 -- raised on every rank at the same step
                reason = str(e)
        if comm is None:
            import warnings
            warnings.warn(f"native RCCL not used ({reason}); gradient all-reduce through torch.distributed "
                          "on every rank")
        NATIVE_STATUS[key] = {"native": comm is not None,
                              "rccl_nranks": getattr(comm, "nranks", None),
                              "self_check_err": getattr(comm, "self_check", None),
                              "fallback_reason": reason}
        _NATIVE_COMMS[key] = comm
        if comm is not None and not _ATEXIT:
            # left to process-exit teardown, the communicators would go after
            # the HIP runtime; callers that tear down earlier call it themselves
            import atexit
            atexit.register(close_native_comms)
            _ATEXIT = True
    return _NATIVE_COMMS[key]


def native_status(key=None) -> Optional[dict]:
    """The native-communicator decision for `key` (_comm_key(dist, group,
    device)); without a key the most recent one.  None before any."""
    if key is not None:
        return NATIVE_STATUS.get(key)
    return next(reversed(NATIVE_STATUS.values())) if NATIVE_STATUS else None


def close_native_comms() -> None:
    """Destroy the native RCCL communicators (before the process group goes:
    every rank calls it at the same point, after its last collective)."""
    for key, comm in list(_NATIVE_COMMS.items()):
        if comm is not None:
            comm.close()
        del _NATIVE_COMMS[key]


class GradAllReduce:
    """Mean-all-reduce of `params`' .grad through one flat bucket.

    The bucket is allocated once (re-allocated only if the parameter count
    changes, e.g. after densification) and reused every step.  A missing
    .grad counts as zeros, so ranks whose view saw none of a parameter still
    take part in the collective.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], dist=None, group=None, chunks: Optional[int] = None,
                 min_chunk_rows: Optional[int] = None):
        if dist is None:
            import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.params: List[torch.nn.Parameter] = list(params)
        self._flat: Optional[torch.Tensor] = None
        self._sizes: List[int] = []
        # overlap ranges: `chunks` when every range keeps >= min_chunk_rows
        # Gaussians (smaller launches would not fill the GPU)
        # default: 4 ranges above one rank (each range's reduction overlaps the
        # gather / projection backward of the ranges after it, and its Adam
        # update the reductions after it: GradAllReduce.reduce_and_step), 1 at
        # world size 1.  Through native RCCL a range costs ~32 us of host time
        # and ~10 us of GPU time more than one whole-bucket call (world-size-1
        # rehearsal, profiles/r03/dist/); through torch.distributed's coalescing
        # manager it was ~70 us.
        if chunks is None:
            env = os.environ.get("GS_ALLREDUCE_CHUNKS")
            world = dist.get_world_size(group) if (hasattr(dist, "is_initialized") and dist.is_initialized()) else 1
            chunks = int(env) if env else (4 if world > 1 else 1)
        self.chunks = int(chunks)
        self.min_chunk_rows = int(min_chunk_rows if min_chunk_rows is not None
                                  else os.environ.get("GS_ALLREDUCE_MIN_ROWS", 1 << 16))
        self._works: list = []
        # coalesced range reductions (torch's _coalescing_manager): RCCL only
        self._coalesce = (os.environ.get("GS_ALLREDUCE_COALESCE", "1") != "0" and hasattr(dist, "is_initialized")
                          and dist.is_initialized() and dist.get_backend(group) == "nccl")
        self.ranges_reduced = 0  # rows_ready calls so far (diagnostic)
        self.host_s = {"rows_ready": 0.0, "reduce_and_step": 0.0}  # host seconds spent issuing (diagnostic)
        # RCCL (backend "nccl") forms the mean inside the reduction (ReduceOp.AVG,
        # NCCL >= 2.10; this image's RCCL is 2.27); gloo has no AVG: SUM, then one
        # division.  Decided once, here, from the backend: a collective that
        # fails later is an error, never retried with another op (a retry on
        # one rank would issue a collective the others never do).
        self._avg: bool = (dist.is_initialized() and dist.get_backend(group) == "nccl"
                           and hasattr(dist.ReduceOp, "AVG")) if hasattr(dist, "is_initialized") else False
        # backend "nccl": the collectives go to RCCL directly (rccl.RcclComm, one
        # communicator per process group and device, ncclAvg, established and
        # self-checked by all ranks together), unless GS_DP_NATIVE=0
        self._native = None
        self.native_status = {"native": False, "rccl_nranks": None, "self_check_err": None,
                              "fallback_reason": "GS_DP_NATIVE=0" if self._avg else "backend is not nccl"}
        mode = os.environ.get("GS_DP_NATIVE", "1")
        # "force": try native RCCL over any backend's process group (a rehearsal
        # of the establishment protocol, e.g. two gloo ranks on one GPU, where
        # RCCL refuses the duplicate device and every rank must fall back)
        if (self._avg and mode != "0") or (mode == "force" and torch.cuda.is_available()
                                            and hasattr(dist, "is_initialized") and dist.is_initialized()):
            self._native = _native_comm(dist, group)
            # this group's own decision (a cached communicator's, not the
            # newest entry: another group may have been added since)
            self.native_status = dict(native_status(_comm_key(dist, group, None)))
            if self._native is not None:
                self._avg = True  # ncclAvg forms the mean (no division after the reduction)

    def _bucket(self) -> torch.Tensor:
        sizes = [p.numel() for p in self.params]
        if self._flat is None or sizes != self._sizes or self._flat.device != self.params[0].device:
            self._sizes = sizes
            self._flat = torch.empty(sum(sizes), dtype=torch.float32, device=self.params[0].device)
        return self._flat

    # -- zero-copy path ------------------------------------------------------
    def attach(self, model) -> "GradAllReduce":
        """Let `model`'s render backward write its gradients straight into the
        bucket (GaussianRenderer asks grad_destinations at backward time):
        all_reduce_mean then copies nothing in or out -- 2 x 56 B per Gaussian
        of HBM traffic and ten copy launches less per step."""
        model._gs_grad_sink = self
        return self

    def overlap_chunks(self) -> int:
        """How many Gaussian ranges the render backward should hand to
        rows_ready (1: one range, reduced as soon as it is done)."""
        n = self.params[0].shape[0] if self.params else 0
        return max(1, min(self.chunks, n // max(1, self.min_chunk_rows)))

    def rows_ready(self, lo: int, hi: int) -> None:
        """Gradient rows [lo, hi) of every parameter are final in the bucket
        (queued on the current stream): reduce them asynchronously."""
        t0 = time.perf_counter()
        try:
            self._rows_ready(lo, hi)
        finally:
            self.host_s["rows_ready"] += time.perf_counter() - t0

    def _rows_ready(self, lo: int, hi: int) -> None:
        flat = self._bucket()
        n = self.params[0].shape[0]
        op = self.dist.ReduceOp.AVG if self._avg else self.dist.ReduceOp.SUM
        self.ranges_reduced += 1
        if self._native is not None:
            # the range's slice of every parameter (the whole bucket: one piece)
            if lo == 0 and hi == n:
                pieces = [(flat.data_ptr(), flat.numel())]
            else:
                pieces, off = [], 0
                for size in self._sizes:
                    cols = size // n
                    pieces.append((flat.data_ptr() + 4 * (off + lo * cols), (hi - lo) * cols))
                    off += size
            k = len(self._works)
            self._native.all_reduce(k, pieces, avg=True)
            self._works.append((lo, hi, k))
            return
        if lo == 0 and hi == n:  # every row: the whole bucket in one call
            self._works.append((lo, hi, [self.dist.all_reduce(flat, op=op, group=self.group, async_op=True)]))
            return
        # the range's slice of every parameter, coalesced into one collective
        # (one RCCL group launch) where the backend supports it
        slices, off = [], 0
        for size in self._sizes:
            cols = size // n
            slices.append(flat[off + lo * cols: off + hi * cols])
            off += size
        cm_fn = getattr(self.dist, "_coalescing_manager", None)
        if cm_fn is not None and self._coalesce:
            with cm_fn(group=self.group, device=flat.device, async_ops=True) as cm:
                for t in slices:
                    self.dist.all_reduce(t, op=op, group=self.group)
            self._works.append((lo, hi, [cm]))
            return
        self._works.append((lo, hi, [self.dist.all_reduce(t, op=op, group=self.group, async_op=True)
                                     for t in slices]))

    def set_timing(self, on: bool) -> bool:
        """Time each collective on the GPU from now on (True) or stop (False);
        returns whether this bucket can: native RCCL only, whose collective
        stream is this process's own (torch.distributed runs RCCL on streams
        it does not expose, gloo on host threads)."""
        if self._native is None:
            return False
        self._native.collective_ms(reset=True)
        self._native.timing = bool(on)
        return True

    def collective_gpu_ms(self) -> Optional[List[float]]:
        """GPU milliseconds of each collective issued since set_timing(True),
        in issue order (waits for them); None where set_timing cannot time."""
        return self._native.collective_ms(reset=True) if self._native is not None else None

    def covers(self, leaves) -> bool:
        """Do `leaves` write every parameter of the bucket?  Only then may the
        backward hand rows to rows_ready (a parameter no kernel writes would
        be reduced from uninitialised bucket memory)."""
        return {id(t) for t in leaves} == {id(p) for p in self.params}

    def grad_destinations(self, leaves) -> Optional[List[torch.Tensor]]:
        """Bucket views shaped like `leaves`, when every leaf is one of this
        bucket's parameters and none holds a .grad yet (autograd then adopts
        the views as the .grad tensors; onto an existing .grad it would add,
        so the kernels need a buffer of their own).  None otherwise."""
        ids = [id(p) for p in self.params]
        if any(id(t) not in ids or t.grad is not None for t in leaves):
            return None
        views = torch.split(self._bucket(), self._sizes)
        return [views[ids.index(id(t))].view_as(t) for t in leaves]

    @staticmethod
    def _aliases(p, v) -> bool:
        g = p.grad
        return g is not None and g.is_contiguous() and g.numel() == v.numel() and g.data_ptr() == v.data_ptr()

    def all_reduce_mean(self) -> None:
        flat = self._bucket()
        views = torch.split(flat, self._sizes)
        in_place = [self._aliases(p, v) for p, v in zip(self.params, views)]
        if self._works:
            # the backward reduced the bucket range by range (rows_ready)
            for _, _, ws in self._works:
                self._wait(ws)
            self._works = []
            if not self._avg:
                flat.div_(self.dist.get_world_size(self.group))
            return self._copy_out(views, in_place)
        for p, v, ok in zip(self.params, views, in_place):
            if ok:
                continue
            if p.grad is None:
                v.zero_()
            else:
                v.copy_(p.grad.reshape(-1))
        world = self.dist.get_world_size(self.group)
        if self._native is not None:
            self._native.all_reduce(0, [(flat.data_ptr(), flat.numel())], avg=True)
            self._native.wait(0)
            return self._copy_out(views, in_place)
        if self._avg:
            # RCCL divides inside the reduction: no extra pass over the bucket
            self.dist.all_reduce(flat, op=self.dist.ReduceOp.AVG, group=self.group)
        else:
            self.dist.all_reduce(flat, op=self.dist.ReduceOp.SUM, group=self.group)
            flat.div_(world)
        self._copy_out(views, in_place)

    def reduce_and_step(self, optimizer) -> None:
        """all_reduce_mean() then optimizer.step(), pipelined when the
        backward handed its rows over in ranges (rows_ready) and every
        gradient is the bucket itself: range k's Adam update is queued behind
        range k's all-reduce only (FusedAdam.step_ranges), so it overlaps the
        reductions of the later ranges.  Bit-identical to the unpipelined
        sequence (the same reduced values, an elementwise update)."""
        t0 = time.perf_counter()
        try:
            self._reduce_and_step(optimizer)
        finally:
            self.host_s["reduce_and_step"] += time.perf_counter() - t0

    def _reduce_and_step(self, optimizer) -> None:
        flat = self._bucket()
        views = torch.split(flat, self._sizes)
        pipelined = (len(self._works) > 1 and hasattr(optimizer, "step_ranges")
                     and all(self._aliases(p, v) for p, v in zip(self.params, views)))
        if not pipelined:
            self.all_reduce_mean()
            optimizer.step()
            return
        works, self._works = self._works, []
        n = self.params[0].shape[0]
        world = self.dist.get_world_size(self.group)

        def before(k):
            lo, hi, ws = works[k]
            self._wait(ws)  # (RCCL: the current stream waits for this range's collective)
            if not self._avg:
                for v in views:
                    v.view(n, -1)[lo:hi].div_(world)
        optimizer.step_ranges([(lo, hi) for lo, hi, _ in works], before)

    def _wait(self, ws) -> None:
        """Make the current stream wait for one range's collective(s): torch
        Work objects, or the native communicator's range index."""
        if isinstance(ws, int):
            self._native.wait(ws)
            return
        for w in ws:
            w.wait()

    def _copy_out(self, views, in_place) -> None:
        for p, v, ok in zip(self.params, views, in_place):
            if ok:
                continue
            if p.grad is None:
                p.grad = v.view_as(p).clone()
            else:
                p.grad.copy_(v.view_as(p))
