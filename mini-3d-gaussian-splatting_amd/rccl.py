"""Native RCCL for the gradient bucket's all-reduces.

torch.distributed issues an all-reduce at 22 us of host time, a coalesced
group of the five parameter slices of a Gaussian range at 59 us, and a CUDA
event record at 9 us (measured on the box, tools/coll_host_cost.py); with the
bucket reduced in several ranges that host time, not the GPU, set the pace
of the step's tail.  This module drives RCCL directly through ctypes -- the
same librccl torch loaded (one RCCL in the process) -- on a communicator of
its own over the process group's ranks:

  * one non-blocking HIP stream for the collectives;
  * per range k: an event recorded on the compute stream right after the
    range's gradient kernels, the collective stream waits for it (so range
    k's reduction overlaps the kernels queued after it), ncclGroupStart /
    ncclAllReduce per slice (ncclAvg: the mean formed inside the reduction) /
    ncclGroupEnd, and a "done" event the consumer (Adam for range k) makes the
    compute stream wait for.

The unique id travels through the torch process group once (a 128-byte
broadcast).  Every rank issues the same ranges in the same order, as
collectives must match.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Sequence, Tuple

import torch

from . import _native

NCCL_FLOAT32 = 7
NCCL_SUM, NCCL_AVG = 0, 4
HIP_EVENT_DISABLE_TIMING = 0x2


class _UniqueId(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


_LIBS = None


def _libs():
    """(librccl, libamdhip64): the instances torch already loaded."""
    global _LIBS
    if _LIBS is None:
        tl = os.path.join(os.path.dirname(torch.__file__), "lib")
        p = os.path.join(tl, "librccl.so")
        rccl = C.CDLL(p if os.path.exists(p) else "librccl.so.1")
        p = os.path.join(tl, "libamdhip64.so")
        hip = C.CDLL(p if os.path.exists(p) else "libamdhip64.so.7")
        vp = C.c_void_p
        rccl.ncclGetUniqueId.argtypes = [C.POINTER(_UniqueId)]
        rccl.ncclCommInitRank.argtypes = [C.POINTER(vp), C.c_int, _UniqueId, C.c_int]
        rccl.ncclAllReduce.argtypes = [vp, vp, C.c_size_t, C.c_int, C.c_int, vp, vp]
        rccl.ncclGroupStart.argtypes = []
        rccl.ncclGroupEnd.argtypes = []
        rccl.ncclCommDestroy.argtypes = [vp]
        rccl.ncclGetErrorString.argtypes = [C.c_int]
        rccl.ncclGetErrorString.restype = C.c_char_p
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclGroupStart", "ncclGroupEnd",
                  "ncclCommDestroy"):
            getattr(rccl, f).restype = C.c_int
        hip.hipEventCreateWithFlags.argtypes = [C.POINTER(vp), C.c_uint]
        hip.hipEventRecord.argtypes = [vp, vp]
        hip.hipStreamWaitEvent.argtypes = [vp, vp, C.c_uint]
        hip.hipEventDestroy.argtypes = [vp]
        for f in ("hipEventCreateWithFlags", "hipEventRecord", "hipStreamWaitEvent", "hipEventDestroy"):
            getattr(hip, f).restype = C.c_int
        _LIBS = (rccl, hip)
    return _LIBS


class RcclError(RuntimeError):
    pass


def _check_nccl(rccl, r: int, what: str):
    if r != 0:
        raise RcclError(f"{what}: {rccl.ncclGetErrorString(r).decode(errors='replace')} ({r})")


def _check_hip(r: int, what: str):
    if r != 0:
        raise RcclError(f"{what}: hipError {r}")


class RcclComm:
    """An RCCL communicator over the ranks of `group` (torch process group of
    backend "nccl"), with its own collective stream and per-range events."""

    def __init__(self, dist, group=None, device=None):
        rccl, hip = _libs()
        self._rccl, self._hip = rccl, hip
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        uid = _UniqueId()
        if self.rank == 0:
            _check_nccl(rccl, rccl.ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")
        buf = torch.frombuffer(bytearray(C.string_at(C.addressof(uid), 128)), dtype=torch.uint8).to(self.device)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(buf, src=src, group=group)
        C.memmove(C.addressof(uid), bytes(buf.cpu().numpy().tobytes()), 128)
        self._comm = C.c_void_p()
        _check_nccl(rccl, rccl.ncclCommInitRank(C.byref(self._comm), self.world, uid, self.rank), "ncclCommInitRank")
        self._stream = torch.cuda.Stream(device=self.device)
        self._ready: List[C.c_void_p] = []
        self._done: List[C.c_void_p] = []

    def _events(self, k: int):
        while len(self._ready) <= k:
            for lst in (self._ready, self._done):
                ev = C.c_void_p()
                _check_hip(self._hip.hipEventCreateWithFlags(C.byref(ev), HIP_EVENT_DISABLE_TIMING), "hipEventCreate")
                lst.append(ev)
        return self._ready[k], self._done[k]

    def all_reduce(self, k: int, pieces: Sequence[Tuple[int, int]], avg: bool = True) -> None:
        """Reduce (sum, or mean with avg) the fp32 buffers `pieces` [(device
        pointer, element count)] in place, as range k: after everything
        queued so far on the current stream, on the collective stream."""
        rccl, hip = self._rccl, self._hip
        ready, done = self._events(k)
        comp = C.c_void_p(_native.stream_ptr(self.device))
        coll = C.c_void_p(self._stream.cuda_stream)
        _check_hip(hip.hipEventRecord(ready, comp), "hipEventRecord")
        _check_hip(hip.hipStreamWaitEvent(coll, ready, 0), "hipStreamWaitEvent")
        op = NCCL_AVG if avg else NCCL_SUM
        group = len(pieces) > 1
        if group:
            _check_nccl(rccl, rccl.ncclGroupStart(), "ncclGroupStart")
        try:
            for ptr, count in pieces:
                if count > 0:
                    _check_nccl(rccl, rccl.ncclAllReduce(ptr, ptr, count, NCCL_FLOAT32, op, self._comm, coll),
                                "ncclAllReduce")
        finally:
            if group:
                _check_nccl(rccl, rccl.ncclGroupEnd(), "ncclGroupEnd")
        _check_hip(hip.hipEventRecord(done, coll), "hipEventRecord")

    def wait(self, k: int) -> None:
        """The current stream waits for range k's collective (host does not block)."""
        comp = C.c_void_p(_native.stream_ptr(self.device))
        _check_hip(self._hip.hipStreamWaitEvent(comp, self._done[k], 0), "hipStreamWaitEvent")

    def close(self) -> None:
        if self._comm:
            torch.cuda.synchronize(self.device)
            self._rccl.ncclCommDestroy(self._comm)
            self._comm = C.c_void_p()
        for ev in self._ready + self._done:
            self._hip.hipEventDestroy(ev)
        self._ready, self._done = [], []
