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

Establishing the communicator is a collective decision (every rank takes the
native path, or none does): construction runs four steps -- load the
libraries, make the unique id (rank 0; its status rides on the id's
broadcast), ncclCommInitRank, a self-check collective -- and after each step
that can fail on some ranks only, the ranks all-reduce an "ok" flag over the
torch process group (`agree`).  A step that failed anywhere raises RcclError on
every rank at the same point, so the caller (distributed._native_comm) falls
back to torch.distributed on all ranks together.  The self-check runs the
production call shape -- a grouped ncclAllReduce of two slices at non-zero
offsets with ncclAvg on the collective stream behind an event -- on
rank-dependent integer-valued data, checks the mean on every rank, and checks
ncclCommCount / ncclCommUserRank against the process group.

Bounded in time: ncclCommInitRank (step 3) blocks until
every rank has joined the communicator's bootstrap, so a rank that fails
inside it before joining (a device error on that rank alone, a transport that
never connects) would leave the others blocked in the call, where no
agreement can reach them.  The call therefore runs on a helper thread (with
the rank's device made current there); the rank waits for it at most
INIT_TIMEOUT_S and then joins the agreement either way.  A rank whose init
has not returned by then reports failure, every rank falls back to
torch.distributed at that step, and the stuck thread is abandoned (if its
call ever returns, the thread aborts the communicator it got).  The
self-check collective (step 4) is bounded by SELF_CHECK_TIMEOUT_S.  (A
non-blocking init, ncclCommInitRankConfig with blocking = 0, would make every
later call on the communicator asynchronous -- ncclInProgress -- a mode this
module's call sequence was never run in on more than one GPU.)
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import time
from typing import List, Sequence, Tuple

import torch

from . import _native

NCCL_FLOAT32 = 7
NCCL_SUM, NCCL_AVG = 0, 4
HIP_EVENT_DISABLE_TIMING = 0x2
HIP_ERROR_NOT_READY = 600
# seconds the self-check collective may take (the first collective of a
# communicator also sets up its connections); past it the check fails on this
# rank, and with it the native path on every rank
SELF_CHECK_TIMEOUT_S = float(os.environ.get("GS_RCCL_CHECK_TIMEOUT", "60"))
# seconds ncclCommInitRank may take on its helper thread before this rank
# reports the init failed (every rank then falls back together)
INIT_TIMEOUT_S = float(os.environ.get("GS_RCCL_INIT_TIMEOUT", "60"))


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
        rccl.ncclCommAbort.argtypes = [vp]
        rccl.ncclCommCount.argtypes = [vp, C.POINTER(C.c_int)]
        rccl.ncclCommUserRank.argtypes = [vp, C.POINTER(C.c_int)]
        rccl.ncclGetErrorString.argtypes = [C.c_int]
        rccl.ncclGetErrorString.restype = C.c_char_p
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclGroupStart", "ncclGroupEnd",
                  "ncclCommDestroy", "ncclCommAbort", "ncclCommCount", "ncclCommUserRank"):
            getattr(rccl, f).restype = C.c_int
        hip.hipEventCreateWithFlags.argtypes = [C.POINTER(vp), C.c_uint]
        hip.hipEventRecord.argtypes = [vp, vp]
        hip.hipStreamWaitEvent.argtypes = [vp, vp, C.c_uint]
        hip.hipEventDestroy.argtypes = [vp]
        hip.hipEventQuery.argtypes = [vp]
        hip.hipEventSynchronize.argtypes = [vp]
        hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), vp, vp]
        for f in ("hipEventCreateWithFlags", "hipEventRecord", "hipStreamWaitEvent", "hipEventDestroy",
                  "hipEventQuery", "hipEventSynchronize", "hipEventElapsedTime"):
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


SELF_CHECK_COUNT = 1027  # elements of the self-check buffer (two slices: 600 + 427)


class RcclComm:
    """An RCCL communicator over the ranks of `group` (torch process group of
    backend "nccl"), with its own collective stream and per-range events.

    `agree(ok) -> bool` is the ranks' logical AND of `ok` (an all-reduce over
    the process group, distributed._agreement); without it each rank decides
    alone (world size 1, or tests).  `coll_device` is where the process
    group's collectives take their tensors (cuda for nccl, cpu for gloo).
    Attributes after construction: nranks (ncclCommCount), self_check (the
    largest relative error of the check's mean)."""

    def __init__(self, dist, group=None, device=None, agree=None, coll_device=None):
        agree = agree if agree is not None else (lambda ok: ok)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._coll_device = coll_device if coll_device is not None else self.device
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._comm = C.c_void_p()
        self._ready: List[C.c_void_p] = []
        self._done: List[C.c_void_p] = []
        # collective GPU time (diagnostic, off by default): a timing event pair
        # on the collective stream around each range's ncclGroupStart..End,
        # i.e. the collective's own execution, not its wait for the compute
        # stream's "ready" event (set_timing / collective_ms)
        self.timing = False
        self._tpool: List[Tuple[C.c_void_p, C.c_void_p]] = []
        self._tpairs: List[Tuple[C.c_void_p, C.c_void_p]] = []
        self._stream = None
        self.nranks = None
        self.self_check = None

        def step(what, fn):
            err = None
            try:
                fn()
            except Exception as e:  # noqa: BLE001 -- every failure is decided collectively below
                err = f"{what}: {e}"
            if not agree(err is None):
                self._abort()
                raise RcclError(err or f"{what} failed on another rank")

        # 1. the libraries (and a stream of our own)
        step("load", self._load)
        # 2. the unique id: rank 0 makes it; its status rides on the broadcast
        uid = _UniqueId()
        ok, err0 = 1, None
        if self.rank == 0:
            try:
                self._get_unique_id(uid)
            except Exception as e:  # noqa: BLE001
                ok, err0 = 0, f"ncclGetUniqueId: {e}"
        raw = bytearray(C.string_at(C.addressof(uid), 128)) + bytearray([ok])
        buf = torch.frombuffer(raw, dtype=torch.uint8).to(self._coll_device)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(buf, src=src, group=group)
        got = bytes(buf.cpu().numpy().tobytes())
        if got[128] != 1:
            self._abort()
            raise RcclError(err0 or "ncclGetUniqueId failed on rank 0")
        C.memmove(C.addressof(uid), got[:128], 128)
        # 3. the communicator (bounded in time: a helper thread); 4. the
        # self-check collective (bounded too)
        step("ncclCommInitRank", lambda: self._init_comm_bounded(uid))
        step("self-check", self._self_check)

    # -- construction steps (overridable: tests drive the protocol with fakes) --
    def _load(self) -> None:
        self._rccl, self._hip = _libs()
        self._stream = torch.cuda.Stream(device=self.device)

    def _get_unique_id(self, uid: "_UniqueId") -> None:
        _check_nccl(self._rccl, self._rccl.ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")

    def _init_comm_bounded(self, uid: "_UniqueId") -> None:
        """_init_comm on a helper thread, waited for at most INIT_TIMEOUT_S.
        Past it this rank reports failure (RcclError) and abandons the thread:
        the thread, should its call ever return, aborts the communicator
        itself (under the lock, so exactly one side owns it)."""
        lock, st, done = threading.Lock(), {"finished": False, "abandoned": False, "err": None}, threading.Event()

        def run():
            try:
                if self.device is not None and self.device.type == "cuda":
                    torch.cuda.set_device(self.device)  # (HIP's current device is per thread)
                self._init_comm(uid)
            except BaseException as e:  # noqa: BLE001 -- reported by the waiting thread
                st["err"] = e
            finally:
                with lock:
                    st["finished"] = True
                    abandoned = st["abandoned"]
                if abandoned and self._comm and getattr(self, "_rccl", None) is not None:
                    self._rccl.ncclCommAbort(self._comm)
                    self._comm = C.c_void_p()
                done.set()

        th = threading.Thread(target=run, name=f"rccl-init-rank{self.rank}", daemon=True)
        th.start()
        done.wait(INIT_TIMEOUT_S)
        with lock:
            if not st["finished"]:
                st["abandoned"] = True
        if st["abandoned"]:
            self._init_abandoned = True  # (_abort leaves the communicator to the thread)
            raise RcclError(f"ncclCommInitRank did not return within {INIT_TIMEOUT_S:g} s on rank {self.rank}")
        if st["err"] is not None:
            raise st["err"]

    def _init_comm(self, uid: "_UniqueId") -> None:
        rccl = self._rccl
        _check_nccl(rccl, rccl.ncclCommInitRank(C.byref(self._comm), self.world, uid, self.rank), "ncclCommInitRank")
        cnt, me = C.c_int(-1), C.c_int(-1)
        _check_nccl(rccl, rccl.ncclCommCount(self._comm, C.byref(cnt)), "ncclCommCount")
        _check_nccl(rccl, rccl.ncclCommUserRank(self._comm, C.byref(me)), "ncclCommUserRank")
        if cnt.value != self.world or me.value != self.rank:
            raise RcclError(f"communicator has {cnt.value} ranks (this one {me.value}); "
                            f"the process group {self.world} (this one {self.rank})")
        self.nranks = cnt.value

    def _self_check(self) -> None:
        """The production call shape on known values: x_i = (rank + 1)(i mod 97
        + 1) in two slices, mean-reduced as range 0 behind an event; the mean
        is (world + 1) / 2 (i mod 97 + 1) on every rank (integer sums: exact in
        any order; ncclAvg's scaling by 1 / world rounds once)."""
        n, cut = SELF_CHECK_COUNT, 600
        base = (torch.arange(n, dtype=torch.float32, device=self.device) % 97) + 1
        x = base * float(self.rank + 1)
        ptr = x.data_ptr()
        self.all_reduce(0, [(ptr, cut), (ptr + 4 * cut, n - cut)], avg=True)
        # bounded: a collective that never completes (a first multi-rank run
        # whose transport does not work) fails the check instead of hanging
        # the job; _abort then aborts the communicator (ncclCommAbort)
        self.wait_done(0, SELF_CHECK_TIMEOUT_S)
        self.wait(0)
        torch.cuda.synchronize(self.device)
        want = base * (self.world + 1) / 2.0
        err = float(((x - want).abs() / want).max())
        self.self_check = err
        if not err <= 1e-6:
            raise RcclError(f"self-check mean off by {err:.3g} (relative)")

    def _abort(self) -> None:
        """Drop a half-built communicator without waiting for other ranks."""
        rccl, hip = getattr(self, "_rccl", None), getattr(self, "_hip", None)
        if self._comm and rccl is not None and not getattr(self, "_init_abandoned", False):
            try:
                rccl.ncclCommAbort(self._comm)
            finally:
                self._comm = C.c_void_p()
        if hip is not None:
            for ev in self._ready + self._done + [e for p in self._tpool + self._tpairs for e in p]:
                hip.hipEventDestroy(ev)
        self._ready, self._done, self._tpool, self._tpairs = [], [], [], []

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
        tp = self._timing_pair() if self.timing else None
        if tp is not None:
            _check_hip(hip.hipEventRecord(tp[0], coll), "hipEventRecord")
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
        if tp is not None:
            _check_hip(hip.hipEventRecord(tp[1], coll), "hipEventRecord")
            self._tpairs.append(tp)
        _check_hip(hip.hipEventRecord(done, coll), "hipEventRecord")

    def _timing_pair(self):
        if self._tpool:
            return self._tpool.pop()
        pair = (C.c_void_p(), C.c_void_p())
        for ev in pair:
            _check_hip(self._hip.hipEventCreateWithFlags(C.byref(ev), 0), "hipEventCreate")
        return pair

    def collective_ms(self, reset: bool = True) -> List[float]:
        """GPU milliseconds of each collective issued since the last reset
        while `timing` was on (waits for them), in issue order."""
        out = []
        for t0, t1 in self._tpairs:
            _check_hip(self._hip.hipEventSynchronize(t1), "hipEventSynchronize")
            ms = C.c_float(0.0)
            _check_hip(self._hip.hipEventElapsedTime(C.byref(ms), t0, t1), "hipEventElapsedTime")
            out.append(float(ms.value))
        if reset:
            self._tpool.extend(self._tpairs)
            self._tpairs = []
        return out

    def wait_done(self, k: int, timeout_s: float) -> None:
        """The host waits (polling) for range k's collective, at most timeout_s."""
        deadline = time.monotonic() + timeout_s
        while True:
            r = self._hip.hipEventQuery(self._done[k])
            if r == 0:
                return
            if r != HIP_ERROR_NOT_READY:
                raise RcclError(f"hipEventQuery: hipError {r}")
            if time.monotonic() > deadline:
                raise RcclError(f"collective {k} did not complete within {timeout_s:g} s")
            time.sleep(0.0005)

    def wait(self, k: int) -> None:
        """The current stream waits for range k's collective (host does not block)."""
        comp = C.c_void_p(_native.stream_ptr(self.device))
        _check_hip(self._hip.hipStreamWaitEvent(comp, self._done[k], 0), "hipStreamWaitEvent")

    def close(self) -> None:
        if self._comm:
            torch.cuda.synchronize(self.device)
            self._rccl.ncclCommDestroy(self._comm)
            self._comm = C.c_void_p()
        for ev in self._ready + self._done + [e for p in self._tpool + self._tpairs for e in p]:
            self._hip.hipEventDestroy(ev)
        self._ready, self._done, self._tpool, self._tpairs = [], [], [], []
