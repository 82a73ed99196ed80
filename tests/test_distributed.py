"""Data-parallel grad all-reduce over gloo, world_size 2, CPU."""
import os
import time
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = pkg.GaussianModel()
        m.create_from_random(100, generator=torch.Generator().manual_seed(0))  # identical replicas
        params = m.grad_parameters()
        g = torch.Generator().manual_seed(100 + rank)
        for i, p in enumerate(params):
            if rank == 1 and i == 4:
                p.grad = None  # a rank whose view produced no grad for a param
            else:
                p.grad = torch.randn(p.shape, generator=g)
        local = [None if p.grad is None else p.grad.clone() for p in params]
        red = pkg.distributed.GradAllReduce(params, dist)
        red.all_reduce_mean()
        q.put(_by_value(rank, local, [p.grad.clone() for p in params]))
    finally:
        dist.destroy_process_group()


def _by_value(rank, local, reduced):
    """Queue payload as numpy copies: torch tensors would travel as shared-memory
    handles that vanish when the worker exits before the parent has read them."""
    npy = lambda ts: [None if t is None else t.detach().numpy().copy() for t in ts]
    return rank, npy(local), npy(reduced)


def _from_value(ts):
    return [None if a is None else torch.from_numpy(a) for a in ts]


@pytest.mark.parametrize("world", [2, 3])
def test_grad_all_reduce_mean_gloo(world):
    """The mean over the ranks (world 3: a mean that is not a power-of-two
    scaling); a rank with no grad for a parameter counts as zeros."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(world):
        r, local, reduced = q.get(timeout=120)
        res[r] = (_from_value(local), _from_value(reduced))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i in range(5):
        loc = [res[r][0][i] for r in range(world)]
        ref = next(t for t in loc if t is not None)
        exp = sum((t if t is not None else torch.zeros_like(ref)).double() for t in loc) / world
        assert torch.allclose(res[0][1][i].double(), exp, atol=1e-6)
        for r in range(1, world):
            assert torch.equal(res[0][1][i], res[r][1][i])  # replicas stay identical


def _worker_zero_copy(rank, world, port, q, ranges=None):
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = pkg.GaussianModel()
        m.create_from_random(50, generator=torch.Generator().manual_seed(0))
        params = m.grad_parameters()
        red = pkg.distributed.GradAllReduce(params, dist).attach(m)
        assert m._gs_grad_sink is red
        # what the render backward does: write into the bucket views, which
        # autograd then adopts as the .grad tensors
        dest = red.grad_destinations(params)
        assert dest is not None and [d.shape for d in dest] == [p.shape for p in params]
        g = torch.Generator().manual_seed(200 + rank)
        for p, d in zip(params, dest):
            d.copy_(torch.randn(p.shape, generator=g))
            p.grad = d
        local = [p.grad.clone() for p in params]
        ptrs = [p.grad.data_ptr() for p in params]
        assert red.grad_destinations(params) is None  # a .grad exists: the kernels need fresh buffers
        for lo, hi in ranges or ():
            red.rows_ready(lo, hi)  # what the chunked backward does after each range
        red.all_reduce_mean()
        assert [p.grad.data_ptr() for p in params] == ptrs  # reduced in place, no copies
        q.put(_by_value(rank, local, [p.grad.clone() for p in params]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ranges", [None, [(0, 17), (17, 34), (34, 50)]])
def test_grad_all_reduce_zero_copy_gloo(ranges):
    """The backward writes into the bucket (GradAllReduce.attach): the mean is
    formed in place and the .grad tensors stay views of the bucket -- also
    when the backward hands over row ranges as they finish (rows_ready: one
    asynchronous all-reduce per parameter slice, waited for in all_reduce_mean)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_zero_copy, args=(r, 2, port, q, ranges)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(2):
        r, local, reduced = q.get(timeout=120)
        res[r] = (_from_value(local), _from_value(reduced))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i in range(len(res[0][0])):
        exp = (res[0][0][i] + res[1][0][i]) / 2
        assert torch.allclose(res[0][1][i], exp, atol=1e-6)
        assert torch.equal(res[0][1][i], res[1][1][i])


class _ElementwiseOpt:
    """CPU stand-in for FusedAdam's interface (step / step_ranges): an
    elementwise update p -= lr * g * (1 + g^2), so that a range-wise run and a
    whole run are comparable bit for bit, as Adam's are."""

    def __init__(self, params, lr=0.1):
        self.params, self.lr = params, lr

    @torch.no_grad()
    def _rows(self, lo=None, hi=None):
        for p in self.params:
            if p.grad is None:
                continue
            g = p.grad if lo is None else p.grad[lo:hi]
            t = p if lo is None else p[lo:hi]
            t -= self.lr * g * (1 + g * g)

    def step(self):
        self._rows()

    def step_ranges(self, ranges, before=None):
        for k, (lo, hi) in enumerate(ranges):
            if before is not None:
                before(k)
            self._rows(lo, hi)


def _worker_pipelined(rank, world, port, q, ranges):
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        results = []
        for rr in (None, ranges):  # unpipelined, then pipelined, from the same start
            m = pkg.GaussianModel()
            m.create_from_random(60, generator=torch.Generator().manual_seed(0))
            params = m.grad_parameters()
            red = pkg.distributed.GradAllReduce(params, dist).attach(m)
            opt = _ElementwiseOpt(params)
            for it in range(2):
                dest = red.grad_destinations(params)
                g = torch.Generator().manual_seed(300 + 10 * rank + it)
                for p, d in zip(params, dest):
                    d.copy_(torch.randn(p.shape, generator=g))
                    p.grad = d
                for lo, hi in rr or ():
                    red.rows_ready(lo, hi)
                red.reduce_and_step(opt)
                for p in params:
                    p.grad = None
            results.append([p.detach().clone() for p in params])
        q.put(_by_value(rank, results[0], results[1]))
    finally:
        dist.destroy_process_group()


def test_reduce_and_step_pipelined_equals_unpipelined_gloo():
    """GradAllReduce.reduce_and_step: with the rows handed over in ranges,
    range k's update runs after range k's all-reduce only (step_ranges);
    the parameters equal the one-reduction, one-step run bit for bit, on both
    ranks (gloo, world size 2, two steps)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ranges = [(0, 13), (13, 40), (40, 60)]
    procs = [ctx.Process(target=_worker_pipelined, args=(r, 2, port, q, ranges)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(2):
        r, whole, piped = q.get(timeout=120)
        res[r] = (_from_value(whole), _from_value(piped))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        for a, b in zip(*res[r]):
            assert torch.equal(a, b)
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)  # replicas identical


def test_covers_needs_every_bucket_parameter():
    """rows_ready is only attached when the render writes every bucket
    parameter (advisor, round 2): a parameter outside the render's leaves
    (features_rest with sh_degree 0) would otherwise be reduced from
    uninitialised bucket memory."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__ as ge
    pkg = ge.load_package()
    m = pkg.GaussianModel()
    m.create_from_random(10, generator=torch.Generator().manual_seed(0))
    params = m.grad_parameters()

    class _D:  # a process group stand-in: covers() needs no collective
        @staticmethod
        def is_initialized():
            return False
    red = pkg.distributed.GradAllReduce(params, _D())
    assert red.covers(list(params))
    assert not red.covers(list(params)[:-1])
    assert not red.covers(list(params) + [m._features_rest])


def _worker_native_decision(rank, world, port, q, fail):
    """Drive distributed._native_comm over gloo with a fake communicator
    (rccl.RcclComm's construction steps overridden) that fails step `fail`
    (load / uid / init / check / import) on rank 1 only, or never."""
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import importlib
        rccl = importlib.import_module(pkg.__name__ + ".rccl")
        RcclComm, RcclError = rccl.RcclComm, rccl.RcclError
        calls = []

        class Fake(RcclComm):
            def _load(self):
                calls.append("load")
                if fail == "load" and self.rank == 1:
                    raise OSError("librccl.so: cannot open shared object file")

            def _get_unique_id(self, uid):
                calls.append("uid")
                if fail == "uid":
                    raise RcclError("ncclGetUniqueId: unhandled system error (2)")
                uid.internal = b"fake-id"

            def _init_comm(self, uid):
                calls.append("init")
                assert uid.internal.startswith(b"fake-id")  # rank 0's id reached every rank
                if fail == "init" and self.rank == 1:
                    raise RcclError("ncclCommInitRank: invalid usage (5)")
                if fail == "init_hang" and self.rank == 1:
                    import threading
                    threading.Event().wait()  # (never returns: a rank stuck in the bootstrap)
                self.nranks = self.world

            def _self_check(self):
                calls.append("check")
                if fail == "check" and self.rank == 1:
                    raise RcclError("self-check mean off by 0.5 (relative)")
                self.self_check = 0.0

        factory = Fake
        rccl.INIT_TIMEOUT_S = 3.0  # (the hang case: both ranks must be back well within the test's limit)
        t0 = time.monotonic()
        if fail == "import" and rank == 1:
            # this rank cannot import the native module: the real _native_comm path
            sys.modules[pkg.__name__ + ".rccl"] = None
            factory = None
        comm = pkg.distributed._native_comm(dist, None, factory=factory, device=torch.device("cpu"))
        st = dict(pkg.distributed.native_status())
        # the process group still works and every rank issues the same collectives
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t)
        pkg.distributed.close_native_comms()
        q.put((rank, comm is not None, st, calls, float(t), time.monotonic() - t0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail", [None, "load", "uid", "init", "init_hang", "check", "import"])
def test_native_comm_decided_by_all_ranks_gloo(fail):
    """Round-3 review item 3 / advisor: the native-RCCL choice is collective.
    Whichever construction step fails on one rank (library load, rank 0's
    unique id, communicator init, the self-check collective, the module
    import), both ranks fall back to torch.distributed together, at the same
    step, with the reason recorded -- no rank hangs in a broadcast and no mix
    of transports; with no failure both take the native path and record the
    communicator's rank count."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_native_decision, args=(r, 2, port, q, fail)) for r in range(2)]
    for p in procs:
        p.start()
    res, took = {}, {}
    for _ in range(2):
        r, native, st, calls, tsum, dt = q.get(timeout=120)
        res[r], took[r] = (native, st, calls, tsum), dt
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0] == (fail is None)
    for r in (0, 1):
        native, st, calls, tsum = res[r]
        assert tsum == 3.0
        assert st["native"] == (fail is None)
        if fail is None:
            assert st["rccl_nranks"] == 2 and st["fallback_reason"] is None
        else:
            assert st["rccl_nranks"] is None and st["fallback_reason"]
    # both ranks stop after the same step (rank 0 alone makes the unique id)
    done = {None: ["load", "init", "check"], "load": ["load"], "uid": ["load"], "init": ["load", "init"],
            "init_hang": ["load", "init"], "check": ["load", "init", "check"]}
    if fail in done:
        for r in (0, 1):
            assert [c for c in res[r][2] if c != "uid"] == done[fail]
        assert res[0][2].count("uid") == (0 if fail == "load" else 1) and "uid" not in res[1][2]
    if fail == "load":
        assert "another rank" in res[0][1]["fallback_reason"] and "librccl" in res[1][1]["fallback_reason"]
    if fail == "check":
        assert "another rank" in res[0][1]["fallback_reason"] and "self-check" in res[1][1]["fallback_reason"]
    if fail == "uid":
        assert "ncclGetUniqueId" in res[0][1]["fallback_reason"] and "rank 0" in res[1][1]["fallback_reason"]
    if fail == "import":
        assert "import rccl" in res[1][1]["fallback_reason"] and "another rank" in res[0][1]["fallback_reason"]
    if fail == "init_hang":
        # a rank stuck in ncclCommInitRank reports failure
        # after INIT_TIMEOUT_S (3 s here); both ranks fall back, neither hangs
        assert "did not return within 3 s on rank 1" in res[1][1]["fallback_reason"]
        assert "another rank" in res[0][1]["fallback_reason"]
        assert max(took.values()) < 30.0


def test_self_check_wait_is_bounded():
    """A collective that never completes fails the self-check after the
    timeout (RcclError, so every rank falls back) instead of hanging the job;
    a completed one returns, and an event error is reported as such."""
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    import importlib
    pkg = ge.load_package()
    rccl = importlib.import_module(pkg.__name__ + ".rccl")

    class Hip:
        def __init__(self, codes):
            self.codes = list(codes)

        def hipEventQuery(self, ev):
            return self.codes.pop(0) if len(self.codes) > 1 else self.codes[0]

    comm = object.__new__(rccl.RcclComm)
    comm._done = [None]
    comm._hip = Hip([rccl.HIP_ERROR_NOT_READY])
    t0 = time.monotonic()
    with pytest.raises(rccl.RcclError, match="did not complete"):
        comm.wait_done(0, 0.05)
    assert time.monotonic() - t0 < 5.0
    comm._hip = Hip([rccl.HIP_ERROR_NOT_READY, rccl.HIP_ERROR_NOT_READY, 0])
    comm.wait_done(0, 5.0)
    comm._hip = Hip([rccl.HIP_ERROR_NOT_READY, 719])
    with pytest.raises(rccl.RcclError, match="hipError 719"):
        comm.wait_done(0, 5.0)
