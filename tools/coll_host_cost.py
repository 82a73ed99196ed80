"""Host cost of issuing the gradient all-reduce through torch.distributed
(RCCL, world size 1, env:// rendezvous; not product code): per call, for the
whole 56 MB bucket, a coalesced group of five slices, five separate calls, and
Work.wait().  usage: RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29600 \
LOCAL_RANK=0 python tools/coll_host_cost.py"""
import time

import torch
import torch.distributed as dist


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    n = 1_000_000
    flat = torch.zeros(14 * n, device=dev)
    sizes = [3 * n, 3 * n, n, 3 * n, 4 * n]
    views = torch.split(flat, sizes)
    lo, hi = 0, n // 2
    slices = [v.view(n, -1)[lo:hi].reshape(-1) for v in views]
    op = dist.ReduceOp.AVG
    reps = 200

    def timed(label, fn):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"{label:44s} {1e6 * (t1 - t0) / reps:8.1f} us host per call", flush=True)

    timed("all_reduce(bucket, async) + wait", lambda: dist.all_reduce(flat, op=op, async_op=True).wait())
    timed("all_reduce(bucket, async), no wait", lambda: dist.all_reduce(flat, op=op, async_op=True))
    torch.cuda.synchronize()

    def coalesced():
        with dist._coalescing_manager(device=dev, async_ops=True) as cm:
            for t in slices:
                dist.all_reduce(t, op=op)
        return cm
    timed("coalesced 5 slices (async)", coalesced)
    timed("coalesced 5 slices + wait", lambda: coalesced().wait())
    timed("5 separate async slices", lambda: [dist.all_reduce(t, op=op, async_op=True) for t in slices])
    w = dist.all_reduce(flat, op=op, async_op=True)
    timed("Work.wait() (done)", lambda: w.wait())
    e = torch.cuda.Event()
    timed("torch.cuda.Event record", lambda: e.record())
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
