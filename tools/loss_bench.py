"""Fused loss (gs_loss_forward + gs_loss_backward) timing and output dump,
for a bitwise A/B of two library builds (GPU tool).

    GS_LIB_PATH=ab/loss_old.so python tools/loss_bench.py gpurun_out/loss_a.npz
    python tools/loss_bench.py gpurun_out/loss_b.npz
    python tools/bitcmp.py cmp gpurun_out/loss_a.npz gpurun_out/loss_b.npz

Per shape: loss values and the gradient for seeded pred/target, and the
mean wall time of forward + backward over 20 iterations (run it under
rocprofv3 --kernel-trace --stats for the kernel times alone).  An optional
second argument keeps only the shapes containing it (e.g. 1080)."""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = [((3, 800, 800), 11), ((3, 1080, 1920), 11), ((3, 37, 53), 11), ((3, 64, 48), 7), ((2, 33, 17), 3),
         ((1, 5, 7), 11), ((3, 40, 40), 1)]


def main(out, only=""):
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    dev = torch.device("cuda", 0)
    res = {}
    for shape, K in CASES:
        if only and only not in "x".join(map(str, shape)):
            continue
        g = torch.Generator().manual_seed(sum(shape) + K)
        p = torch.rand(shape, generator=g)
        t = (p + 0.1 * torch.randn(shape, generator=g)).clamp(0, 1)
        p, t = p.to(dev), t.to(dev)

        def run():
            q = p.clone().requires_grad_()
            tot, l1, ds = pkg.loss.photometric_loss(q, t, 0.2, K)
            tot.backward()
            return tot, l1, ds, q.grad

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            r = run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 20 * 1e3
        tag = "x".join(map(str, shape)) + f"_k{K}"
        for name, v in zip(("total", "l1", "dssim", "grad"), r):
            res[f"{tag}_{name}"] = v.detach().float().cpu().numpy()
        print(f"{tag}: {ms:.3f} ms fwd+bwd (wall)  total={r[0].item():.7f}", flush=True)
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
