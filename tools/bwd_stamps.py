"""Per-wave phase timing of the blend backward (debug build with s_memtime
stamps).  usage: GS_LIB_PATH=<stamps build> python tools/bwd_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from stubs import Cam
    dev = torch.device("cuda", 0)
    W, H = 1920, 1080
    sc = pkg.synthetic.make_scene(1_000_000, W, H, seed=0)
    m = pkg.synthetic.to_model(sc, pkg.GaussianModel, dev)
    g = torch.Generator().manual_seed(1)
    cot = [(torch.rand(s, generator=g) * 2 - 1).to(dev) for s in ((3, H, W), (1, H, W), (1, H, W))]
    for _ in range(3):
        for p in m.grad_parameters():
            p.grad = None
        out = pkg.GaussianRenderer().render(Cam(W, H, sc.fovx, sc.fovy), m, pkg.RenderSettings(H, W, torch.zeros(3)))
        torch.autograd.backward([out["image"], out["alpha"], out["depth"]], cot)
    torch.cuda.synchronize()
    lib = pkg._native.load()
    n = 8192 * 4 * 6
    buf = (C.c_ulonglong * n)()
    assert lib.gs_debug_stamps(buf, C.c_size_t(n)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 4, 6)[:120 * 68].astype(np.float64)
    nb = (a[..., 5].astype(np.uint64) >> np.uint64(40)).astype(np.float64)
    a[..., 5] = (a[..., 5].astype(np.uint64) & np.uint64((1 << 40) - 1)).astype(np.float64)
    names = ["prologue", "phaseA", "waitX", "phaseB+stage", "waitY", "epilogue"]
    tot = a.sum(axis=(0, 1))
    print("cycles summed over all waves (fraction):")
    for k, v in zip(names, tot):
        print(f"  {k:14s} {v:.4g}  ({v / tot.sum():.3f})")
    per_wave = a.sum(axis=2)
    print("per-wave total cycles: mean %.4g  max %.4g" % (per_wave.mean(), per_wave.max()))
    print("batches per tile: mean %.1f max %d" % (nb[:, 0].mean(), nb[:, 0].max()))
    print("per batch (mean over waves): phaseA %.0f waitX %.0f phaseB %.0f waitY %.0f cycles" %
          tuple(a[..., k].sum() / max(nb.sum(), 1) for k in (1, 2, 3, 4)))


if __name__ == "__main__":
    main()
