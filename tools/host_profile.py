"""Host-side profile of the bench step (render + backward + fused Adam) at a
small config, where the step is bound by host work rather than by kernels:
cProfile over K steps, top functions by own time.
usage: python tools/host_profile.py [gaussians width height steps]"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    n, w, h, k = (int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (5000, 256, 256, 500)))
    pkg = ge.load_package()
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
    from stubs import Cam
    dev = torch.device("cuda", 0)
    sc = pkg.synthetic.make_scene(n, w, h, seed=0)
    m = pkg.synthetic.to_model(sc, pkg.GaussianModel, dev)
    params = m.grad_parameters()
    opt = pkg.optim.FusedAdam([{"params": [p], "lr": 1e-3} for p in params])
    cam, settings = Cam(w, h, sc.fovx, sc.fovy), pkg.RenderSettings(h, w, torch.zeros(3))
    r = pkg.GaussianRenderer()
    g = torch.Generator().manual_seed(1)
    cot = [(torch.rand(s, generator=g) * 2 - 1).to(dev) for s in ((3, h, w), (1, h, w), (1, h, w))]

    def step():
        opt.zero_grad(set_to_none=True)
        out = r.render(cam, m, settings)
        torch.autograd.backward([out["image"], out["alpha"], out["depth"]], cot)
        opt.step()

    for _ in range(50):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        step()
    torch.cuda.synchronize()
    print(f"{k} steps at {n} Gaussians {w}x{h}: {(time.perf_counter() - t0) / k * 1e3:.3f} ms each (no profiler)")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(k):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
