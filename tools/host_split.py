"""Where the host time of a small-config bench step goes: wall time per step
of zero_grad / render / backward / Adam, and inside them the time spent in
the library's C calls (gs_render_forward holds the frame's one read-back
wait).  No profiler: perf_counter around each part, and the library's
functions wrapped by a timing proxy of _native.load().
usage: python tools/host_split.py [gaussians width height steps]"""
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


class _Timed:
    def __init__(self, lib, acc):
        self._lib, self._acc, self._cache = lib, acc, {}

    def __getattr__(self, name):
        f = self._cache.get(name)
        if f is None:
            raw = getattr(self._lib, name)
            if not name.startswith("gs_") or not callable(raw):
                return raw
            acc = self._acc

            def f(*a, _raw=raw, _n=name):
                t0 = time.perf_counter()
                try:
                    return _raw(*a)
                finally:
                    acc[_n] += time.perf_counter() - t0
            self._cache[name] = f
        return f


def main():
    n, w, h, k = (int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (5000, 256, 256, 500)))
    pkg = ge.load_package()
    N = pkg._native
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
    from stubs import Cam
    dev = torch.device("cuda", 0)
    sc = pkg.synthetic.make_scene(n, w, h, seed=0)
    m = pkg.synthetic.to_model(sc, pkg.GaussianModel, dev)
    params = m.grad_parameters()
    opt = pkg.optim.FusedAdam([{"params": [p], "lr": 1e-3} for p in params])
    for p in params:
        opt.set_output(p, torch.empty_like(p))
    cam, settings = Cam(w, h, sc.fovx, sc.fovy), pkg.RenderSettings(h, w, torch.zeros(3))
    r = pkg.GaussianRenderer()
    g = torch.Generator().manual_seed(1)
    cot = [(torch.rand(s, generator=g) * 2 - 1).to(dev) for s in ((3, h, w), (1, h, w), (1, h, w))]
    parts = defaultdict(float)

    def step(timed):
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        t1 = time.perf_counter()
        out = r.render(cam, m, settings)
        t2 = time.perf_counter()
        torch.autograd.backward([out["image"], out["alpha"], out["depth"]], cot)
        t3 = time.perf_counter()
        opt.step()
        t4 = time.perf_counter()
        if timed:
            parts["zero_grad"] += t1 - t0
            parts["render"] += t2 - t1
            parts["backward"] += t3 - t2
            parts["adam"] += t4 - t3

    for _ in range(50):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        step(False)
    torch.cuda.synchronize()
    plain = (time.perf_counter() - t0) / k
    lib = N.load()
    acc = defaultdict(float)
    proxy = _Timed(lib, acc)
    N.load = lambda: proxy
    # the rasterizer's own Python around the library calls (the rest of
    # "render" / "backward" is torch: autograd Function dispatch, the engine)
    RZ = pkg.rasterizer
    for fn in ("forward_pipeline", "backward_pipeline", "rasterize"):
        raw = getattr(RZ, fn)

        def timed(*a, _raw=raw, _n=fn, **k):
            t0 = time.perf_counter()
            try:
                return _raw(*a, **k)
            finally:
                parts["py " + _n] += time.perf_counter() - t0
        setattr(RZ, fn, timed)
    import importlib
    importlib.import_module(pkg.__name__ + ".renderer").rasterize = RZ.rasterize
    parts.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        step(True)
    torch.cuda.synchronize()
    timed = (time.perf_counter() - t0) / k
    us = 1e6 / k
    print(f"{k} steps at {n} Gaussians {w}x{h}: {plain * 1e3:.4f} ms/step plain, {timed * 1e3:.4f} with the "
          f"timing proxy")
    for name, v in parts.items():
        print(f"  {name:10s} {v * us:8.1f} us/step")
    for name, v in sorted(acc.items(), key=lambda x: -x[1]):
        print(f"    C {name:24s} {v * us:8.1f} us/step")


if __name__ == "__main__":
    main()
