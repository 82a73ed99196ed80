"""GPU densification (gs_densify_count / gs_densify_emit) against a torch
statement of the semantics in include/gsplat_mi355x.h ("Densification"),
which follow gaussian_model.py:131-197 and optimizer.py:64.  The reference's
own densify cannot run (_append_points reads a missing `_scaling_log`,
gaussian_model.py:229), so this row's parity is pinned to that statement."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
M64 = (1 << 64) - 1


def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def normal_of(seed, i, k):
    h = mix64(seed ^ mix64(i * 4 + k))
    u1 = ((h >> 40) + 1) * 2.0 ** -24
    u2 = ((h >> 16) & 0xFFFFFF) * 2.0 ** -24
    return math.sqrt(-2.0 * math.log(u1)) * math.cos(2 * math.pi * u2)


def ref_densify(m, grad, th, extent, min_op, seed, masks=False):
    """The statement; masks=True also returns (keep, split, clone, hot, s, o)
    over the input Gaussians (the trainer parity test remaps Adam moments
    with them and checks no decision sits on a threshold)."""
    xyz, fdc, frest, scl, rot, op = [p.detach().cpu().double() for p in m.parameter_list()]
    g = grad.detach().cpu().double()
    n = xyz.shape[0]
    s = scl.exp().mean(-1)
    hot = g.norm(dim=-1) > th
    split, clone = hot & (s > 0.03 * extent), hot & (s < 0.01 * extent)
    o = torch.sigmoid(op[:, 0])
    alive = o > min_op
    child_op = torch.logit(o).clamp(-6, 6)
    child_alive = torch.sigmoid(child_op) > min_op
    keep, sp, cl = ~split & alive, split & child_alive, clone & alive
    q = F.normalize(rot, dim=-1)
    w, x, y, z = q.unbind(-1)
    d = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y + w * z), 2 * (x * z - w * y)], -1)
    off = d * (s * 0.5)[:, None]
    jit = torch.tensor([[normal_of(seed, i, k) for k in range(3)] for i in range(n)], dtype=torch.float64)
    rows = {
        "xyz": [xyz[keep], (xyz - off)[sp], (xyz + off)[sp], (xyz + jit * (s * 0.5)[:, None])[cl]],
        "fdc": [fdc[keep], fdc[sp], fdc[sp], fdc[cl]],
        "frest": [frest[keep], frest[sp], frest[sp], frest[cl]],
        "scl": [scl[keep], torch.log(scl.exp() * 0.75)[sp], torch.log(scl.exp() * 0.75)[sp], scl[cl]],
        "rot": [rot[keep], q[sp], q[sp], rot[cl]],
        "op": [op[keep], child_op[sp, None], child_op[sp, None], op[cl]],
    }
    out = {k: torch.cat(v) for k, v in rows.items()}, (int(keep.sum()), int(sp.sum()), int(cl.sum()))
    if masks:
        return out + ((keep, sp, cl, hot, s, o),)
    return out


def _model(pkg, cuda, n=6000, seed=4):
    syn = pkg.synthetic
    sc = syn.make_scene(n, 64, 48, seed=seed, sigma_range=(0.002, 0.05))
    g = torch.Generator().manual_seed(seed)
    sc.opacity[:] = torch.randn(n, 1, generator=g) * 3.0  # some below the 0.01 prune line
    m = syn.to_model(sc, pkg.GaussianModel, cuda)
    m._features_rest.data.normal_(generator=None)
    grad = (torch.randn(n, 3, generator=g) * 3e-4).to(cuda)
    return m, grad


def test_densify_matches_statement(pkg, cuda):
    m, grad = _model(pkg, cuda)
    ext = 1.0
    ref, counts = ref_densify(m, grad, 2e-4, ext, 0.01, 77)
    info = m.densify_and_prune(2e-4, ext, 0.01, seed=77, xyz_grad=grad)
    assert (info["kept"], info["split"], info["cloned"]) == counts
    assert counts[1] > 10 and counts[2] > 10 and info["n"] == counts[0] + 2 * counts[1] + counts[2]
    got = dict(zip(["xyz", "fdc", "frest", "scl", "rot", "op"], [p.detach().cpu().double() for p in m.parameter_list()]))
    for k in ref:
        # children's opacity logit(sigmoid(x)) loses ~1e-5 to fp32 cancellation in 1 - o
        tol = 1e-4 if k == "op" else 1e-5
        err = (got[k] - ref[k]).abs().max().item() if ref[k].numel() else 0.0
        assert err < tol, (k, err)


def test_densify_flags_and_empty(pkg, cuda):
    m, grad = _model(pkg, cuda, n=2000, seed=8)
    n0 = m.get_num_points()
    info = m.densify_and_prune(1e9, 1.0, 0.0, xyz_grad=grad)  # threshold never reached, no prune
    assert info == {"kept": n0, "split": 0, "cloned": 0, "n": n0}
    m.density_and_clone(2e-4, 1.0)  # reference-named wrapper: grad None -> nothing
    assert m.get_num_points() == n0
    m.prune_points(torch.arange(n0, device=cuda) % 2 == 0)
    assert m.get_num_points() == (n0 + 1) // 2


def test_densify_remaps_adam_state(pkg, cuda):
    m, grad = _model(pkg, cuda, n=3000, seed=11)
    opt = pkg.optim.FusedAdam([{"params": [p], "lr": 1e-3} for p in m.parameter_list()])
    for p in m.parameter_list():
        p.grad = torch.randn_like(p) * 1e-3
    opt.step()
    before = {i: (opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone())
              for i, p in enumerate(m.parameter_list())}
    _, counts = ref_densify(m, grad, 2e-4, 1.0, 0.01, 5)
    xyz_before = m._xyz.detach().clone()
    op = torch.sigmoid(m._opacity.detach()[:, 0])
    s = m._scaling.detach().exp().mean(-1)
    hot = grad.norm(dim=-1) > 2e-4
    keep = ~(hot & (s > 0.03)) & (op > 0.01)
    info = m.densify_and_prune(2e-4, 1.0, 0.01, optimizer=opt, seed=5, xyz_grad=grad)
    assert info["kept"] == counts[0] == int(keep.sum())
    params = m.parameter_list()
    assert [g["params"][0] for g in opt.param_groups] == params
    for i, p in enumerate(params):
        st = opt.state[p]
        assert st["exp_avg"].shape == p.shape
        assert torch.equal(st["exp_avg"][:info["kept"]], before[i][0][keep])
        assert torch.equal(st["exp_avg_sq"][:info["kept"]], before[i][1][keep])
        assert st["exp_avg"][info["kept"]:].abs().max().item() == 0.0 if info["n"] > info["kept"] else True
    assert torch.equal(m._xyz.detach()[:info["kept"]], xyz_before[keep])
    for p in params:
        p.grad = torch.randn_like(p) * 1e-3
    opt.step()  # the remapped state is usable
