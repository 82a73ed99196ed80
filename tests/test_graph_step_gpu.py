"""The replayed training step (graph_step.GraphedStep):
render forward + backward + FusedAdam captured once as a HIP graph over a
device-resident frame (no host read-back), replayed -- equal to the eager
step (GaussianRenderer.render -> autograd -> FusedAdam.step) bit for bit,
including steps whose frame failed on the device (a tile workspace below T,
a depth-key window that misses) and were skipped by the Adam launch and
redone on the host path."""
import pytest
import torch

pytestmark = pytest.mark.gpu

N_G, W, H = 20_000, 320, 240


def _setup(pkg, cuda, seed=0, shadow=False):
    scene = pkg.synthetic.make_scene(N_G, W, H, seed=seed)
    model = pkg.synthetic.to_model(scene, pkg.GaussianModel, cuda)
    opt = pkg.optim.FusedAdam([{"params": [model._xyz], "lr": 1.6e-4}, {"params": [model._features_dc], "lr": 2.5e-3},
                               {"params": [model._opacity], "lr": 0.05}, {"params": [model._scaling], "lr": 5e-3},
                               {"params": [model._rotation], "lr": 1e-3}])
    if shadow:
        for p in model.grad_parameters():
            opt.set_output(p, torch.empty_like(p))

    class Cam:
        _width, _height, _FoVx, _FoVy = W, H, scene.fovx, scene.fovy

        def world_view_transform(self):
            return torch.eye(4)
    settings = pkg.RenderSettings(image_height=H, image_width=W, bg_color=torch.tensor([0.1, 0.2, 0.3]))
    g = torch.Generator().manual_seed(1)
    cot = [(torch.rand(s, generator=g) * 2 - 1).to(cuda) for s in ((3, H, W), (1, H, W), (1, H, W))]
    return model, opt, Cam(), settings, cot


def _eager(pkg, model, opt, cam, settings, cot, steps):
    r = pkg.GaussianRenderer()
    out = None
    for _ in range(steps):
        opt.zero_grad(set_to_none=True)
        out = r.render(cam, model, settings)
        torch.autograd.backward([out["image"], out["alpha"], out["depth"]], cot)
        opt.step()
    torch.cuda.synchronize()
    return out


def _assert_same_state(ma, oa, mb, ob):
    for pa, pb in zip(ma.grad_parameters(), mb.grad_parameters()):
        assert torch.equal(pa.detach(), pb.detach())
        sa, sb = oa.state[pa], ob.state[pb]
        if not sa:
            assert not sb
            continue
        assert sa["step"] == sb["step"]
        assert torch.equal(sa["exp_avg"], sb["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"])
        oa_out, ob_out = oa.param_out.get(pa), ob.param_out.get(pb)
        if oa_out is not None:
            assert torch.equal(oa_out, ob_out)


def test_graph_replays_equal_eager_steps(pkg, cuda):
    """Six steps: one eager (Adam state, T), five replays of one graph -- the
    parameters, moments and step counts equal six eager steps bit for bit,
    and the last replay's image / gradients equal the last eager frame's."""
    ma, oa, cam, st, cot = _setup(pkg, cuda)
    out = _eager(pkg, ma, oa, cam, st, cot, 6)
    mb, ob, cam_b, st_b, cot_b = _setup(pkg, cuda)
    gs = pkg.GraphedStep(pkg.GaussianRenderer(), cam_b, mb, st_b, cot_b, ob)
    with torch.cuda.stream(gs.stream):
        for _ in range(6):
            gs.step()
    gs.finish()
    assert gs.redone == [] and gs.replays == 5 and gs.graph is not None and gs.graph.num_nodes > 10
    _assert_same_state(ma, oa, mb, ob)
    for k in ("image", "alpha", "depth"):
        assert torch.equal(out[k].detach(), getattr(gs, k))
    assert torch.equal(out["viewspace_points"].detach(), gs.means2d)
    assert torch.equal(out["visibility_filter"], gs.vis)
    for p, g in gs.leaf_grad:
        q = dict(zip(map(id, mb.grad_parameters()), ma.grad_parameters()))[id(p)]
        assert torch.equal(q.grad, g), "gradient of the last step"
    gs.close()


def test_graph_failed_frames_are_skipped_and_redone(pkg, cuda):
    """A capture with a tile workspace below T (GS_FRAME_NEED_CAPACITY), then
    one with a depth-key window the depths miss (GS_FRAME_WINDOW_MISS): each
    failed replay -- and the one queued behind it -- updates nothing on the
    device, is redone eagerly, and the graph is captured again.  Eight steps
    equal eight eager steps bit for bit (shadow parameter outputs, as the
    bench, and in place)."""
    for shadow in (False, True):
        ma, oa, cam, st, cot = _setup(pkg, cuda, seed=3, shadow=shadow)
        _eager(pkg, ma, oa, cam, st, cot, 8)
        mb, ob, cam_b, st_b, cot_b = _setup(pkg, cuda, seed=3, shadow=shadow)
        gs = pkg.GraphedStep(pkg.GaussianRenderer(), cam_b, mb, st_b, cot_b, ob)
        gs.capacity = 256  # far below T: the first capture's frames fail
        with torch.cuda.stream(gs.stream):
            gs.step()  # eager, then the capture
            assert gs.graph is not None and gs._cap == 256
            # the next capture (after the capacity recovery) gets a window all
            # visible depths miss: keys based above the largest depth's bits
            gs.window = (0x7F000000, 16)
            for _ in range(7):
                gs.step()
        gs.finish()
        flags = [f for f, _ in gs.redone]
        assert len(flags) == 2, gs.redone
        assert flags[0] & pkg._native.GS_FRAME_NEED_CAPACITY
        assert flags[1] & pkg._native.GS_FRAME_WINDOW_MISS
        assert all(k >= 1 for _, k in gs.redone)
        assert gs.window == "auto" and gs._cap > 256
        _assert_same_state(ma, oa, mb, ob)
        gs.close()


def test_graph_event_pairs_time_the_blend_backward(pkg, cuda):
    """The blend backward's event pair recorded inside every replay (event
    record nodes re-pointed per replay): one positive interval per timed
    replay, of the order of the kernel's eager duration."""
    mb, ob, cam, st, cot = _setup(pkg, cuda)
    gs = pkg.GraphedStep(pkg.GaussianRenderer(), cam, mb, st, cot, ob)
    with torch.cuda.stream(gs.stream):
        gs.step()
        gs.step()
        gs.timing = True
        for _ in range(4):
            gs.step()
        gs.timing = False
    gs.finish()
    ms = gs.blend_backward_ms()
    assert len(ms) == 4 and all(0.0 < x < 50.0 for x in ms), ms
    gs.close()


def test_fused_adam_in_the_projection_backward(pkg, cuda):
    """the optimizer in the backward
    (gs_project_backward_adam) -- replayed steps whose projection backward
    applies the Adam update itself, no gradient written -- equal eager steps
    (autograd + FusedAdam.step) bit for bit: parameters, moments, step counts,
    with shadow outputs and in place; a failed frame is skipped there too."""
    for shadow in (False, True):
        ma, oa, cam, st, cot = _setup(pkg, cuda, seed=5, shadow=shadow)
        _eager(pkg, ma, oa, cam, st, cot, 6)
        mb, ob, cam_b, st_b, cot_b = _setup(pkg, cuda, seed=5, shadow=shadow)
        gs = pkg.GraphedStep(pkg.GaussianRenderer(), cam_b, mb, st_b, cot_b, ob, fused_adam=True)
        gs.capacity = 512  # (one failed replay pair, redone: the fused update skipped on the device)
        with torch.cuda.stream(gs.stream):
            for _ in range(6):
                gs.step()
        gs.finish()
        assert len(gs.redone) == 1 and gs.redone[0][0] & pkg._native.GS_FRAME_NEED_CAPACITY
        _assert_same_state(ma, oa, mb, ob)
        gs.close()


@pytest.mark.parametrize("size", ["C2", "C3"])
def test_graph_replay_at_benchmark_size(pkg, cuda, size):
    """The capacity-sized launches at the BASELINE sizes (C2: 100k Gaussians,
    800x800; C3: 1M, 1920x1080, T = 4.4M list entries): three replayed steps
    with the optimizer in the backward and shadow parameter outputs (the
    bench's step) equal three eager steps bit for bit -- parameters, moments,
    and the last frame's image, alpha, depth."""
    n, w, h = {"C2": (100_000, 800, 800), "C3": (1_000_000, 1920, 1080)}[size]
    res = []
    for graph in (False, True):
        scene = pkg.synthetic.make_scene(n, w, h, seed=0)
        model = pkg.synthetic.to_model(scene, pkg.GaussianModel, cuda)
        opt = pkg.optim.FusedAdam([{"params": [model._xyz], "lr": 1.6e-4},
                                   {"params": [model._features_dc], "lr": 2.5e-3},
                                   {"params": [model._opacity], "lr": 0.05}, {"params": [model._scaling], "lr": 5e-3},
                                   {"params": [model._rotation], "lr": 1e-3}])
        for p in model.grad_parameters():
            opt.set_output(p, torch.empty_like(p))

        class Cam:
            _width, _height, _FoVx, _FoVy = w, h, scene.fovx, scene.fovy

            def world_view_transform(self):
                return torch.eye(4)
        st = pkg.RenderSettings(image_height=h, image_width=w, bg_color=torch.zeros(3))
        g = torch.Generator().manual_seed(1)
        cot = [(torch.rand(s, generator=g) * 2 - 1).to(cuda) for s in ((3, h, w), (1, h, w), (1, h, w))]
        if graph:
            gs = pkg.GraphedStep(pkg.GaussianRenderer(), Cam(), model, st, cot, opt, fused_adam=True)
            with torch.cuda.stream(gs.stream):
                for _ in range(4):
                    gs.step()
            gs.finish()
            assert gs.redone == [] and gs.replays == 3
            imgs = (gs.image.clone(), gs.alpha.clone(), gs.depth.clone())
            gs.close()
        else:
            out = _eager(pkg, model, opt, Cam(), st, cot, 4)
            imgs = tuple(out[k].detach().clone() for k in ("image", "alpha", "depth"))
        state = [(opt.param_out[p].clone(), opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone(),
                  opt.state[p]["step"]) for p in model.grad_parameters() if p in opt.state]
        res.append((imgs, state))
        del model, opt
        torch.cuda.empty_cache()
    (ia, sa), (ib, sb) = res
    for x, y in zip(ia, ib):
        assert torch.equal(x, y)
    assert len(sa) == len(sb) == 5
    for a_, b_ in zip(sa, sb):
        assert a_[3] == b_[3]
        for x, y in zip(a_[:3], b_[:3]):
            assert torch.equal(x, y)
