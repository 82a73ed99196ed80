"""How much slower is the gradient gather when it walks the Gaussians in the
order their last tile row completes (the band order VERDICT r05 item 2's
overlap would need) instead of index order?  C3 frame, one backward, then
k_gather_slots timed with HIP events over 20 launches in each order (the
sums must be the same bits).  GPU tool: python tools/gather_order_probe.py"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pkg = ge.load_package()
RZ, N = pkg.rasterizer, pkg._native
dev = torch.device("cuda:0")
W, H, n = 1920, 1080, 1_000_000
scene = pkg.synthetic.make_scene(n, W, H, seed=0)
model = pkg.synthetic.to_model(scene, pkg.GaussianModel, dev)


class Cam:
    _width, _height, _FoVx, _FoVy = W, H, scene.fovx, scene.fovy

    def world_view_transform(self):
        return torch.eye(4)


st = pkg.RenderSettings(image_height=H, image_width=W, bg_color=torch.zeros(3))
camp = pkg.camera_params(Cam(), st)
g = torch.Generator().manual_seed(1)
cot = [(torch.rand(s, generator=g) * 2 - 1).to(dev) for s in ((3, H, W), (1, H, W), (1, H, W))]
op = torch.sigmoid(model._opacity).squeeze(1)
with torch.no_grad():
    for _ in range(3):
        img, al, dp, m2, cn, _, vis, fr = RZ.forward_pipeline(camp, model._xyz, None, model._scaling, model._rotation,
                                                              model._features_dc[:, 0, :], op, need_grad=True)
        RZ.backward_pipeline(camp, fr, model._xyz, None, model._scaling, model._rotation, model._features_dc[:, 0, :],
                             op, m2, cn, cot[0], cot[1], cot[2], None, None, outputs=(img, al, dp))
torch.cuda.synchronize()
lib = N.load()
fo = fr._o()[0]
fws = fr.frame_ws.data_ptr()
rects = fr.rects
ty1 = (rects[:, 1] >> 16).to(torch.int64)
band = torch.where(vis, ty1, torch.full_like(ty1, 1 << 20))
perm = torch.sort(band, stable=True).indices.to(torch.int32)
sums = {}
for name, order in (("index", None), ("band", perm), ("index", None), ("band", perm)):
    out = torch.empty((n, 10), dtype=torch.float32, device=dev)
    ga = N.GsProjectBwdArgs()
    ga.g.n = n
    ga.vis, ga.rects, ga.pair_offset = vis.data_ptr(), fws + fo[1], fws + fo[8]
    ga.pair_grads = None
    ga.order = N.ptr(order)
    # the frame's partials and flags (single batch at the default tile)
    pg = torch.empty((fr.T * fr.groups, N.GS_PARTIAL_STRIDE), dtype=torch.float32, device=dev)
    ba = N.GsRenderBwdArgs()
    fa = fr.fa
    ba.cam, ba.fb, ba.M, ba.T, ba.tile_alt = fa.cam, fa.fb, fr.M, fr.T, fa.tile_alt
    ba.g, ba.means2d, ba.conics, ba.vis = fa.g, fa.means2d, fa.conics, fa.vis
    ba.image, ba.alpha, ba.depth = img.data_ptr(), al.data_ptr(), dp.data_ptr()
    ba.g_image, ba.g_alpha, ba.g_depth = (c.data_ptr() for c in cot)
    ba.pair_grads, ba.flags_zeroed, ba.project = pg.data_ptr(), 0, 0
    N.check(lib.gs_render_backward(C.byref(ba), N.stream_ptr()), "bwd")
    ga.pair_grads, ga.slot_live, ga.grad_sums, ga.partial_groups = pg.data_ptr(), fr.slot_live.data_ptr(), out.data_ptr(), fr.groups
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    N.check(lib.gs_gather_partials(C.byref(ga), 0, N.stream_ptr()), "warm")
    e0.record()
    for _ in range(20):
        N.check(lib.gs_gather_partials(C.byref(ga), 0, N.stream_ptr()), "gather")
    e1.record()
    torch.cuda.synchronize()
    print(f"gather, {name} order: {e0.elapsed_time(e1) / 20 * 1000:.1f} us per launch", flush=True)
    sums.setdefault(name, out)
print("same sums:", torch.equal(sums["index"], sums["band"]))
