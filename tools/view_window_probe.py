import sys, torch, numpy as np
sys.path.insert(0, '.')
import __graft_entry__ as ge
import bench
pkg = ge.load_package()
from mini3dgs_amd import rasterizer as RZ
dev = torch.device('cuda', 0)
W, H = 1920, 1080
scene = pkg.synthetic.make_scene(1_000_000, W, H, seed=0)
model = pkg.synthetic.to_model(scene, pkg.GaussianModel, dev)
r = pkg.GaussianRenderer()
st = pkg.RenderSettings(image_height=H, image_width=W, bg_color=torch.zeros(3))
for v in (0, 3, 5, 7):
    cam = bench.BenchCamera(W, H, scene.fovx, scene.fovy, bench.view_matrix(v))
    RZ._MSD_BACKOFF.clear()
    calls = {'n': 0}
    orig = RZ.forward_pipeline
    for i in range(6):
        with torch.no_grad():
            out = r.render(cam, model, st)
        torch.cuda.synchronize()
        print('view', v, 'frame', i, 'window', RZ._window_for(dev), 'backoff', RZ._MSD_BACKOFF.get(dev, 0), flush=True)
    # bucket sizes from the keys of the last frame
