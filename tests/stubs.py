"""Duck-typed camera / Gaussian stand-ins with the contract the reference
renderer reads (renderer.py:59,88-94,135,140-150,166) -- the same contract
the reference's own test stubs satisfy (tests/test_renderer.py:7-53)."""
import numpy as np
import torch


class Cam:
    def __init__(self, w, h, fovx, fovy, wv=None, method=True):
        self._width, self._height = int(w), int(h)
        self._FoVx, self._FoVy = float(fovx), float(fovy)
        self._wv = torch.eye(4) if wv is None else torch.as_tensor(np.asarray(wv, np.float32))
        if not method:  # reference Camera style: a tensor attribute
            self.world_view_transform = self._wv

    def world_view_transform(self):
        return self._wv


class Gauss:
    def __init__(self, xyz, cov3d, logits, opacity, device):
        t = lambda a: torch.tensor(np.asarray(a, np.float32), device=device, requires_grad=True)
        n = np.asarray(xyz).shape[0]
        self.xyz, self.cov = t(xyz), t(np.asarray(cov3d).reshape(n, 3, 3))
        feats = np.zeros((n, 16, 3), np.float32)
        feats[:, 0, :] = np.asarray(logits, np.float32).reshape(n, 3)
        self.feats = t(feats)
        self.op = t(np.asarray(opacity, np.float32).reshape(n, 1))

    @property
    def get_xyz(self):
        return self.xyz

    @property
    def get_covariance(self):
        return self.cov

    @property
    def get_features(self):
        return self.feats

    @property
    def get_opacity(self):
        return self.op


def grad_or_zero(t, shape):
    return t.grad.detach().cpu().numpy() if t.grad is not None else np.zeros(shape, np.float32)
