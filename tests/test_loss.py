"""Fused L1 + D-SSIM (gs_loss_forward / gs_loss_backward) against a plain
PyTorch fp32 statement of the reference's formula (src/core/loss.py:9-63,
completed with the missing `return 1 - ssim.mean()`), forward values and
autograd gradients.  The reference SSIMLoss itself returns None, so this
row's parity is pinned to the formula, not to reference outputs."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def torch_loss(pred, target, lam=0.2, K=11):
    """loss.py:17-39 + :56-58 in fp32 (pred/target [C,H,W])."""
    x = torch.arange(K, device=pred.device).float() - (K - 1) / 2
    g1d = torch.exp(-x ** 2 / (2 * (K / 6) ** 2))
    g1d = (g1d / g1d.sum()).view(1, 1, K)
    pad = K // 2
    C = pred.shape[0]
    wx = g1d.unsqueeze(2).repeat(C, 1, 1, 1)  # [C,1,1,K]
    wy = g1d.unsqueeze(3).repeat(C, 1, 1, 1)  # [C,1,K,1]

    def blur(img):
        out = F.conv2d(img[None], wx, padding=(0, pad), groups=C)
        return F.conv2d(out, wy, padding=(pad, 0), groups=C)[0]

    mu_x, mu_y = blur(pred), blur(target)
    sigma_x = blur(pred ** 2) - mu_x ** 2
    sigma_y = blur(target ** 2) - mu_y ** 2
    sigma_xy = blur(pred * target) - mu_x * mu_y
    ssim = ((2 * mu_x * mu_y + 0.01 ** 2) * (2 * sigma_xy + 0.03 ** 2)) / (
        (mu_x ** 2 + mu_y ** 2 + 0.01 ** 2) * (sigma_x + sigma_y + 0.03 ** 2))
    dssim = 1 - ssim.clamp(0, 1).mean()
    l1 = (pred - target).abs().mean()
    return (1 - lam) * l1 + lam * dssim, l1, dssim


def _pair(shape, seed, dev, blur_target=False):
    g = torch.Generator().manual_seed(seed)
    p = torch.rand(shape, generator=g)
    t = (p + 0.1 * torch.randn(shape, generator=g)).clamp(0, 1) if blur_target else torch.rand(shape, generator=g)
    return p.to(dev), t.to(dev)


@pytest.mark.parametrize("shape,lam,K", [((3, 64, 48), 0.2, 11), ((3, 37, 53), 0.2, 11), ((1, 5, 7), 0.5, 11),
                                         ((3, 40, 40), 1.0, 7), ((2, 33, 17), 0.0, 3), ((3, 270, 480), 0.2, 11)])
def test_fused_loss_matches_torch(pkg, cuda, shape, lam, K):
    p, t = _pair(shape, sum(shape), cuda, blur_target=True)
    p1 = p.clone().requires_grad_()
    total, l1, dssim = pkg.loss.photometric_loss(p1, t, lam, K)
    total.backward()
    p2 = p.clone().requires_grad_()
    rt, rl1, rd = torch_loss(p2, t, lam, K)
    rt.backward()
    assert math.isclose(l1.item(), rl1.item(), rel_tol=2e-6, abs_tol=1e-7)
    assert math.isclose(dssim.item(), rd.item(), rel_tol=1e-5, abs_tol=1e-6)
    assert math.isclose(total.item(), rt.item(), rel_tol=1e-5, abs_tol=1e-6)
    err = (p1.grad - p2.grad).abs().max().item()
    assert err <= 1e-3 * p2.grad.abs().max().item() + 1e-9, err


def test_modules_and_batched_input(pkg, cuda):
    p, t = _pair((1, 3, 32, 40), 3, cuda)
    d = pkg.SSIMLoss()(p, t)
    _, _, rd = torch_loss(p[0], t[0], 1.0, 11)
    assert math.isclose(d.item(), rd.item(), rel_tol=1e-5)
    total, logs = pkg.GaussianLoss(0.2)(p, t)
    rt, rl1, rd = torch_loss(p[0], t[0], 0.2, 11)
    assert set(logs) == {"l1", "dssim", "total_loss"} and all(isinstance(v, float) for v in logs.values())
    assert math.isclose(logs["total_loss"], rt.item(), rel_tol=1e-5)
    assert math.isclose(logs["l1"], rl1.item(), rel_tol=1e-5)
    # identical images: D-SSIM 0, L1 0, gradient of the L1 term 0 (sign(0) = 0)
    q = p.clone().requires_grad_()
    tot, l1, ds = pkg.loss.photometric_loss(q, p, 0.2)
    tot.backward()
    assert l1.item() == 0.0 and abs(ds.item()) < 1e-6 and q.grad.abs().max().item() < 1e-5


def test_loss_deterministic(pkg, cuda):
    p, t = _pair((3, 135, 240), 9, cuda)
    res = []
    for _ in range(2):
        q = p.clone().requires_grad_()
        tot, _, _ = pkg.loss.photometric_loss(q, t)
        tot.backward()
        res.append((tot.detach().clone(), q.grad.clone()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
