"""Torch fp32 statement of the view-dependent colour logits,
the reference the HIP SH path is checked against (test infrastructure).

The reference renders sigmoid(features[:,0,:]) only (renderer.py:88-92;
MathUtils.spherical_harmonics_eval returns coeffs[:,0], math_utils.py:45-49),
so degree 0 must equal that exactly; degrees 1..3 add the real SH terms of
dir = normalize(xyz - campos) with the 3DGS basis constants and signs:
  logit = f_dc + sum_{k=1}^{(d+1)^2-1} Y_k(dir) f_rest[k-1]
Parity for d > 0 is against this statement only (the reference has no SH
colour to compare with: parity unpinned w.r.t. the reference there)."""
import torch

C1 = 0.4886025119029199
C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
      1.445305721320277, -0.5900435899266435)


def sh_basis(d: torch.Tensor) -> torch.Tensor:
    """[N,3] unit directions -> [N,15] basis Y_1..Y_15."""
    x, y, z = d.unbind(-1)
    xx, yy, zz = x * x, y * y, z * z
    return torch.stack([
        -C1 * y, C1 * z, -C1 * x,
        C2[0] * (x * y), C2[1] * (y * z), C2[2] * (2 * zz - xx - yy), C2[3] * (x * z), C2[4] * (xx - yy),
        C3[0] * y * (3 * xx - yy), C3[1] * (x * y) * z, C3[2] * y * (4 * zz - xx - yy),
        C3[3] * z * (2 * zz - 3 * xx - 3 * yy), C3[4] * x * (4 * zz - xx - yy), C3[5] * z * (xx - yy),
        C3[6] * x * (xx - 3 * yy)], dim=-1)


def sh_logits(xyz, f_dc, f_rest, campos, degree: int) -> torch.Tensor:
    """xyz [N,3], f_dc [N,3], f_rest [N,15,3], campos [3] -> logits [N,3]."""
    if degree == 0:
        return f_dc
    v = xyz - campos.to(xyz)
    d = v / v.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    nb = (degree + 1) ** 2 - 1
    Y = sh_basis(d)[:, :nb]
    out = f_dc
    for k in range(nb):
        out = out + Y[:, k:k + 1] * f_rest[:, k, :]
    return out
