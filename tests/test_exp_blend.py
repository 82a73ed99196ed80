"""The blend's exp (csrc/gsplat_mi355x.hip exp_blend), restated in numpy fp32
with an ideal 2^x for v_exp_f32: its 5-operation form on t = -s/2 gives the
same values as the 6-operation form it replaced in round 6 (the remainder in
log2 units on s), and both are within 1 ulp of exp over the range the blend
evaluates (s in [0, 23.1], the :336 skip beyond).  CPU only."""
import numpy as np

F32 = np.float32


def _fma(a, b, c):
    # fp32 fma: the f32 x f32 product is exact in f64, then one rounding of the sum
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F32)


def _exp2(x):  # v_exp_f32, taken as correctly rounded
    return np.exp2(x.astype(np.float64)).astype(F32)


def _full(s, v):
    return np.full_like(s, F32(v))


def exp_blend(t):
    """ph = t log2(e); 2^ph (1 + d), d = t - ph ln2 (ln2 in two parts)."""
    ph = (t * F32(float.fromhex("0x1.715476p+0"))).astype(F32)
    r = _exp2(ph)
    d = _fma(-ph, _full(t, float.fromhex("0x1.62e430p-1")), t)
    d = _fma(-ph, _full(t, -float.fromhex("0x1.05c610p-29")), d)
    return _fma(r, d, r)


def exp_neg_half_r05(s):
    """Rounds 2-5: ph + pl = s (-log2(e) / 2) in log2 units, 2^ph (1 + pl ln2)."""
    c_hi, c_lo = F32(float.fromhex("-0x1.715476p-1")), F32(float.fromhex("-0x1.4ae0bep-27"))
    ph = (s * c_hi).astype(F32)
    pl = _fma(s, _full(s, c_hi), -ph)
    pl = _fma(s, _full(s, c_lo), pl)
    r = _exp2(ph)
    return _fma(r, (pl * F32(float.fromhex("0x1.62e430p-1"))).astype(F32), r)


def test_exp_blend_matches_the_previous_form_and_exp():
    rng = np.random.default_rng(0)
    s = np.concatenate([rng.uniform(0, 23.1, 400_000), rng.uniform(0, 1, 100_000),
                        np.linspace(0, 23.1, 20_001)]).astype(F32)
    t = (F32(-0.5) * s).astype(F32)  # exact: the conic staged as -Q/2 gives t directly
    new, old = exp_blend(t), exp_neg_half_r05(s)
    assert np.array_equal(new, old)
    ref = np.exp(-0.5 * s.astype(np.float64))
    ulp = np.spacing(ref.astype(F32)).astype(np.float64)
    assert (np.abs(new.astype(np.float64) - ref) / ulp).max() <= 1.0
