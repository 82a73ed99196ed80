// gsplat_mi355x.hip -- CDNA4 (gfx950) kernels behind include/gsplat_mi355x.h.
//
// Differentiable tile rasterizer replacing GaussianRenderer.render() of the
// reference (src/core/renderer.py:31-367) and its autograd backward.
// Stages (each cites the reference lines it replaces):
//   k_project_fwd     renderer.py:117-220   projection, 2D cov, conic, radius, culling
//   k_radix_*         renderer.py:231-237   stable LSD radix sort (depth, then tile id)
//   k_bin_*           renderer.py:263-298   tile binning, emitted in depth order
//   k_tile_ranges     renderer.py:266       per-tile list ranges
//   k_blend_fwd       renderer.py:273-367   per-pixel front-to-back compositing
//   k_blend_bwd       autograd of :313-367  replayed front-to-back, per-pair grad slots
//   k_project_bwd     autograd of :117-200  (+ gaussian_model.py:200-207 on the raw path)
//
// Layout and roofline notes: DESIGN.md.  Wave size is 64 everywhere.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "gsplat_mi355x.h"
#include "gs_internal.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;
#ifndef GS_RANGES_X4
#define GS_RANGES_X4 1
#endif
#ifndef GS_SORT_IPT
#define GS_SORT_IPT 8
#endif
constexpr int kSortIpt = GS_SORT_IPT;            // items per thread per sort block (4, 16: slower)
constexpr int kSortChunk = kBlock * kSortIpt;    // 2048 items per block
static_assert(kSortChunk == kSortBlockEntries, "gs_internal.h kSortBlockEntries");
constexpr int kBinChunk = kBlock * 4;            // 1024 Gaussians per binning block (2 and 1 rounds: slower)
#ifndef GS_DEBUG  // 1: report (printf) blend list ranges clamped to the T entries
#define GS_DEBUG 0
#endif
constexpr float kAlphaStop = 0.995f;             // renderer.py:352
// renderer.py:336 skips a pair when w = exp(-s/2) < 1e-5; decided here on
// s: s > 2 ln(1e5).  The same decision except where exp's rounding
// straddles 1e-5 -- the band in which any two fp32 exps (ours, torch's)
// already disagree -- and it saves the compare on w for every evaluated
// pair (C3: the same 9 knife-edge pixels).  Forward and backward share it.
constexpr float kSkipS = 23.0258509f;
// The blend kernels evaluate t = -s/2 directly: the conic coefficients are
// staged as -Q/2 (a power-of-two scaling, exact for every product and sum of
// the reference's s), so the skip is t < -ln(1e5), the same decision.
constexpr float kSkipT = -0.5f * kSkipS;

thread_local char g_err[512];

gs_status fail(gs_status s, const char *fmt, const char *what) {
  snprintf(g_err, sizeof(g_err), fmt, what);
  return s;
}

gs_status check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: launch failed: %s", what, hipGetErrorString(e));
    return GS_ERR_LAUNCH;
  }
  return GS_OK;
}

inline unsigned div_up(long long a, long long b) { return (unsigned)((a + b - 1) / b); }
__device__ __forceinline__ uint32_t div_up_dev(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + b - 1) / b); }

// torch.clamp semantics (NaN propagates)
__device__ __forceinline__ float clamp01(float v) { return v < 0.f ? 0.f : (v > 1.f ? 1.f : v); }
// clamp to [0,1] as the VALU clamp output modifier (folds into the producing
// instruction).  Equals clamp01 for every non-NaN input; NaN -> 0 instead of
// NaN (only reachable from NaN/inf inputs).  Used on the blend's hot path.
__device__ __forceinline__ float sat01(float v) { return __builtin_amdgcn_fmed3f(v, 0.f, 1.f); }
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops
// (lgkmcnt) but NOT for its global loads, unlike __syncthreads() whose
// workgroup fence drains vmcnt -- prefetched gathers stay in flight across it.
// The "memory" clobber keeps the compiler from moving memory ops across.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// wave-uniform "any lane" without the bool -> VGPR -> compare round trip
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
__device__ __forceinline__ float clampf(float v, float lo, float hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

// Dense 40-B gradient partials are 8-B aligned only: 16-B accesses to them go
// through this explicitly under-aligned vector type (global_load/store_dwordx4
// need 4-B alignment on gfx950; a plain float4 would promise 16).  Five
// float2 accesses instead cost the gather ~35 us at C3 (more load
// instructions in flight per partial).
typedef float f4_u8 __attribute__((ext_vector_type(4), aligned(8)));
typedef float f2_u8 __attribute__((ext_vector_type(2), aligned(8)));

// exp(t) for the blend's exponent t = -s/2 (it evaluates the exp only for
// s <= 23.1, t in [-11.6, 0]; beyond, for non-positive-definite conics, it
// stays finite until 2^ph overflows), given t itself: the blend kernels
// compute t from the conic staged as -Q/2 (stage_conic0/1).  ph = t log2(e)
// rounded, 2^ph by v_exp_f32 (no range reduction or ldexp: 2^ph stays a
// normal float here), times (1 + d) with the remainder d = t - ph ln2 in
// natural-log units (Cody-Waite: ln2 in two parts, each fma's product exact).
// ~1 ulp, like expf; forward and backward share it, so their decisions
// replay bit-identically.  5 VALU per pair.  Rounds 2-5 took the remainder
// in log2 units (ph + pl from x log2(e), then 2^ph (1 + pl ln2)) and the
// exponent from s (x = -s/2): 6 VALU, and the same values (round 6: every one
// of 2.6 M sampled t, emulated).  Dropping the remainder's low part instead
// saves a VALU too, but is <= 3 ulp at t = -11.6: 12 knife-edge pixels and
// the scaling gradient's error 5.4e-4 -> 1.2e-3 of scale (round 2).  Not taken.
__device__ __forceinline__ float exp_blend(float t) {
  const float ph = t * 0x1.715476p+0f;
  const float r = __builtin_amdgcn_exp2f(ph);
  float d = __builtin_fmaf(-ph, 0x1.62e430p-1f, t);
  d = __builtin_fmaf(-ph, -0x1.05c610p-29f, d);
  return __builtin_fmaf(r, d, r);
}

// A record's conic staged for the blend loops as -Q/2: t = conic_s(dx, dy,
// h00, ho, h11) is then -s/2 exactly.
__device__ __forceinline__ float4 stage_conic0(float4 r0) {  // (mx, my, q00, q11) -> (mx, my, h00, h11)
  return make_float4(r0.x, r0.y, -0.5f * r0.z, -0.5f * r0.w);
}
__device__ __forceinline__ float4 stage_conic1(float4 r1) {  // (qo, o, r, g) -> (ho, o, r, g)
  return make_float4(-0.5f * r1.x, r1.y, r1.z, r1.w);
}

// s = [dx dy] Q [dx dy]^T for the blend's conic form (q00, qo = Q01+Q10,
// q11) in the reference's unfused order (renderer.py:333).  A fused form
// (5 operations instead of 8) was measured: with ill-conditioned conics the
// cancellation amplifies its ~1-ulp difference into visible errors (needle
// test: 1e-2 image error), so the reference's rounding is kept.
__device__ __forceinline__ float conic_s(float dx, float dy, float q00, float qo, float q11) {
  return ((dx * dx) * q00 + (qo * dx) * dy) + (dy * dy) * q11;
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int lane = threadIdx.x & (kWave - 1);
  return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}

// ---------------------------------------------------------------- scans ----
// Exclusive scan of one u32 per thread over a 256-thread block.
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *s_tmp, uint32_t *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  if (lane == 63) s_tmp[wave] = incl;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    uint32_t x = s_tmp[w];
    base += (w < wave) ? x : 0u;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

// Three exclusive scans over the block at once (one round of shuffles and
// barriers for all three: the single-block scans are latency-bound).
__device__ __forceinline__ uint3 block_exscan3(uint3 v, uint32_t (*s_tmp)[kBlock / kWave], uint3 *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint3 incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t tx = __shfl_up(incl.x, d, 64), ty = __shfl_up(incl.y, d, 64), tz = __shfl_up(incl.z, d, 64);
    if (lane >= d) {
      incl.x += tx;
      incl.y += ty;
      incl.z += tz;
    }
  }
  if (lane == 63) {
    s_tmp[0][wave] = incl.x;
    s_tmp[1][wave] = incl.y;
    s_tmp[2][wave] = incl.z;
  }
  __syncthreads();
  uint3 base = make_uint3(0u, 0u, 0u), tot = make_uint3(0u, 0u, 0u);
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    const uint32_t x = s_tmp[0][w], y = s_tmp[1][w], z = s_tmp[2][w];
    base.x += (w < wave) ? x : 0u;
    base.y += (w < wave) ? y : 0u;
    base.z += (w < wave) ? z : 0u;
    tot.x += x;
    tot.y += y;
    tot.z += z;
  }
  __syncthreads();
  *total = tot;
  return make_uint3(base.x + incl.x - v.x, base.y + incl.y - v.y, base.z + incl.z - v.z);
}

// Lanes of the wave holding the same `nbits`-bit digit (match-any via ballots).
__device__ __forceinline__ unsigned long long match_digit(uint32_t d, int nbits, unsigned long long m) {
  for (int b = 0; b < nbits; ++b) {
    const bool bit = (d >> b) & 1u;
    const unsigned long long bb = __ballot(bit);
    m &= bit ? bb : ~bb;
  }
  return m;
}

// ------------------------------------------------------------ geometry ----
__device__ __forceinline__ void unpack_rect(const uint32_t *rects, uint32_t g, int &tx0, int &tx1,
                                            int &ty0, int &ty1) {
  const uint2 r = reinterpret_cast<const uint2 *>(rects)[g];
  tx0 = (int)(r.x & 0xFFFFu);
  tx1 = (int)(r.x >> 16);
  ty0 = (int)(r.y & 0xFFFFu);
  ty1 = (int)(r.y >> 16);
}
__device__ __forceinline__ uint32_t rect_touches(int tx0, int tx1, int ty0, int ty1) {
  return (tx1 >= tx0 && ty1 >= ty0) ? (uint32_t)((tx1 - tx0 + 1) * (ty1 - ty0 + 1)) : 0u;
}

// Sigma = R(normalize(q)) diag(exp(s)^2) R^T  (gaussian_model.py:200-207,
// math_utils.py:10-26), fp32 in the reference's order.
__device__ __forceinline__ void cov_from_raw(const float *sc, const float *rq, float S[9]) {
  float w = rq[0], x = rq[1], y = rq[2], z = rq[3];
  for (int it = 0; it < 2; ++it) {  // get_rotation normalises, build_rotation_matrix again
    float n = sqrtf(w * w + x * x + y * y + z * z);
    n = n < 1e-12f ? 1e-12f : n;
    w /= n; x /= n; y /= n; z /= n;
  }
  const float R[9] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y - w * z), 2.f * (x * z + w * y),
                      2.f * (x * y + w * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - w * x),
                      2.f * (x * z - w * y), 2.f * (y * z + w * x), 1.f - 2.f * (x * x + y * y)};
  float s2[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float s = expf(sc[k]);
    s2[k] = s * s;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      S[i * 3 + j] = ((R[i * 3] * s2[0]) * R[j * 3] + (R[i * 3 + 1] * s2[1]) * R[j * 3 + 1]) +
                     (R[i * 3 + 2] * s2[2]) * R[j * 3 + 2];
}

// ------------------------------------------------- view-dependent colour ----
// Real SH basis Y_1..Y_15 (degrees 1..3) with the 3DGS constants and signs;
// Y_0 is folded into the DC logit (gs_gaussians.sh_degree in the header).
constexpr float kSH1 = 0.4886025119029199f;
constexpr float kSH2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                           -1.0925484305920792f, 0.5462742152960396f};
constexpr float kSH3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                           0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                           -0.5900435899266435f};

__device__ __forceinline__ void sh_basis(float x, float y, float z, float Y[15]) {
  const float xx = x * x, yy = y * y, zz = z * z;
  Y[0] = -kSH1 * y;
  Y[1] = kSH1 * z;
  Y[2] = -kSH1 * x;
  Y[3] = kSH2[0] * (x * y);
  Y[4] = kSH2[1] * (y * z);
  Y[5] = kSH2[2] * (2.f * zz - xx - yy);
  Y[6] = kSH2[3] * (x * z);
  Y[7] = kSH2[4] * (xx - yy);
  Y[8] = kSH3[0] * y * (3.f * xx - yy);
  Y[9] = kSH3[1] * (x * y) * z;
  Y[10] = kSH3[2] * y * (4.f * zz - xx - yy);
  Y[11] = kSH3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
  Y[12] = kSH3[4] * x * (4.f * zz - xx - yy);
  Y[13] = kSH3[5] * z * (xx - yy);
  Y[14] = kSH3[6] * x * (xx - 3.f * yy);
}

// dY_k/d(x, y, z) contracted with per-basis weights w[k] (the direction is
// treated as free; the caller projects through the normalisation)
__device__ __forceinline__ void sh_basis_vjp(float x, float y, float z, const float w[15], int nb, float d[3]) {
  const float xx = x * x, yy = y * y, zz = z * z;
  float dx = -kSH1 * w[2], dy = -kSH1 * w[0], dz = kSH1 * w[1];
  if (nb > 3) {
    dx += kSH2[0] * y * w[3] - 2.f * kSH2[2] * x * w[5] + kSH2[3] * z * w[6] + 2.f * kSH2[4] * x * w[7];
    dy += kSH2[0] * x * w[3] + kSH2[1] * z * w[4] - 2.f * kSH2[2] * y * w[5] - 2.f * kSH2[4] * y * w[7];
    dz += kSH2[1] * y * w[4] + 4.f * kSH2[2] * z * w[5] + kSH2[3] * x * w[6];
  }
  if (nb > 8) {
    dx += 6.f * kSH3[0] * x * y * w[8] + kSH3[1] * y * z * w[9] - 2.f * kSH3[2] * x * y * w[10] -
          6.f * kSH3[3] * x * z * w[11] + kSH3[4] * (4.f * zz - 3.f * xx - yy) * w[12] +
          2.f * kSH3[5] * x * z * w[13] + kSH3[6] * (3.f * xx - 3.f * yy) * w[14];
    dy += kSH3[0] * (3.f * xx - 3.f * yy) * w[8] + kSH3[1] * x * z * w[9] +
          kSH3[2] * (4.f * zz - xx - 3.f * yy) * w[10] - 6.f * kSH3[3] * y * z * w[11] -
          2.f * kSH3[4] * x * y * w[12] - 2.f * kSH3[5] * y * z * w[13] - 6.f * kSH3[6] * x * y * w[14];
    dz += kSH3[1] * x * y * w[9] + 8.f * kSH3[2] * y * z * w[10] + kSH3[3] * (6.f * zz - 3.f * xx - 3.f * yy) * w[11] +
          8.f * kSH3[4] * x * z * w[12] + kSH3[5] * (xx - yy) * w[13];
  }
  d[0] = dx;
  d[1] = dy;
  d[2] = dz;
}

__device__ __forceinline__ int sh_rest_count(int degree) { return (degree + 1) * (degree + 1) - 1; }

// Colour logits of Gaussian g: the DC logits, plus the SH terms when enabled.
// dir / inv_norm are returned for the backward.
__device__ __forceinline__ void color_logits(const gs_gaussians &G, const gs_camera &c, int g, float xw, float yw,
                                             float zw, float lg[3], float dir[3], float &inv_norm) {
  const float *cl = G.color_logits + (int64_t)g * G.color_stride;
  lg[0] = cl[0];
  lg[1] = cl[1];
  lg[2] = cl[2];
  inv_norm = 0.f;
  if (G.sh_degree <= 0) return;
  const float vx = xw - c.campos[0], vy = yw - c.campos[1], vz = zw - c.campos[2];
  const float nrm = sqrtf((vx * vx + vy * vy) + vz * vz);
  inv_norm = 1.f / fmaxf(nrm, 1e-12f);
  dir[0] = vx * inv_norm;
  dir[1] = vy * inv_norm;
  dir[2] = vz * inv_norm;
  float Y[15];
  sh_basis(dir[0], dir[1], dir[2], Y);
  const int nb = sh_rest_count(G.sh_degree);
  const float *r = G.sh_rest + (int64_t)g * G.sh_rest_stride;
  for (int k = 0; k < nb; ++k) {
    lg[0] += Y[k] * r[3 * k];
    lg[1] += Y[k] * r[3 * k + 1];
    lg[2] += Y[k] * r[3 * k + 2];
  }
}

// =================================================== stage 1: projection ==
// kHot: raw scale/rotation and DC colour (training); every input load is
// issued at the top (under the visibility branch they were waited for in
// further round trips).
template <bool kHot>
__global__ __launch_bounds__(kBlock) void k_project_fwd(gs_project_args a) {
  __shared__ uint32_t s_mm[2][kBlock / kWave];
  const int g = blockIdx.x * kBlock + threadIdx.x;
  bool visible = false;
  uint32_t zbits = 0u;
  if (g < a.g.n) {
    const gs_camera &c = a.cam;
    const float *X3 = a.g.xyz + (int64_t)g * a.g.xyz_stride;
    const float xw = X3[0], yw = X3[1], zw = X3[2];
    float scl_pre[3] = {0.f, 0.f, 0.f}, rot_pre[4] = {0.f, 0.f, 0.f, 0.f}, cl_pre[3] = {0.f, 0.f, 0.f};
    float op_pre = 0.f;
    if constexpr (kHot) {
#pragma unroll
      for (int k = 0; k < 3; ++k) scl_pre[k] = a.g.scaling[(int64_t)g * 3 + k];
#pragma unroll
      for (int k = 0; k < 4; ++k) rot_pre[k] = a.g.rotation[(int64_t)g * 4 + k];
#pragma unroll
      for (int k = 0; k < 3; ++k) cl_pre[k] = a.g.color_logits[(int64_t)g * a.g.color_stride + k];
      op_pre = a.g.opacity[(int64_t)g * a.g.opacity_stride];
    }
    float S[9];
    if (!kHot && a.g.cov3d) {
      const float *cp = a.g.cov3d + (int64_t)g * 9;
#pragma unroll
      for (int k = 0; k < 9; ++k) S[k] = cp[k];
    } else {
      cov_from_raw(kHot ? scl_pre : a.g.scaling + (int64_t)g * 3, kHot ? rot_pre : a.g.rotation + (int64_t)g * 4, S);
    }
    const float *R = c.view;  // rows [R | t]
    // Xc = Xw @ Rv.T + Tv (renderer.py:154)
    float Xc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      Xc[i] = ((xw * R[i * 4] + yw * R[i * 4 + 1]) + zw * R[i * 4 + 2]) + R[i * 4 + 3];
    const float X = Xc[0], Y = Xc[1], Z = Xc[2];
    const float mx = (c.fx * X) / Z + c.cx;      // :161
    const float my = ((-c.fy) * Y) / Z + c.cy;   // :162
    // cov_cam = (Rv @ Sigma) @ Rv.T (:168)
    float RS[9], C[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        RS[i * 3 + j] = (R[i * 4] * S[j] + R[i * 4 + 1] * S[3 + j]) + R[i * 4 + 2] * S[6 + j];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        C[i * 3 + j] = (RS[i * 3] * R[j * 4] + RS[i * 3 + 1] * R[j * 4 + 1]) + RS[i * 3 + 2] * R[j * 4 + 2];
    // J (:171-177)
    const float iz = 1.0f / Z;
    const float J[6] = {c.fx * iz, 0.f, (((-c.fx) * X) * iz) * iz, 0.f, (-c.fy) * iz, ((c.fy * Y) * iz) * iz};
    float JC[6];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        JC[i * 3 + j] = (J[i * 3] * C[j] + J[i * 3 + 1] * C[3 + j]) + J[i * 3 + 2] * C[6 + j];
    float V[4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        V[i * 2 + j] = (JC[i * 3] * J[j * 3] + JC[i * 3 + 1] * J[j * 3 + 1]) + JC[i * 3 + 2] * J[j * 3 + 2];
    V[0] += 1e-6f;  // :182-183
    V[3] += 1e-6f;
    // conic = inv(cov2d) (:186) and lambda_max (:188) in double: LAPACK-grade
    const double va = V[0], vb = V[1], vc = V[2], vd = V[3];
    const double det = va * vd - vb * vc;
    const float q0 = (float)(vd / det), q1 = (float)(-vb / det), q2 = (float)(-vc / det),
                q3 = (float)(va / det);
    const double hm = 0.5 * (va + vd), hd = 0.5 * (va - vd);
    const float lmax = (float)(hm + sqrt(hd * hd + vc * vc));
    const float r = clampf(3.0f * sqrtf(lmax), c.radius_min, c.radius_max);  // :190-192
    const int W = c.image_width, H = c.image_height;
    // culling (:218)
    visible = (Z > 0.f) && (mx >= -r) && (mx < (float)W + r) && (my >= -r) && (my < (float)H + r) &&
              (r > 0.f);
    reinterpret_cast<float2 *>(a.means2d)[g] = make_float2(mx, my);
    reinterpret_cast<float4 *>(a.conics)[g] = make_float4(q0, q1, q2, q3);
    a.radii[g] = r;
    a.vis[g] = visible ? 1 : 0;
    // tile rectangle (:278-293), int() truncation toward zero
    uint32_t rx = 1u, ry = 1u;  // empty: tx0=1 > tx1=0
    uint32_t rinfo = 0u;        // record word 11: tx0 | ty0 << 12 | (tiles wide - 1) << 24
    if (visible) {
      const int ri = (int)r, icx = (int)mx, icy = (int)my;
      int x0 = icx - ri, x1 = icx + 1 + ri, y0 = icy - ri, y1 = icy + 1 + ri;
      x0 = x0 < 0 ? 0 : x0;
      y0 = y0 < 0 ? 0 : y0;
      x1 = x1 > W ? W : x1;
      y1 = y1 > H ? H : y1;
      if (x0 < x1 && y0 < y1) {
        const int T = c.tile_size;  // GaussianRenderer(tile_size) (:290-293)
        rx = (uint32_t)(x0 / T) | ((uint32_t)((x1 - 1) / T) << 16);
        ry = (uint32_t)(y0 / T) | ((uint32_t)((y1 - 1) / T) << 16);
        rinfo = (uint32_t)(x0 / T) | ((uint32_t)(y0 / T) << 12) | ((uint32_t)((x1 - 1) / T - x0 / T) << 24);
      }
      float cl[3], dir[3], inv_norm;
      if constexpr (kHot) {
        cl[0] = cl_pre[0]; cl[1] = cl_pre[1]; cl[2] = cl_pre[2];
        (void)dir; (void)inv_norm;
      } else {
        color_logits(a.g, c, g, xw, yw, zw, cl, dir, inv_norm);
      }
      float op = kHot ? op_pre : a.g.opacity[(int64_t)g * a.g.opacity_stride];
      if (a.g.opacity_is_logit) op = 1.f / (1.f + expf(-op));  // get_opacity
      float4 *rec = reinterpret_cast<float4 *>(a.records) + 3 * (int64_t)g;
      // record: mx my q00 q11 | qo o r g | b z off rinfo -- (q00, q11) adjacent so
      // that the blend's dx^2 q00, dy^2 q11 are one packed multiply
      const float cr = 1.f / (1.f + expf(-cl[0])), cg = 1.f / (1.f + expf(-cl[1])), cb = 1.f / (1.f + expf(-cl[2]));  // sigmoid (:90)
      rec[0] = make_float4(mx, my, q0, q3);
      rec[1] = make_float4(q1 + q2, op, cr, cg);
      rec[2] = make_float4(cb, Z, 0.f, __uint_as_float(rinfo));
    }
    reinterpret_cast<uint2 *>(a.rects)[g] = make_uint2(rx, ry);
    zbits = __float_as_uint(Z);
    const uint32_t kmask = a.key_bits >= 32 ? 0xFFFFFFFFu : (1u << a.key_bits) - 1u;
    // (a key outside the window is caught by the caller from counters[2..3])
    a.depth_keys[g] = visible ? ((zbits - a.key_base) & kmask) : kmask;
  }
  // the block's min / max of the visible depth bits (plain stores, reduced by gs_bin_count)
  uint32_t mn = visible ? zbits : 0xFFFFFFFFu, mx = visible ? zbits : 0u;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, d, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
  }
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
  if (lane == 0) {
    s_mm[0][wave] = mn;
    s_mm[1][wave] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 1; w < kBlock / kWave; ++w) {
      mn = min(mn, s_mm[0][w]);
      mx = max(mx, s_mm[1][w]);
    }
    a.key_minmax[2 * blockIdx.x] = mn;
    a.key_minmax[2 * blockIdx.x + 1] = mx;
  }
}

// ===================================================== radix sort =========
// Pass p sorts digit (key >> shift) & mask.  One block = kSortChunk items;
// wave w owns the contiguous quarter of the chunk, walked in kSortIpt rounds
// of 64 (order = wave, round, lane: stable).  No global atomics: per-block
// digit counts -> per-digit row scan (+ row totals) -> the scatter derives
// the digit bases from the 256 totals itself.
// n_dev (a device-resident frame's tile sort, launched before T is known on
// the host): the items are min(*n_dev, n); n -- the capacity -- sizes the
// grid and nb stays the count table's row stride.  Blocks past the items
// leave at once; the scans run over the live blocks' columns only.
__device__ __forceinline__ int live_items(int n, const uint32_t *n_dev) {
  return n_dev ? (int)min((uint32_t)n, *n_dev) : n;
}

__global__ __launch_bounds__(kBlock) void k_radix_hist(const uint32_t *__restrict__ keys, int n, int shift,
                                                       int nbits, uint32_t *counts, int nb,
                                                       const uint32_t *n_dev = nullptr) {
  n = live_items(n, n_dev);
  if ((long long)blockIdx.x * kSortChunk >= n) return;
  __shared__ uint32_t hist[kRadix];
  hist[threadIdx.x] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t mask = (1u << nbits) - 1u;
  const long long base = (long long)blockIdx.x * kSortChunk + wave * (kSortChunk / 4);
  // all rounds' keys in one round trip: unconditional loads (clamped index;
  // a load under a branch is waited for at its join)
  uint32_t kr[kSortIpt];
#pragma unroll
  for (int r = 0; r < kSortIpt; ++r) {
    const long long idx = base + r * 64 + lane;
    kr[r] = keys[idx < n ? idx : n - 1];
  }
  // one LDS atomic per key (the LDS serialises equal addresses itself;
  // ballot-matched digit counts were 9 us slower on the tile sort)
#pragma unroll
  for (int r = 0; r < kSortIpt; ++r) {
    const long long idx = base + r * 64 + lane;
    if (idx < n) atomicAdd(&hist[(kr[r] >> shift) & mask], 1u);
  }
  __syncthreads();
  if (threadIdx.x <= mask) counts[(size_t)threadIdx.x * nb + blockIdx.x] = hist[threadIdx.x];
}

// row d of counts -> exclusive prefix over blocks; totals[d] = row sum.
// Thread t owns a contiguous run of `per` (<= kScanPer) entries of each
// 256 * per stretch (loads all in flight): one block scan per stretch (nb <=
// 4096, 8.4M keys: one) instead of one per 256 entries.
constexpr int kScanPer = 16;
__global__ __launch_bounds__(kBlock) void k_radix_scan(uint32_t *counts, uint32_t *totals, int nb,
                                                       const uint32_t *n_dev = nullptr) {
  __shared__ uint32_t s_tmp[4];
  const int d = blockIdx.x;
  uint32_t *row = counts + (size_t)d * nb;  // (row stride: the launch's nb)
  if (n_dev) nb = min(nb, (int)div_up_dev(*n_dev, kSortChunk));
  const int per = min(kScanPer, (nb + kBlock - 1) / kBlock);
  uint32_t carry = 0, tot;
  for (int c = 0; c < nb; c += kBlock * per) {
    const int i0 = c + (int)threadIdx.x * per;
    uint32_t v[kScanPer];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      v[k] = (k < per && i0 + k < nb) ? row[i0 + k] : 0u;
      sum += v[k];
    }
    uint32_t run = carry + block_exscan(sum, s_tmp, &tot);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      if (k < per && i0 + k < nb) row[i0 + k] = run;
      run += v[k];
    }
    carry += tot;
  }
  if (threadIdx.x == 0) totals[d] = carry;
}

template <bool kIota>  // values = input positions (the first pass of an iota-valued sort)
__global__ __launch_bounds__(kBlock) void k_radix_scatter(const uint32_t *__restrict__ keys_in,
                                                          const uint32_t *__restrict__ vals_in,
                                                          uint32_t *__restrict__ keys_out,
                                                          uint32_t *__restrict__ vals_out, int n, int shift,
                                                          int nbits, const uint32_t *counts,
                                                          const uint32_t *totals, int nb,
                                                          const uint32_t *n_dev = nullptr) {
  n = live_items(n, n_dev);
  if ((long long)blockIdx.x * kSortChunk >= n) return;
  __shared__ uint32_t wcnt[4][kRadix];
  __shared__ uint32_t s_lbase[kRadix];  // block-local start of each digit
  __shared__ uint32_t s_gbase[kRadix];  // global start of this block's run of each digit
  __shared__ uint32_t s_k[kSortChunk], s_v[kSortChunk];
  __shared__ uint32_t s_tmp[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int w = 0; w < 4; ++w) wcnt[w][threadIdx.x] = 0;
  const uint32_t mask = (1u << nbits) - 1u;
  const long long blk0 = (long long)blockIdx.x * kSortChunk;
  const long long base = blk0 + wave * (kSortChunk / 4);
  // all rounds' keys and values in one round trip (unconditional, clamped),
  // requested before the digit-base scan so that they fly during it
  uint32_t k_[kSortIpt], v_[kSortIpt];
#pragma unroll
  for (int r = 0; r < kSortIpt; ++r) {
    const long long idx = base + r * 64 + lane;
    const long long ci = idx < n ? idx : n - 1;
    k_[r] = keys_in[ci];
    v_[r] = kIota ? (uint32_t)idx : vals_in[ci];
  }
  // (also in flight; rows and totals exist for the pass's 2^nbits digits only)
  const bool dig = threadIdx.x <= mask;
  const uint32_t my_prefix = dig ? counts[(size_t)threadIdx.x * nb + blockIdx.x] : 0u;
  uint32_t tot;
  const uint32_t dbase = block_exscan(dig ? totals[threadIdx.x] : 0u, s_tmp, &tot);  // includes a barrier
  uint32_t rk[kSortIpt];
#pragma unroll
  for (int r = 0; r < kSortIpt; ++r) {
    const long long idx = base + r * 64 + lane;
    const bool valid = idx < n;
    const uint32_t key = valid ? k_[r] : 0u;
    const uint32_t val = valid ? v_[r] : 0u;
    const uint32_t d = (key >> shift) & mask;
    const unsigned long long m = match_digit(d, nbits, __ballot(valid));
    const uint32_t below = (uint32_t)__popcll(m & lanemask_lt());
    uint32_t old = 0;
    if (valid) old = wcnt[wave][d];
    if (valid && below == 0) wcnt[wave][d] = old + (uint32_t)__popcll(m);
    k_[r] = key;
    v_[r] = val;
    rk[r] = valid ? old + below : 0xFFFFFFFFu;
  }
  __syncthreads();
  {
    // per digit: wave prefixes inside the block, block count, then the
    // block-local digit start (scan over digits)
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t t = wcnt[w][threadIdx.x];
      wcnt[w][threadIdx.x] = run;
      run += t;
    }
    const uint32_t lb = block_exscan(run, s_tmp, &tot);  // barrier inside
    s_lbase[threadIdx.x] = lb;
    s_gbase[threadIdx.x] = dbase + my_prefix;
  }
  __syncthreads();
  // locally sorted chunk in LDS (stable: wave, round, lane order within a digit)
#pragma unroll
  for (int r = 0; r < kSortIpt; ++r) {
    if (rk[r] != 0xFFFFFFFFu) {
      const uint32_t d = (k_[r] >> shift) & mask;
      const uint32_t lp = s_lbase[d] + wcnt[wave][d] + rk[r];
      s_k[lp] = k_[r];
      s_v[lp] = v_[r];
    }
  }
  __syncthreads();
  // write out: consecutive threads -> consecutive positions of one digit run
  const int cnt = (int)min((long long)kSortChunk, (long long)n - blk0);
  for (int i = threadIdx.x; i < cnt; i += kBlock) {
    const uint32_t key = s_k[i];
    const uint32_t d = (key >> shift) & mask;
    const uint32_t dst = s_gbase[d] + (uint32_t)i - s_lbase[d];
    keys_out[dst] = key;
    vals_out[dst] = s_v[i];
  }
}

// Bucket sort after one MSD pass (gs_depth_sort_msd): workgroup d sorts the
// items whose top 8 key bits are d -- a contiguous, index-ordered run of the
// MSD pass's output -- by their low `lowbits` bits, in LDS, in place.  Stable
// LSD passes as in k_radix_scatter (wave w owns a contiguous segment, walked
// in rounds of 64; ballot match ranking), but the data stays in LDS between
// passes.  Bucket 255 holds the culled sentinel only (the caller's window
// keeps visible keys below 255 << lowbits) and is left as the MSD pass wrote
// it: index order, what the LSD sort gives equal keys.  A bucket over
// kMsdCap items is left unsorted and flagged: 0xFFFFFFFF in *overflow (the
// caller's depth-max word, so its window check fails and it sorts again).
constexpr int kMsdThreads = 1024;
constexpr int kMsdWaves = kMsdThreads / kWave;
constexpr int kMsdIpt = 16;
constexpr int kMsdCap = kMsdThreads * kMsdIpt;  // 16384 items: 128 KB of keys + values in LDS

// kWhole (gs_internal_small_sort): one workgroup sorts a whole array of
// n <= kMsdCap keys by their low `lowbits` bits -- the bucket is everything,
// read from keys / vals (vals NULL: the input positions) and written to
// keys_out / vals_out.  One launch instead of a radix sort's 3 per pass, for
// the small frames whose steps are bound by launches.
template <bool kWhole = false>
__global__ __launch_bounds__(kMsdThreads) void k_msd_bucket_sort(uint32_t *__restrict__ keys,
                                                               uint32_t *__restrict__ vals,
                                                               const uint32_t *__restrict__ totals, int lowbits,
                                                               uint32_t *overflow, uint32_t whole_n = 0u,
                                                               uint32_t *__restrict__ keys_out = nullptr,
                                                               uint32_t *__restrict__ vals_out = nullptr,
                                                               const uint32_t *whole_n_dev = nullptr) {
  if (kWhole && whole_n_dev) whole_n = min(whole_n, *whole_n_dev);  // (a device-resident frame's T)
  __shared__ uint32_t s_k[kMsdCap], s_v[kMsdCap];
  __shared__ uint32_t wcnt[kMsdWaves][kRadix];
  __shared__ uint32_t s_lbase[kRadix];
  __shared__ uint32_t s_tmp[4];
  __shared__ uint32_t s_seg[2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t d0 = blockIdx.x;  // the bucket (grid: 255; bucket 255 is never sorted)
  if (kWhole) {
    if (threadIdx.x == 0) {
      s_seg[0] = 0u;
      s_seg[1] = whole_n;
    }
  } else if (wave == 0) {
    // start = totals[0 .. d0) summed, size = totals[d0]
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t t = (uint32_t)(4 * lane + k);
      s += t < d0 ? totals[t] : 0u;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += (uint32_t)__shfl_xor((int)s, o, 64);
    if (lane == 0) {
      s_seg[0] = s;
      s_seg[1] = totals[d0];
    }
  }
  __syncthreads();
  const uint32_t start = s_seg[0], size = s_seg[1];
  if constexpr (kWhole) {
    if (size <= 1u) {
      if (threadIdx.x == 0 && size == 1u) {
        keys_out[0] = keys[0];
        vals_out[0] = vals ? vals[0] : 0u;
      }
      return;
    }
  } else if (size <= 1u) {
    return;
  }
  if (size > (uint32_t)kMsdCap) {
    if (threadIdx.x == 0) *overflow = 0xFFFFFFFFu;
    return;
  }
  // wave w: items [w seg, (w + 1) seg), seg a multiple of 64; order (wave, round, lane)
  const uint32_t seg = (size + kMsdThreads - 1) / kMsdThreads * kWave;
  const int rounds = (int)(seg / kWave);
  // every round's key and value requested at once: unconditional loads of a
  // clamped index (a load under a branch is waited for at its join)
  uint32_t k_[kMsdIpt], v_[kMsdIpt];
#pragma unroll
  for (int r = 0; r < kMsdIpt; ++r) {
    const uint32_t i = (uint32_t)wave * seg + (uint32_t)(r * kWave + lane);
    const uint32_t ic = (r < rounds && i < size) ? i : 0u;
    k_[r] = keys[start + ic];
    v_[r] = (kWhole && !vals) ? ic : vals[start + ic];
  }
  const int passes = (lowbits + kRadixBits - 1) / kRadixBits;
  int shift = 0;
  for (int p = 0; p < passes; ++p) {
    const int nbits = (lowbits - shift + (passes - p) - 1) / (passes - p);
    const uint32_t mask = (1u << nbits) - 1u;
    for (int t = threadIdx.x; t < kMsdWaves * kRadix; t += kMsdThreads) (&wcnt[0][0])[t] = 0u;
    __syncthreads();
    uint32_t rk[kMsdIpt];
#pragma unroll
    for (int r = 0; r < kMsdIpt; ++r) {
      rk[r] = 0xFFFFFFFFu;
      if (r < rounds) {  // wave-uniform
        const uint32_t i = (uint32_t)wave * seg + (uint32_t)(r * kWave + lane);
        const bool valid = i < size;
        const uint32_t dg = (k_[r] >> shift) & mask;
        const unsigned long long m = match_digit(dg, nbits, __ballot(valid));
        const uint32_t below = (uint32_t)__popcll(m & lanemask_lt());
        uint32_t old = 0;
        if (valid) old = wcnt[wave][dg];
        if (valid && below == 0) wcnt[wave][dg] = old + (uint32_t)__popcll(m);
        if (valid) rk[r] = old + below;
      }
    }
    __syncthreads();
    // per digit: wave prefixes, then the block-local digit start (scan over
    // the 256 digits by the first four waves)
    uint32_t run = 0;
    if (threadIdx.x < kRadix) {
      for (int w = 0; w < kMsdWaves; ++w) {
        const uint32_t t = wcnt[w][threadIdx.x];
        wcnt[w][threadIdx.x] = run;
        run += t;
      }
    }
    uint32_t incl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = (uint32_t)__shfl_up((int)incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (threadIdx.x < kRadix && lane == 63) s_tmp[wave] = incl;
    __syncthreads();
    if (threadIdx.x < kRadix) {
      uint32_t base = 0;
      for (int w = 0; w < wave; ++w) base += s_tmp[w];
      s_lbase[threadIdx.x] = base + incl - run;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kMsdIpt; ++r) {
      if (rk[r] != 0xFFFFFFFFu) {
        const uint32_t dg = (k_[r] >> shift) & mask;
        const uint32_t lp = s_lbase[dg] + wcnt[wave][dg] + rk[r];
        s_k[lp] = k_[r];
        s_v[lp] = v_[r];
      }
    }
    __syncthreads();
    shift += nbits;
    if (p + 1 < passes) {
#pragma unroll
      for (int r = 0; r < kMsdIpt; ++r) {
        const uint32_t i = (uint32_t)wave * seg + (uint32_t)(r * kWave + lane);
        const uint32_t ic = (r < rounds && i < size) ? i : 0u;  // (unconditional, as above)
        k_[r] = s_k[ic];
        v_[r] = s_v[ic];
      }
    }
  }
  uint32_t *ko = kWhole ? keys_out : keys, *vo = kWhole ? vals_out : vals;
  for (uint32_t i = threadIdx.x; i < size; i += kMsdThreads) {
    ko[start + i] = s_k[i];
    vo[start + i] = s_v[i];
  }
}

// ======================================================== binning =========
// The binning workspace: 5 nb words of per-block partials, then the
// depth-ordered rectangles (n uint2, 16-B aligned).
__device__ __forceinline__ uint2 *sorted_rects(uint32_t *partials, int nb) {
  return reinterpret_cast<uint2 *>(partials + ((5 * nb + 3) & ~3));
}

// partials[0..nb): touches per block (depth order), partials[nb..2nb): visible per index chunk,
// [2nb..3nb): index-order slots per chunk, [3nb..5nb): depth-bits min / max per chunk
// The tile sort's first-pass digit counts (k_radix_hist's table), built by
// k_bin_emit as it writes the entries (gs_internal_bin_emit_hist): the
// table, zeroed by k_bin_partials, the kernel before it in the stream.
struct TileHist {
  uint32_t *counts;     // [2^bits, nb_sort] (row d: digit d's count per sort block)
  uint32_t zero_words;  // words k_bin_partials clears: 2^bits * div_up(capacity, kSortChunk)
  int bits;             // first pass digit width (shift 0); 0: no table
};

__global__ __launch_bounds__(kBlock) void k_bin_partials(gs_bin_args a, uint32_t *partials, int nb, TileHist th) {
  __shared__ uint32_t s_tmp3[3][kBlock / kWave];
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < th.zero_words; i += gridDim.x * kBlock) th.counts[i] = 0u;
  const long long base = (long long)blockIdx.x * kBinChunk;
  constexpr int kR = kBinChunk / kBlock;
  // Loads unconditional (clamped index) and all rounds' at once: two round
  // trips (ids, then their rects/vis) instead of two per round -- a load
  // under a branch is waited for at the branch's join.  The index-order
  // rects of the second half are requested here too.
  uint32_t gi[kR];
  uint2 rc_own[kR];
#pragma unroll
  for (int i = 0; i < kR; ++i) {
    const long long k = base + i * kBlock + threadIdx.x;
    const long long kc = k < a.n ? k : a.n - 1;
    gi[i] = a.sorted_ids[kc];
    rc_own[i] = reinterpret_cast<const uint2 *>(a.rects)[kc];
  }
  uint32_t sum = 0, nvis = 0;
  uint2 rc_d[kR];
  uint32_t vis_o[kR];
#pragma unroll
  for (int i = 0; i < kR; ++i) {
    const long long k = base + i * kBlock + threadIdx.x;
    rc_d[i] = reinterpret_cast<const uint2 *>(a.rects)[gi[i]];
    vis_o[i] = a.vis[k < a.n ? k : a.n - 1];  // M is a total: counted in index order (coalesced)
  }
#pragma unroll
  for (int i = 0; i < kR; ++i) {
    const long long k = base + i * kBlock + threadIdx.x;
    if (k < a.n) {
      sum += rect_touches((int)(rc_d[i].x & 0xFFFFu), (int)(rc_d[i].x >> 16), (int)(rc_d[i].y & 0xFFFFu),
                          (int)(rc_d[i].y >> 16));
      nvis += vis_o[i] ? 1u : 0u;
    }
  }
  // Gradient slots are numbered in Gaussian-index order (a Gaussian's
  // touches consecutive), so that gs_project_backward's threads g, g+1 read
  // adjacent slot ranges: here each Gaussian's exclusive prefix of touches
  // inside this block's index chunk (k_bin_emit adds the chunk's offset).
  uint32_t cnt[kR];
#pragma unroll
  for (int i = 0; i < kR; ++i) {
    const long long g = base + i * kBlock + threadIdx.x;
    cnt[i] = g < a.n ? rect_touches((int)(rc_own[i].x & 0xFFFFu), (int)(rc_own[i].x >> 16),
                                    (int)(rc_own[i].y & 0xFFFFu), (int)(rc_own[i].y >> 16))
                     : 0u;
  }
  // the block's touches (depth order) and visible count, and round 0's slot
  // prefix, in one scan
  uint3 t3;
  const uint3 e3 = block_exscan3(make_uint3(sum, nvis, cnt[0]), s_tmp3, &t3);
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = t3.x;
    partials[nb + blockIdx.x] = t3.y;
  }
  // the depth-ordered rectangles, for k_bin_emit to read coalesced
  uint2 *srect = sorted_rects(partials, nb);
#pragma unroll
  for (int i = 0; i < kR; ++i) {
    const long long k = base + i * kBlock + threadIdx.x;
    if (k < a.n) srect[k] = rc_d[i];
  }
  // rounds 1..3's prefixes in one more scan (integer sums: any grouping)
  static_assert(kR == 4, "the slot prefix scans assume four rounds per binning block");
  uint3 u3;
  const uint3 f3 = block_exscan3(make_uint3(cnt[1], cnt[2], cnt[3]), s_tmp3, &u3);
  const uint32_t ex[kR] = {e3.z, f3.x, f3.y, f3.z};
  const uint32_t tt[kR] = {t3.z, u3.x, u3.y, u3.z};
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < kR; ++i) {
    const long long g = base + i * kBlock + threadIdx.x;
    if (g < a.n) a.pair_offset[g] = carry + ex[i];
    carry += tt[i];
  }
  if (threadIdx.x == 0) partials[2 * nb + blockIdx.x] = carry;
  // the projection blocks of this chunk (kBinChunk / kBlock of them): their
  // depth-bits min / max, folded for k_bin_scan_partials
  constexpr int kPB = kBinChunk / kBlock;
  if (threadIdx.x < kPB) {
    const int pb = blockIdx.x * kPB + threadIdx.x, npb = (a.n + kBlock - 1) / kBlock;
    const bool ok = pb < npb;
    uint32_t mn = ok ? a.key_minmax[2 * pb] : 0xFFFFFFFFu, mx = ok ? a.key_minmax[2 * pb + 1] : 0u;
#pragma unroll
    for (int d = 1; d < kPB; d <<= 1) {
      mn = min(mn, (uint32_t)__shfl_xor((int)mn, d, 64));
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
    }
    if (threadIdx.x == 0) {
      partials[3 * nb + blockIdx.x] = mn;
      partials[4 * nb + blockIdx.x] = mx;
    }
  }
}

// exclusive scan of the touch partials (single block); counters[0] = M, [1] = T,
// [2] / [3] = min / max visible depth bits (the projection's per-block values)
// The depth-key window held (rasterizer.window_holds): every visible bits(Z)
// - key_base below the window's limit -- 2^key_bits - 1, and 255 <<
// (key_bits - 8) from 9 bits on (gs_depth_sort_msd's sentinel bucket).
__device__ __forceinline__ bool window_held(uint32_t key_base, int key_bits, uint32_t zmin, uint32_t zmax) {
  if (key_bits <= 0 || key_bits >= 32 || zmin > zmax) return true;
  const uint64_t full = (1ull << key_bits) - 1ull;
  const uint64_t lim = key_bits >= 9 ? min(full, 255ull << (key_bits - 8)) : full;
  return zmin >= key_base && (uint64_t)(zmax - key_base) < lim;
}

__global__ __launch_bounds__(kBlock) void k_bin_scan_partials(gs_bin_args a, uint32_t *partials, int nb) {
  uint32_t *const counters = a.counters, *const host_counters = a.host_counters;
  __shared__ uint32_t s_tmp3[3][kBlock / kWave];
  __shared__ uint32_t s_mm[2][kBlock / kWave];
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
  uint32_t carry = 0, vis = 0, slots = 0;
  // a chunk's three partials loaded unconditionally (clamped index) and the
  // next chunk's in flight during this one's scans: no load waits under a
  // branch (the compiler waited for each conditional load at its join)
  auto ld = [&](int i, uint32_t *v) {
    const int ci = i < nb ? i : nb - 1;
    v[0] = partials[ci];
    v[1] = partials[nb + ci];
    v[2] = partials[2 * nb + ci];
    v[3] = partials[3 * nb + ci];
    v[4] = partials[4 * nb + ci];
  };
  uint32_t vn[5];
  ld((int)threadIdx.x, vn);
  for (int c = 0; c < nb; c += kBlock) {
    const int i = c + threadIdx.x;
    const uint32_t v0 = i < nb ? vn[0] : 0u, v1 = i < nb ? vn[1] : 0u, v2 = i < nb ? vn[2] : 0u;
    // (a clamped reload of the last chunk only repeats a value: harmless for min / max)
    mn = min(mn, vn[3]);
    mx = max(mx, vn[4]);
    ld(i + kBlock, vn);
    // touches (depth order), visible, index-order slot chunks (k_bin_partials):
    // exclusive offsets of the first and third in place
    uint3 t3;
    const uint3 e = block_exscan3(make_uint3(v0, v1, v2), s_tmp3, &t3);
    if (i < nb) {
      partials[i] = carry + e.x;
      partials[2 * nb + i] = slots + e.z;
    }
    carry += t3.x;
    vis += t3.y;
    slots += t3.z;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, d, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
  }
  if ((threadIdx.x & (kWave - 1)) == 0) {
    s_mm[0][threadIdx.x >> 6] = mn;
    s_mm[1][threadIdx.x >> 6] = mx;
  }
  __syncthreads();  // s_mm
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) {
      mn = min(mn, s_mm[0][w]);
      mx = max(mx, s_mm[1][w]);
    }
    // what a device-resident frame cannot do on the device (GS_FRAME_*): its
    // later stages see T_eff = 0 entries (empty lists, memory-safe)
    uint32_t status = 0u;
    if ((long long)carry > a.capacity) status |= GS_FRAME_NEED_CAPACITY;
    if (!window_held(a.key_base, a.key_bits, mn, mx)) status |= GS_FRAME_WINDOW_MISS;
    if (vis == 0u) status |= GS_FRAME_EMPTY;
    counters[0] = vis;
    counters[1] = carry;
    counters[2] = mn;
    counters[3] = mx;
    counters[4] = status;
    counters[5] = status ? 0u : carry;
    uint32_t seq = a.host_seq;
    if (a.frame_seq) {  // (one block, one thread: a plain increment)
      seq = *a.frame_seq + 1u;
      *a.frame_seq = seq;
    }
    // the sticky step flags: the first frame that sets them is recorded for
    // the host (its replays from there on updated nothing)
    uint32_t sticky = status;
    bool first_fail = status != 0u;
    if (a.step_flags) {
      const uint32_t old = atomicOr(a.step_flags, status);
      sticky = old | status;
      first_fail = old == 0u && status != 0u;
    }
    if (host_counters) {  // (M, T, depth range, status) straight to the host's pinned buffer
      host_counters[0] = vis;
      host_counters[1] = carry;
      host_counters[2] = mn;
      host_counters[3] = mx;
      host_counters[5] = status;
      host_counters[6] = sticky;
      if (first_fail) host_counters[7] = seq;
      __threadfence_system();  // the counters reach the host before the sequence word
      host_counters[4] = seq;
      __threadfence_system();
    }
  }
}

// Emission, coalesced: per round of 256 depth-ordered Gaussians, scan their
// touch counts into LDS and mark each output position with its Gaussian (a
// byte per position, a window of kOwnerCap positions at a time: one window
// per round unless the round's rectangles average more than 64 tiles); then
// every thread writes consecutive output entries, looking its Gaussian up in
// one LDS read (a binary search over the offsets took 8 dependent ones).
// Runs [lo, hi) longer than kWaveFillRun, flagged per lane by `wide`, are
// written by the wave's active lanes together, one run after another:
// fill(position, value of the lane that owns the run).  Every active lane of
// the wave must call it (ballots and shuffles inside, outside the divergent
// fill loop); lanes with nothing to fill pass wide = false.  Lanes that have
// already left the kernel (a partial last wave) take no part: the stride is
// the number of active lanes, not 64.
constexpr uint32_t kWaveFillRun = 32;
template <typename Fill>
__device__ __forceinline__ void wave_fill_runs(bool wide, uint32_t lo, uint32_t hi, uint32_t value, Fill fill) {
  unsigned long long m = __ballot(wide);
  if (!m) return;
  const unsigned long long act = __ballot(1);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nact = (uint32_t)__popcll(act), rank = (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
  while (m) {
    const int l = __ffsll(m) - 1;
    m &= m - 1;
    const uint32_t rlo = (uint32_t)__shfl((int)lo, l, 64), rhi = (uint32_t)__shfl((int)hi, l, 64);
    const uint32_t v = (uint32_t)__shfl((int)value, l, 64);
    for (uint32_t o = rlo + rank; o < rhi; o += nact) fill(o, v);
  }
}

constexpr uint32_t kOwnerCap = kBlock * 64;
// sort blocks a binning block's output may span with its digit counts in LDS
// (a block emits ~4.5 K entries at C3, ~3 sort blocks); counts past them go
// straight to the table
#ifndef GS_HIST_SPAN
#define GS_HIST_SPAN 8
#endif
constexpr int kHistSpan = GS_HIST_SPAN;
// kHist: the fused first-pass histogram (GS_EMIT_TILE_HIST, off); the product
// instantiation carries neither its LDS table nor its registers
template <bool kHist>
__global__ __launch_bounds__(kBlock) void k_bin_emit(gs_bin_args a, const uint32_t *partials, TileHist th) {
  __shared__ uint32_t s_off[kBlock + 1];
  __shared__ uint32_t s_g[kBlock];
  __shared__ uint2 s_rect[kBlock];
  __shared__ uint32_t s_tmp[4];
  __shared__ uint32_t s_tmp3[3][kBlock / kWave];
  __shared__ uint8_t s_owner[kOwnerCap];
  __shared__ uint32_t s_hist[kHist ? kHistSpan * kRadix : 1];
  const long long base = (long long)blockIdx.x * kBinChunk;
  // a device-resident frame that failed (gs_bin_count's status): no entry is
  // emitted and every rectangle of the chunk is cleared, so the frame's
  // backward gathers zero slots per Gaussian -- never a slot past the
  // capacity (the caller redoes the frame on the host path)
  if (a.device_counts && a.counters[4] != 0u) {
    for (int r = 0; r < kBinChunk / kBlock; ++r) {
      const long long g = base + r * kBlock + threadIdx.x;
      if (g < a.n) reinterpret_cast<uint2 *>(const_cast<uint32_t *>(a.rects))[g] = make_uint2(1u, 1u);
    }
    return;
  }
  // T entries do not fit: do nothing (the caller re-emits into T-sized
  // buffers; the slot pass below is not idempotent, so it must run once)
  const uint32_t T = a.counters[1];
  if ((long long)T > a.capacity) return;
  uint32_t out_base = partials[blockIdx.x];
  // first-pass digit counts of the entries this block writes: sort block
  // (out_base + o) / kSortChunk, digit key & hmask (shift 0)
  const bool hist = kHist && th.bits > 0;
  const uint32_t hmask = (1u << th.bits) - 1u, nbs = (T + kSortChunk - 1) / kSortChunk;
  const uint32_t hb0 = out_base / kSortChunk;
  if (hist) {
    for (int i = threadIdx.x; i < kHistSpan * kRadix; i += kBlock) s_hist[i] = 0u;
    // (ordered before the first use by the barriers inside the prefix scans)
  }
  constexpr int kR = kBinChunk / kBlock;
  // all rounds' ids and rects unconditionally (clamped): one round trip for
  // the block
  uint32_t gr[kR];
  uint2 rcr[kR];
  uint32_t offr[kR];
  const uint2 *srect = sorted_rects(const_cast<uint32_t *>(partials), (int)gridDim.x);
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const long long k = base + r * kBlock + threadIdx.x;
    const long long kc = k < a.n ? k : a.n - 1;
    gr[r] = a.sorted_ids[kc];
    rcr[r] = srect[kc];  // (k_bin_partials' depth-ordered copy: no gather by id)
    offr[r] = a.pair_offset[kc];  // (index order, for the slot pass below)
  }
  // every round's touch counts and their prefixes up front (three rounds in
  // one scan: the scans are latency-bound)
  static_assert(kR == 4, "the emission's prefix scans assume four rounds per binning block");
  uint32_t cntr[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const long long k = base + r * kBlock + threadIdx.x;
    if (k < a.n) {
      cntr[r] = rect_touches((int)(rcr[r].x & 0xFFFFu), (int)(rcr[r].x >> 16), (int)(rcr[r].y & 0xFFFFu),
                             (int)(rcr[r].y >> 16));
    } else {
      cntr[r] = 0u;
      gr[r] = 0xFFFFFFFFu;
      rcr[r] = make_uint2(1u, 1u);
    }
  }
  uint3 ta;
  uint32_t tb;
  const uint3 ea = block_exscan3(make_uint3(cntr[0], cntr[1], cntr[2]), s_tmp3, &ta);
  const uint32_t eb = block_exscan(cntr[3], s_tmp, &tb);
  const uint32_t exr[kR] = {ea.x, ea.y, ea.z, eb}, totr[kR] = {ta.x, ta.y, ta.z, tb};
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const uint32_t g = gr[r], cnt = cntr[r], ex = exr[r], tot = totr[r];
    const uint2 rc = rcr[r];
    if (r) __syncthreads();  // the previous round's owner-map and offset reads are done
    s_off[threadIdx.x] = ex;
    s_g[threadIdx.x] = g;
    s_rect[threadIdx.x] = rc;
    if (threadIdx.x == 0) s_off[kBlock] = tot;
    // (tot is block-uniform: every thread runs the same windows)
    for (uint32_t wb = 0; wb < tot; wb += kOwnerCap) {
      if (wb) __syncthreads();  // the previous window's owner reads are done
      const uint32_t lo_c = ex > wb ? ex : wb, hi_c = min(ex + cnt, wb + kOwnerCap);
      // short runs by their own lane; a wide rectangle's run (up to a whole
      // window) by its wave, 64 entries per step
      const bool wide = hi_c > lo_c + kWaveFillRun;
      if (!wide)
        for (uint32_t o = lo_c; o < hi_c; ++o) s_owner[o - wb] = (uint8_t)threadIdx.x;
      wave_fill_runs(wide, lo_c - wb, hi_c - wb, threadIdx.x, [&](uint32_t o, uint32_t owner) {
        s_owner[o] = (uint8_t)owner;
      });
      __syncthreads();
      const uint32_t wend = min(tot, wb + kOwnerCap);
      for (uint32_t o = wb + threadIdx.x; o < wend; o += kBlock) {
        const int lo = s_owner[o - wb];
        const uint2 rr = s_rect[lo];
        const uint32_t tx0 = rr.x & 0xFFFFu, ty0 = rr.y & 0xFFFFu;
        const uint32_t wt = (rr.x >> 16) - tx0 + 1u;
        const uint32_t loc = o - s_off[lo];
        const uint32_t row = loc / wt;
        const uint32_t key = (ty0 + row) * (uint32_t)a.tiles_x + tx0 + (loc - row * wt);
        a.tile_keys[out_base + o] = key;
        a.pair_gauss[out_base + o] = s_g[lo];
        if (hist) {
          const uint32_t sb = (out_base + o) / kSortChunk, d = key & hmask;
          if (sb - hb0 < (uint32_t)kHistSpan)
            atomicAdd(&s_hist[(sb - hb0) * kRadix + d], 1u);
          else
            atomicAdd(&th.counts[(size_t)d * nbs + sb], 1u);
        }
      }
    }
    out_base += tot;
  }
  if (hist) {
    __syncthreads();
    // (integer sums: the table is the same whatever order the blocks add in)
    for (int i = threadIdx.x; i < kHistSpan * kRadix; i += kBlock) {
      const uint32_t v = s_hist[i], sb = hb0 + (uint32_t)(i / kRadix), d = (uint32_t)(i % kRadix);
      if (v && sb < nbs && d <= hmask) atomicAdd(&th.counts[(size_t)d * nbs + sb], v);
    }
  }
  // Gradient slots, in Gaussian-index order over this block's index chunk
  // (coalesced): the chunk's offset + each Gaussian's prefix in the chunk
  // (k_bin_partials); the first slot is also kept in the record (word 10) for
  // the backward.  Records of culled Gaussians are never read.
  const uint32_t cbase = partials[2 * gridDim.x + blockIdx.x];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const long long g = base + r * kBlock + threadIdx.x;
    if (g < a.n) {
      const uint32_t slot = cbase + offr[r];
      a.pair_offset[g] = slot;
      a.records[(size_t)g * GS_RECORD_FLOATS + 10] = __uint_as_float(slot);
    }
  }
}

// Every tile's [start, end) from the tile-sorted keys, empty tiles included
// (no memset): position p in [0, T] is a boundary when key[p-1] != key[p]
// (key[-1] = -1, key[T] = num_tiles); it closes the previous tile, opens the
// next and writes the tiles in between as empty at p.
// Four consecutive positions per thread (the default tile's four-cell slot
// flags): one 16-B key load, the previous key from the neighbouring lane, one
// 16-B flag store.  Same writes as k_tile_ranges.
__global__ __launch_bounds__(kBlock) void k_tile_ranges4(gs_range_args a) {
  const long long p0 = 4 * ((long long)blockIdx.x * kBlock + threadIdx.x);
  const long long T = live_items(a.num_pairs, a.num_pairs_dev);
  if (p0 > T) return;
  const int lane = threadIdx.x & 63;
  uint4 k = make_uint4(0u, 0u, 0u, 0u);
  if (p0 + 3 < T) {
    k = reinterpret_cast<const uint4 *>(a.sorted_keys)[p0 / 4];
  } else {
    if (p0 < T) k.x = a.sorted_keys[p0];
    if (p0 + 1 < T) k.y = a.sorted_keys[p0 + 1];
    if (p0 + 2 < T) k.z = a.sorted_keys[p0 + 2];
  }
  // the key before p0: the previous lane's last one (its positions end at p0 - 1)
  uint32_t before = (uint32_t)__shfl_up((int)k.w, 1, 64);
  if (lane == 0) before = p0 > 0 ? a.sorted_keys[p0 - 1] : 0u;
  if (a.slot_live) {
    if (p0 + 3 < T)
      reinterpret_cast<uint4 *>(a.slot_live)[p0 / 4] = make_uint4(0u, 0u, 0u, 0u);
    else
      for (long long q = p0; q < T; ++q) reinterpret_cast<uint32_t *>(a.slot_live)[q] = 0u;
  }
  const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long p = p0 + i;
    const bool in = p <= T;  // (lanes past the end take part in the wave fills with nothing to fill)
    const long long prev = !in ? 0 : (p > 0 ? (long long)(i ? kk[i - 1] : before) : -1);
    const long long cur = !in ? 0 : (p < T ? (long long)kk[i] : (long long)a.num_tiles);
    const bool edge = in && cur != prev;
    if (edge && prev >= 0) a.ranges[2 * prev + 1] = (uint32_t)p;
    if (edge && cur < a.num_tiles) a.ranges[2 * cur] = (uint32_t)p;
    const uint32_t t0 = (uint32_t)(prev + 1), t1 = edge ? (uint32_t)cur : t0;
    const bool wide = edge && t1 > t0 + kWaveFillRun;
    if (edge && !wide)
      for (uint32_t t = t0; t < t1; ++t) a.ranges[2 * t] = a.ranges[2 * t + 1] = (uint32_t)p;
    wave_fill_runs(wide, t0, t1, (uint32_t)p, [&](uint32_t t, uint32_t q) { a.ranges[2 * t] = a.ranges[2 * t + 1] = q; });
  }
}

__global__ __launch_bounds__(kBlock) void k_tile_ranges(gs_range_args a) {
  const long long p = (long long)blockIdx.x * kBlock + threadIdx.x;
  a.num_pairs = live_items(a.num_pairs, a.num_pairs_dev);
  if (p > a.num_pairs) return;
  if (a.slot_live && p < a.num_pairs) {  // slot p's flags for the backward (coalesced)
    if (a.cells == 4)
      reinterpret_cast<uint32_t *>(a.slot_live)[p] = 0u;
    else if (a.cells == 1)
      a.slot_live[p] = 0;
    else
      for (int c = 0; c < a.cells; ++c) a.slot_live[p * a.cells + c] = 0;
  }
  const long long prev = p > 0 ? (long long)a.sorted_keys[p - 1] : -1;
  const long long cur = p < a.num_pairs ? (long long)a.sorted_keys[p] : (long long)a.num_tiles;
  const bool edge = cur != prev;
  if (edge && prev >= 0) a.ranges[2 * prev + 1] = (uint32_t)p;
  if (edge && cur < a.num_tiles) a.ranges[2 * cur] = (uint32_t)p;
  // the empty tiles in between: a short gap by its lane, a long one (a sparse
  // frame) by the wave, 64 tiles per step
  const uint32_t t0 = (uint32_t)(prev + 1), t1 = edge ? (uint32_t)cur : t0;
  const bool wide = t1 > t0 + kWaveFillRun;
  if (!wide)
    for (uint32_t t = t0; t < t1; ++t) a.ranges[2 * t] = a.ranges[2 * t + 1] = (uint32_t)p;
  wave_fill_runs(wide, t0, t1, (uint32_t)p, [&](uint32_t t, uint32_t q) { a.ranges[2 * t] = a.ranges[2 * t + 1] = q; });
}

// ======================================================== blend fwd =======
// Cells: a tile of edge L (GaussianRenderer.tile_size) is covered from its
// origin by QX x QX cells of 8x8 pixels, QX = ceil(L/8) (edge cells clipped
// to the tile); a wave renders one cell, lane l its pixel (l&7, l>>3), and
// blends the tile's whole list (renderer.py:302-319).  L = 16: the tile's
// four 8x8 quadrants.
struct CellGeom {
  int L, QX;
  __device__ explicit CellGeom(int tile_size) : L(tile_size), QX((tile_size + 7) >> 3) {}
  __device__ int cells() const { return QX * QX; }
};

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d, 64));
  return v;
}

// Records staged in LDS are read as 8-byte pairs: ds_read_b64 costs 2 LDS
// cycles per wave-instruction (broadcast), ds_read_b96 8 and ds_read_b128 4
// (MI355X_MICROARCH.md, LDS table): (mx,my) (q00,qo) (q11,o) | (r,g) (b,z).
__device__ __forceinline__ float2 lds_pair(const float2 *p) {
  // volatile keeps each pair its own ds_read_b64 (no merging into b128 / read2)
  typedef __attribute__((address_space(3))) const volatile unsigned long long lds_u64;
  const unsigned long long v = *(lds_u64 *)(p);
  return make_float2(__uint_as_float((uint32_t)v), __uint_as_float((uint32_t)(v >> 32)));
}

// Wave-level culling of list entries: false only if every pixel centre of
// the 8x8 box [x0, x0 + 7] x [y0, y0 + 7] provably has s > 23.1, i.e.
// exp(-s/2) < 1e-5 (the :336 skip): the cell's wave may pass the entry over
// without evaluating it (each lane's own exact test still decides the rest).
// The s <= L ellipse, L = 23.1 * 1.01, lies in the box |x - mx| <= sqrt(L Sxx),
// |y - my| <= sqrt(L Syy), Sigma = Q^-1 for the form Q = [[q00, qo/2],
// [qo/2, q11]] the blend evaluates.  The 1% margin covers the fp32 rounding of
// s: |s_fp32 - s| <= ~4u (q00 dx^2 + |qo dx dy| + q11 dy^2) <= 4u (tr + |qo|)
// tr / det * s, so conics with (tr + |qo|) tr > 1e4 det -- and
// non-positive-definite or NaN ones -- are never culled.
__device__ __forceinline__ bool cell_hit(float mx, float my, float q00, float qo, float q11, float x0, float y0) {
  const float q01 = 0.5f * qo;
  const float det = q00 * q11 - q01 * q01, tr = q00 + q11;
  if (!(tr > 0.f && det > 0.f && (tr + fabsf(qo)) * tr <= 1e4f * det)) return true;
  const float L = 23.1f * 1.01f;
  // v_rcp / v_sqrt (~1 ulp): far inside the 1% margin
  const float id = __builtin_amdgcn_rcpf(det);
  const float hx = __builtin_amdgcn_sqrtf(L * q11 * id), hy = __builtin_amdgcn_sqrtf(L * q00 * id);
  const bool box = mx + hx >= x0 && mx - hx <= x0 + 7.f && my + hy >= y0 && my - hy <= y0 + 7.f;
  if (!box) return false;
  // The ellipse's bounding box meets the cell: the minimum of s over the
  // cell's box decides (a tilted, elongated ellipse's bounding box is much
  // larger than it).  The mean inside the box: s = 0.  Otherwise the minimum
  // lies on an edge: per edge the 1-D minimiser of the quadratic, clamped to
  // the edge.  A point of the box is evaluated, so the fp32 value is s at a
  // feasible point up to rounding -- the same ~4u (tr + |qo|) tr / det
  // relative error as above, inside the 1% margin.
  const float ax0 = x0 - mx, ax1 = x0 + 7.f - mx, ay0 = y0 - my, ay1 = y0 + 7.f - my;
  if (ax0 <= 0.f && ax1 >= 0.f && ay0 <= 0.f && ay1 >= 0.f) return true;
  const float kx = -0.5f * qo * __builtin_amdgcn_rcpf(q11), ky = -0.5f * qo * __builtin_amdgcn_rcpf(q00);
  auto sv = [&](float dx, float dy) { return (dx * dx) * q00 + (qo * dx) * dy + (dy * dy) * q11; };
  const float e0 = sv(ax0, __builtin_amdgcn_fmed3f(kx * ax0, ay0, ay1));
  const float e1 = sv(ax1, __builtin_amdgcn_fmed3f(kx * ax1, ay0, ay1));
  const float e2 = sv(__builtin_amdgcn_fmed3f(ky * ay0, ax0, ax1), ay0);
  const float e3 = sv(__builtin_amdgcn_fmed3f(ky * ay1, ax0, ax1), ay1);
  return fminf(fminf(e0, e1), fminf(e2, e3)) <= L;
}

// Workgroup b -> (tile, cell) and the tile's list range: b, b+8, b+16, ...
// share an XCD (round-robin dispatch; placement is for speed only), so the Q
// cells of a tile read its records through one L2.  Grid: ceil(tiles / 8) *
// 8 Q.  Position (b / 8 / Q) * 8 + b % 8 is the tile.  tile >= num_tiles:
// padding, no range.  (A heaviest-first dispatch order saved 4-9 us per
// launch at C3 but cost ~14 us to sort: tools/variants/README.md.)  The
// range is clamped to the T list entries (scalar, free): a corrupt ranges
// table cannot make the kernels read past sorted_gauss; a -DGS_DEBUG=1 build
// also reports any range it had to clamp.
__device__ __forceinline__ void cell_tile(uint32_t b, int ncell, const uint32_t *ranges, int ntiles, uint32_t T,
                                          int &tile, int &quad, uint32_t &start, uint32_t &end) {
  const uint32_t grp = b >> 3;
  const uint32_t q = (uint32_t)ncell;
  quad = (int)(grp % q);
  tile = (int)((grp / q) * 8u + (b & 7u));
  start = end = 0u;
  if (tile < ntiles) {
    start = __builtin_amdgcn_readfirstlane(ranges[2 * tile]);
    end = __builtin_amdgcn_readfirstlane(ranges[2 * tile + 1]);
#if GS_DEBUG
    if ((end > T || start > end) && threadIdx.x == 0)
      printf("gsplat: tile %d range [%u, %u) outside the %u entries, clamped\n", tile, start, end, T);
#endif
    end = min(end, T);
    start = min(start, end);
  }
}

// Forward blend, one 64-lane workgroup per (tile, 8x8 cell), lane = pixel
// (compact footprints keep the per-pair branches coherent).  The cells of a
// tile run independently (no barrier): each stages its own batches of 64
// records in LDS (the next batch gathered into registers meanwhile), culls
// them against its own box (cell_hit, one ballot per batch) and walks the set
// bits.  Round 1 shared the staging between the four cells of a 16x16 tile
// in a 256-thread block and paid, at every barrier, for its busiest wave;
// here a cell's time is its own work, the records re-read per cell from the
// L2 the tile's cells share (8 us less at C3).  Control flow stays
// wave-uniform (ballots, scalar bit scans); per-lane decisions are
// predicates, and a skipped pair adds exact zeros: the :336 / :340 / :345
// skips are folded into the weight (a skipped pair gets ai = 0, hence
// c = (1 - A) * 0 = +0, and an accepted one c = (1 - A) * ai > 0 -- the
// reference's c exactly), v_cndmask selects instead of SGPR mask arithmetic.
// Each cell writes a liveness word per 64 entries for the backward
// (gs_blend_live_words).
// kCount: also count each pixel's contributing pairs (c > 0) into
// a.pair_counts -- a work counter for the measurement, off in the
// render path.  kT16: tile_size is the default 16 (its cell geometry folds to
// constants).
template <bool kCount, bool kT16>
__global__ __launch_bounds__(kWave) void k_blend_fwd(gs_blend_fwd_args a) {
  __shared__ float2 s_rec[kWave * 6];
  const CellGeom cg(kT16 ? GS_DEFAULT_TILE : a.cam.tile_size);
  const int ncell = cg.cells();
  int tile, quad;
  uint32_t start, end;
  cell_tile(blockIdx.x, ncell, a.ranges, a.tiles_x * a.tiles_y, (uint32_t)a.num_pairs, tile, quad, start, end);
  if (tile >= a.tiles_x * a.tiles_y) return;
  const int lane = threadIdx.x;
  const int cx0 = (quad % cg.QX) * 8, cy0 = (quad / cg.QX) * 8;  // the cell in its tile
  const int x0 = (tile % a.tiles_x) * cg.L + cx0, y0 = (tile / a.tiles_x) * cg.L + cy0;
  const int px = x0 + (lane & 7), py = y0 + (lane >> 3);
  const int W = a.cam.image_width, H = a.cam.image_height;
  const bool inside = cx0 + (lane & 7) < cg.L && cy0 + (lane >> 3) < cg.L && px < W && py < H;
  const float bg0 = a.cam.bg[0], bg1 = a.cam.bg[1], bg2 = a.cam.bg[2];
  float ar = bg0, ag = bg1, ab = bg2;  // out_rgb = bg (renderer.py:273)
  // a lane is done once A >= kAlphaStop (the :352 break); lanes outside the
  // tile or image start done
  float A = inside ? 0.f : 1.f, D = 0.f;
  uint32_t neval = 0, ncontrib = 0;
  // neval (1 + the last entry this lane evaluated while running, :352) is
  // kept lazily: `last` is that count for the running lanes of the last
  // evaluated entry (scalar), copied into a lane's neval only when it stops
  // (its bit leaves the running mask) -- two VALU less per evaluated entry
  uint32_t last = 0;
  unsigned long long runm = __builtin_amdgcn_ballot_w64(A < kAlphaStop);
  const float fx = (float)px, fy = (float)py;
  const float4 *recs = reinterpret_cast<const float4 *>(a.records);
  // liveness word of (this batch, this cell): see gs_blend_live_words
  // (no bitmap: the caller's budget; the backward then replays every entry)
  uint64_t *live = a.live_bits ? a.live_bits + (size_t)quad * a.live_words + start / 64u + (uint32_t)tile : nullptr;
  const uint64_t live_left = a.live_bits ? (uint64_t)a.live_words - (start / 64u + (uint32_t)tile) : 0u;
  float4 n0 = make_float4(0.f, 0.f, 0.f, 0.f), n1 = n0, n2 = n0;
  if (start + (uint32_t)lane < end) {
    const uint32_t gid = a.sorted_gauss[start + lane];
    n0 = recs[3 * (size_t)gid];
    n1 = recs[3 * (size_t)gid + 1];
    n2 = recs[3 * (size_t)gid + 2];
  }
  for (uint32_t b = start; b < end; b += kWave) {
    if (!wave_any(A < kAlphaStop)) break;  // every pixel of the cell done
    // stage the batch (this wave's own earlier reads precede these writes)
    float4 *d = reinterpret_cast<float4 *>(&s_rec[6 * lane]);
    d[0] = stage_conic0(n0);  // (the conic as -Q/2: the loop computes t = -s/2)
    d[1] = stage_conic1(n1);
    d[2] = n2;
    const bool hit = b + (uint32_t)lane < end && cell_hit(n0.x, n0.y, n0.z, n1.x, n0.w, (float)x0, (float)y0);
    const unsigned long long mw = __builtin_amdgcn_ballot_w64(hit);
    unsigned long long m = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(mw >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)mw);
    // the next batch's records in flight while this one composites
    // (fetching the ids a batch earlier, so that this is one round trip, was
    // measured: no change, profiles/r03/experiments.md)
    if (b + kWave + (uint32_t)lane < end) {
      const uint32_t gid = a.sorted_gauss[b + kWave + lane];
      n0 = recs[3 * (size_t)gid];
      n1 = recs[3 * (size_t)gid + 1];
      n2 = recs[3 * (size_t)gid + 2];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the staged records, for every lane
    unsigned long long livem = 0;  // entries some lane of this cell evaluated
    // (packing the hits at compile-time offsets, round 6, so that the loop
    // needs no per-entry address move: no change, profiles/r06/exp5/)
    while (m) {
      const uint32_t bit = (uint32_t)__builtin_ctzll(m);
      m &= ~(1ull << bit);
      uint32_t ja;
      asm volatile("v_mov_b32 %0, %1" : "=v"(ja) : "s"(bit * 48u));
      const float2 *rj = reinterpret_cast<const float2 *>(reinterpret_cast<const char *>(s_rec) + ja);
      const float2 pm = lds_pair(rj), pq = lds_pair(rj + 1), po = lds_pair(rj + 2);
      const float dx = fx - pm.x, dy = fy - pm.y;
      const float t = conic_s(dx, dy, pq.x, po.x, pq.y);  // -s/2 (:333; conic staged as -Q/2)
      const bool run = A < kAlphaStop;
      const unsigned long long rm = __builtin_amdgcn_ballot_w64(run);  // (the compare's own SGPR result)
      const bool lv = run && !(t < kSkipT);  // the :336 skip, decided on s
      if (wave_any(lv)) {
        livem |= 1ull << bit;
        if (rm != runm) {  // lanes stopped since the last evaluated entry (rare)
          asm volatile("" ::: "memory");  // a real branch: not if-converted into every entry
          if ((runm >> lane) & 1ull) neval = last;
          runm = rm;
        }
        last = b - start + bit + 1;
        const float w = sat01(exp_blend(t));             // :334
        const float ai = lv ? sat01(po.y * w) : 0.f;      // :339 (skips folded into the weight)
        const float c = (1.f - A) * ai;                   // :343-344
        const float2 prg = lds_pair(rj + 3), pbz = lds_pair(rj + 4);
        ar = __builtin_fmaf(c, prg.x, ar);
        ag = __builtin_fmaf(c, prg.y, ag);
        ab = __builtin_fmaf(c, pbz.x, ab);
        A = A + c;
        D = __builtin_fmaf(c, pbz.y, D);
        if constexpr (kCount) ncontrib += c > 0.f ? 1u : 0u;
      }
    }
    const uint64_t wi = (b - start) / 64u;
    if (lane == 0 && wi < live_left) live[wi] = livem;
  }
  if ((runm >> lane) & 1ull) neval = last;
  if (inside && A < kAlphaStop) neval = end - start;
  // the cell's last evaluated entry (the backward replays up to it): lanes
  // outside the tile or image evaluated none
  const uint32_t cstop = wave_max_u32(inside ? neval : 0u);
  if (lane == 0) a.cell_neval[(size_t)tile * ncell + quad] = cstop;
  if (!inside) return;
  const size_t HW = (size_t)W * H, p = (size_t)py * W + px;
  const float tb = 1.f - A;
  const float pr = ar + tb * bg0, pg = ag + tb * bg1, pb = ab + tb * bg2;  // :359,364
  a.image[p] = clamp01(pr);
  a.image[HW + p] = clamp01(pg);
  a.image[2 * HW + p] = clamp01(pb);
  a.alpha[p] = clamp01(A);
  a.depth[p] = D / (A + 1e-6f);  // :362
  // The backward's per-pixel state is these outputs plus one byte: which
  // clamps blocked (value outside [0, 1], NaN included).  An unblocked
  // channel's image is the composite itself and A never leaves [0, 1] (each
  // step adds c <= 1 - A, rounded), so alpha is A.
  a.pix_flags[p] = (uint8_t)((pr >= 0.f && pr <= 1.f ? 0u : 1u) | (pg >= 0.f && pg <= 1.f ? 0u : 2u) |
                             (pb >= 0.f && pb <= 1.f ? 0u : 4u) | (A >= 0.f && A <= 1.f ? 0u : 8u));
  if (a.pix_neval) a.pix_neval[p] = neval;
  if constexpr (kCount) a.pair_counts[p] = ncontrib;
}

// ======================================================== blend bwd =======
// One 64-lane workgroup per (tile, 8x8 quadrant); lane = pixel, as in the
// forward's waves.  Nothing couples the four quadrants of a tile (no
// barrier): each walks only the list entries its own pixels evaluated in the
// forward (the liveness bitmap, exact), in list order, and writes one partial
// gradient per (entry, quadrant); gs_project_backward sums a slot's quadrant
// partials.
//  A (pixel-parallel), per live entry: replay the pixel's front-to-back chain
//    -- bit-identical to the forward's decisions -- and put two scalars per
//    pixel into a group buffer: dop = dL/d opacity and the contribution
//    weight c, whose sign bit flags exp(-s/2) > 1 (the weight clamp then
//    blocks dL/ds).
//  B (entry-parallel), per chunk of up to kBwdGroup live entries of a
//    64-entry word (records still staged): lanes 8j..8j+7 sum
//    entry j's 64 pixels -- lane 8j + x takes column x, rows 0..7 -- into the
//    10 gradient values and reduce them with 3 DPP steps.
// The records of a 64-entry word's live entries are gathered lane-parallel
// one word ahead (registers), staged in LDS and read back as broadcasts.
// live entries per phase-B group: 8, lanes 8j .. 8j + 7 on entry j (4 groups
// of 16 lanes: +85 us, tools/variants/README.md)
constexpr int kBwdGroup = 8;
constexpr int kBwdLanes = kWave / kBwdGroup;  // lanes per entry in phase B
// Group buffer rows (dop, c) are padded to 72 float2: phase B's lanes 8j + x
// read row j at pixel x + 8r, and 72 puts rows j = 0..3 of a 32-lane half on
// distinct banks (a stride of 64 would be a 4-way conflict).
constexpr int kBwdRow = kWave + 8;

template <int CTRL>
__device__ __forceinline__ float dpp_row(float v) {
  // bound_ctrl: every pattern used here is a full permutation inside a row
  // (no invalid source lane), so it changes no value -- but it lets the
  // compiler fold the move into the add (v_add_f32_dpp); without it the
  // row_half_mirror step became v_mov 0 + v_mov_dpp + v_add
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
// Sum over the 8 lanes 8j..8j+7 (a DPP half row); each of them gets the sum.
__device__ __forceinline__ float oct_sum(float v) {
  v += dpp_row<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_row<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_row<0x141>(v);  // row_half_mirror: lane x <- lane 7 - x of its 8
  // (empty asm: keeps the last add next to its DPP move, where the two fold
  // into one v_add_f32_dpp, instead of being sunk into the storing lane's branch)
  asm volatile("" : "+v"(v));
  return v;
}

// An entry whose clamps provably never bind: opacity in [1e-20, 1] and a
// conic passing cell_hit's conditioning test (positive definite, fp32 s >= 0
// at every pixel).  Then exp(-s/2) <= 1 and o w <= 1, and an accepted pair
// has c = (1 - A) o w >= 0.005 * 1e-20 * 1e-5 > 0.
__device__ __forceinline__ bool simple_entry(float4 r0, float4 r1) {
  const float q00 = r0.z, q11 = r0.w, qo = r1.x, o = r1.y;
  const float q01 = 0.5f * qo;
  const float det = q00 * q11 - q01 * q01, tr = q00 + q11;
  return o >= 1e-20f && o <= 1.f && tr > 0.f && det > 0.f && (tr + fabsf(qo)) * tr <= 1e4f * det;
}


// One launch replays the cells [cell_begin, cell_begin + cell_count) of every
// tile (the caller's batch: all of them unless a tile's cells would make the
// [T, cells] partial buffer too large; each batch's partials are summed by
// gs_gather_partials before the next batch overwrites them).  kT16: the
// default tile, one batch of its four cells.
// Phase-A lane statistics (gs_blend_backward_lane_stats; the kStats
// instantiation only -- the product kernel carries none of it): per replayed
// (entry, cell), the lanes still running into it and the lanes whose pair
// contributes (c > 0), as two 65-bin histograms, and per workgroup the
// replays, the replays entered with >= 32 running lanes, and the sums of
// running and contributing lanes.
struct BwdStats {
  unsigned long long *hist;  // [2][65]: running lanes, contributing lanes per replay
  uint32_t *per_group;       // [grid][4]
};

template <bool kT16, bool kStats = false>
__global__ __launch_bounds__(kWave) void k_blend_bwd(gs_blend_bwd_args a, BwdStats stats = {nullptr, nullptr}) {
  __shared__ float2 s_dc[kBwdGroup][kBwdRow];  // per group entry and pixel: (dop, c)
  __shared__ uint32_t s_hist[kStats ? 2 * 65 : 1];
  uint32_t n_rep = 0, n_rep32 = 0, sum_run = 0, sum_con = 0;  // (kStats)
  if constexpr (kStats) {
    for (int i = threadIdx.x; i < 2 * 65; i += kWave) s_hist[i] = 0u;
    if (threadIdx.x < 4) stats.per_group[(size_t)blockIdx.x * 4 + threadIdx.x] = 0u;
  }
  __shared__ float4 s_pg[kWave];         // per pixel: dL/drgb (masked), dL/dD
  // the chunk's records (word 10 = slot), staged per chunk from registers:
  // 384 B instead of a word's 3 KB, for occupancy (LDS bounds it)
  __shared__ float2 s_wrec[kBwdGroup * 6];
  const CellGeom cg(kT16 ? GS_DEFAULT_TILE : a.cam.tile_size);
  const int ncell = kT16 ? cg.cells() : a.cell_count;  // partial groups of this batch
  const int cell0 = kT16 ? 0 : a.cell_begin;
  int tile, qb;
  uint32_t start, lend;
  cell_tile(blockIdx.x, ncell, a.ranges, a.tiles_x * a.tiles_y, (uint32_t)a.num_pairs, tile, qb, start, lend);
  if (tile >= a.tiles_x * a.tiles_y) return;
  const int quad = cell0 + qb;  // the cell in its tile; qb its partial group
  const int lane = threadIdx.x;
  const uint32_t tx = (uint32_t)(tile % a.tiles_x), ty = (uint32_t)(tile / a.tiles_x);
  const int cx0 = (quad % cg.QX) * 8, cy0 = (quad / cg.QX) * 8;  // the cell in its tile
  const int x0 = (int)tx * cg.L + cx0, y0 = (int)ty * cg.L + cy0;
  const int px = x0 + (lane & 7), py = y0 + (lane >> 3);
  const int W = a.cam.image_width, H = a.cam.image_height;
  const bool inside = cx0 + (lane & 7) < cg.L && cy0 + (lane >> 3) < cg.L && px < W && py < H;
  if (start >= lend) return;  // empty list: no gradient here (and no entry to read speculatively)
  const float4 *recs = reinterpret_cast<const float4 *>(a.records);
  // The prologue's loads in two round trips, without branches (a load under
  // a branch is waited for at its join): (1) the pixel's state and
  // cotangents, word 0's liveness word and its entries' Gaussian ids;
  // (2) speculatively every word-0 entry's record, not only the live ones.
  // Lanes outside the image / past the list read valid dummies (pixel 0,
  // entry 0), never used.
  // no bitmap (the caller's memory budget): every entry counts as live, and
  // the per-lane tests decide alone (slower, the same sums)
  const unsigned long long *lw =
      a.live_bits ? reinterpret_cast<const unsigned long long *>(a.live_bits) + (size_t)quad * a.live_words +
                        start / 64u + (uint32_t)tile
                  : nullptr;
  const unsigned long long w0 = lw ? lw[0] : ~0ull;
  const uint32_t gid0 = a.sorted_gauss[start + (uint32_t)lane < lend ? start + (uint32_t)lane : 0u];
  const size_t HW = (size_t)W * H;
  const size_t p = inside ? (size_t)py * W + px : 0;
  // the forward's outputs and clamp flags (k_blend_fwd): alpha is A, an
  // unblocked channel's image its composite
  const float im0 = a.image[p], im1 = a.image[HW + p], im2 = a.image[2 * HW + p];
  const float al = a.alpha[p], dep = a.depth[p];
  const uint32_t fl = a.pix_flags[p];
  const float gi0 = a.g_image[p], gi1 = a.g_image[HW + p], gi2 = a.g_image[2 * HW + p];
  const float gal = (a.g_alpha ? a.g_alpha : a.g_image)[p];
  const float gdp = (a.g_depth ? a.g_depth : a.g_image)[p];
  float4 r0 = recs[3 * (size_t)gid0], r1 = recs[3 * (size_t)gid0 + 1], r2 = recs[3 * (size_t)gid0 + 2];
  const float bg0 = a.cam.bg[0], bg1 = a.cam.bg[1], bg2 = a.cam.bg[2];
  // pixel cotangents through clamp / bg composite / depth normalisation
  // (selects, no branch: the compiler would sink the loads into it)
  const float At = inside ? al : 0.f;
  const float tb = 1.f - At;
  const float gR0 = (inside && !(fl & 1u)) ? gi0 : 0.f;
  const float gR1 = (inside && !(fl & 2u)) ? gi1 : 0.f;
  const float gR2 = (inside && !(fl & 4u)) ? gi2 : 0.f;
  // the accumulated colour without the background, where its gradient passes
  // (where it is blocked, gR = 0 and the value is not used)
  const float tr = inside ? im0 - tb * bg0 : 0.f, tg = inside ? im1 - tb * bg1 : 0.f;
  const float tbl = inside ? im2 - tb * bg2 : 0.f;
  const float Dt = inside ? dep * (At + 1e-6f) : 0.f;
  float gA = -gR0 * bg0 - gR1 * bg1 - gR2 * bg2;
  if (inside && a.g_alpha && !(fl & 8u)) gA += gal;
  const bool has_d = inside && a.g_depth;
  const float den = At + 1e-6f;
  const float gD = has_d ? gdp / den : 0.f;
  const float gAd = -gdp * Dt / (den * den);
  if (has_d) gA += gAd;
  // the cell's last evaluated entry: nothing past it carries gradient here
  const uint32_t wstop = __builtin_amdgcn_readfirstlane(a.cell_neval[(size_t)tile * cg.cells() + quad]);
  if (wstop == 0) return;
  s_pg[lane] = make_float4(gR0, gR1, gR2, gD);
  const float fx = (float)px, fy = (float)py;
  const float onemA = 1.f - At;
  // Suffix sums without per-channel state: with X_i = gR . col_i + gD z_i,
  //   sum_k gR_k (accT_k - acc_k) + gD (Dt - D) = K - P,
  //   K = gR . accT + gD Dt (per pixel),  P = gR . acc + gD D (running; acc starts at bg)
  // and dL/dalpha_i = T_i (X_i + (P - K + gA (1 - At)) / T_{i+1}) = T_i (X_i + (P + G0) / T_{i+1}).
  const float K = (gR0 * tr + gR1 * tg) + (gR2 * tbl + gD * Dt);
  const float G0 = __builtin_fmaf(gA, onemA, -K);
  // PG = P + G0 carried as one running sum (a gradient factor, no decision)
  float PG = ((gR0 * bg0 + gR1 * bg1) + gR2 * bg2) + G0;
  float A = 0.f, T1 = 1.f;  // T1 = 1 - A, carried: the next entry's transmittance is this one's rcp argument
  // running (A < 0.995 so far; lanes outside the image never run): replays
  // the forward's per-lane termination, so an entry past the pixel's n_eval
  // is never taken
  bool run = inside;
  const uint32_t nwords = (wstop + 63u) >> 6;
  // liveness word wd of this quadrant, cut at wstop (bits past it were never written)
  auto live_word = [&](uint32_t wd) -> unsigned long long {
    const unsigned long long w = wd == 0 ? w0 : (lw ? lw[wd] : ~0ull);
    // (readfirstlane returns int: widen through uint32_t, never sign-extend)
    const unsigned long long m =
        ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(w >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)w);
    const uint32_t rem = wstop - 64u * wd;
    return rem < 64u ? m & ((1ull << rem) - 1ull) : m;
  };
  // lane l gathers the record of entry 64 wd + l when that entry is live here
  auto fetch = [&](uint32_t wd, unsigned long long m) {
    if ((m >> lane) & 1ull) {
      const uint32_t gid = a.sorted_gauss[start + 64u * wd + (uint32_t)lane];
      r0 = recs[3 * (size_t)gid];
      r1 = recs[3 * (size_t)gid + 1];
      r2 = recs[3 * (size_t)gid + 2];
    }
  };
  // Phase B over a chunk: its k live entries, staged at s_wrec positions
  // 0 .. k - 1 (group order).
  auto phase_b = [&](auto masked_tag, int k) {
    constexpr bool kMasked = decltype(masked_tag)::value;
    // (the group buffer rows were written by this wave: waited for below)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int j = lane / kBwdLanes, col = lane % kBwdLanes;
    if (j < k) {
      const uint32_t e = (uint32_t)j;
      const float4 ia = reinterpret_cast<const float4 *>(s_wrec)[3 * e];  // mx my h00 h11 (h = -q/2)
      const float2 ib = s_wrec[6 * e + 2];                                // ho o
      const float q00 = -2.f * ia.z, q11 = -2.f * ia.w, qo = -2.f * ib.x;  // (exact)
      const uint32_t slot = __float_as_uint(s_wrec[6 * e + 5].x);
      const float hop = -0.5f * ib.y;
      // this lane's pixels (x0 + col, y0 + r): dx = bx, dy = by + (r - rc).
      // The row moments are taken about row rc of the column.  rc = 0 (moments
      // with constant weights r, r^2) unless the chunk holds a Gaussian with
      // sigma_y < 2 px: then rc is the column row nearest each mean (clamped),
      // else such a Gaussian's dy^2 sum cancels -- by^2 S0 + 2 by Soy + Soyy
      // with |by| up to 7 for a result of ~(0.05)^2 S0: 1e4 x fp32 rounding,
      // 1.7e-4 of the tensor's scale measured on a sub-pixel Gaussian (2e-6
      // recentred).  Always recentring cost +28 us per C3 step, this test +7.
      const float bx = (float)(x0 + col) - ia.x;
      const float q01h = 0.5f * qo;
      const bool small_y = q00 < 4.f * (q00 * q11 - q01h * q01h);  // Sigma_yy = q00 / det < 4
      float S0 = 0.f, Soy = 0.f, Soyy = 0.f, g5 = 0.f, g6 = 0.f, g7 = 0.f, g8 = 0.f, g9 = 0.f;
      float rc = 0.f;
      auto moments = [&](auto recenter_tag) {
        constexpr bool kRec = decltype(recenter_tag)::value;
        if constexpr (kRec)
          rc = __builtin_amdgcn_fmed3f(__builtin_rintf(ia.y - (float)y0), 0.f, (float)(kBwdGroup - 1));
#pragma unroll
        for (int r = 0; r < kBwdGroup; ++r) {
          const int p = col + 8 * r;  // phase A's lane of that pixel
          const float2 dc = s_dc[j][p];
          const float dop = dc.x, cs = dc.y;
          const float4 pg = s_pg[p];
          // dL/ds = hop dop: none where the weight clamp bound (sign bit of c)
          // or the pair was skipped (dop = 0 then); a simple entry's clamps
          // never bind.  The moments are summed over dop and scaled by the
          // entry's hop once, after the rows (2 VALU less per row; unmasked,
          // the opacity sum g5 is the moment S0 itself)
          const float ds = kMasked ? (cs > 0.f ? dop : 0.f) : dop;
          const float cw = fabsf(cs);
          S0 += ds;
          if constexpr (kRec) {
            const float w = (float)r - rc;  // exact: small integers
            Soy = __builtin_fmaf(ds, w, Soy);
            Soyy = __builtin_fmaf(ds, w * w, Soyy);
          } else if (r) {
            Soy = __builtin_fmaf(ds, (float)r, Soy);
            Soyy = __builtin_fmaf(ds, (float)(r * r), Soyy);
          }
          if constexpr (kMasked) g5 += dop;
          g6 = __builtin_fmaf(pg.x, cw, g6);
          g7 = __builtin_fmaf(pg.y, cw, g7);
          g8 = __builtin_fmaf(pg.z, cw, g8);
          g9 = __builtin_fmaf(pg.w, cw, g9);
        }
      };
      if (wave_any(small_y)) moments(std::true_type{}); else moments(std::false_type{});
      if constexpr (!kMasked) g5 = S0;
      S0 *= hop;
      Soy *= hop;
      Soyy *= hop;
      const float by = (float)y0 + rc - ia.y;
      // sums of ds dx, ds dy, ds dx^2, ds dx dy, ds dy^2 over the lane's column
      float Sx = bx * S0, Sy = __builtin_fmaf(by, S0, Soy);
      float g2 = bx * Sx, g3 = bx * Sy;
      float g4 = __builtin_fmaf(by, __builtin_fmaf(by, S0, 2.f * Soy), Soyy);
      Sx = oct_sum(Sx); Sy = oct_sum(Sy); g2 = oct_sum(g2); g3 = oct_sum(g3); g4 = oct_sum(g4);
      g5 = oct_sum(g5); g6 = oct_sum(g6); g7 = oct_sum(g7); g8 = oct_sum(g8); g9 = oct_sum(g9);
      if (col == 0) {
        // dmu = -(2 q00 Sx + qo Sy, qo Sx + 2 q11 Sy)
        const float g0 = -(2.f * q00 * Sx + qo * Sy), g1 = -(qo * Sx + 2.f * q11 * Sy);
        const size_t sq = (size_t)slot * (uint32_t)ncell + (uint32_t)qb;
        // (dense 40-B partials, 8-B aligned: f4_u8)
        float *out = a.pair_grads + sq * GS_PARTIAL_STRIDE;
        *reinterpret_cast<f4_u8 *>(out) = f4_u8{g0, g1, g2, g3};
        *reinterpret_cast<f4_u8 *>(out + 4) = f4_u8{g4, g5, g6, g7};
        *reinterpret_cast<f2_u8 *>(out + 8) = f2_u8{g8, g9};
        a.slot_live[sq] = 1;
      }
    }
  };
  unsigned long long mcur = live_word(0);  // (word 0's records are in flight already)
  for (uint32_t wd = 0; wd < nwords; ++wd) {
    // word 10 of a live record becomes the entry's gradient slot (the
    // Gaussian's first slot + this tile's index in its rectangle)
    const bool mine = (mcur >> lane) & 1ull;
    const uint32_t info = __float_as_uint(r2.w);
    const uint32_t slot = __float_as_uint(r2.z) + (ty - ((info >> 12) & 0xFFFu)) * ((info >> 24) + 1u) +
                          (tx - (info & 0xFFFu));
    // packed: the live entry of rank r (bit order) at position r, so a
    // chunk's records sit at compile-time offsets from one base address
    const uint32_t rank =
        __builtin_amdgcn_mbcnt_hi((uint32_t)(mcur >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mcur, 0u));
    // this word's records stay in registers (staged chunk by chunk below)
    // while the next word's are fetched into r0..r2 (staging a whole word's
    // records, 3 KB of LDS, cost occupancy: -13 us when chunked)
    // (the conic staged as -Q/2: phase A computes t = -s/2; phase B undoes it)
    const float4 c0 = stage_conic0(r0), c1 = stage_conic1(r1), c2 = make_float4(r2.x, r2.y, __uint_as_float(slot), 0.f);
    const unsigned long long simple_w = __builtin_amdgcn_ballot_w64(mine && simple_entry(r0, r1));
    const unsigned long long mnext = wd + 1u < nwords ? live_word(wd + 1u) : 0ull;
    fetch(wd + 1u, mnext);  // in flight while this word replays
    // a word whose live entries are all simple (the common case) runs a copy
    // of the loop without the per-entry test
    auto run_word = [&](auto all_simple_tag) {
    constexpr bool kAllSimple = decltype(all_simple_tag)::value;
    unsigned long long m = mcur;
    uint32_t kb = 0;  // packed position of the chunk's first entry
    while (m) {
     // a chunk: the word's next (up to) kBwdGroup live entries
     unsigned long long cm = 0;
     int k = 0;
     // stage the chunk (ranks kb .. kb + kBwdGroup - 1; the previous chunk's
     // reads came before these writes in this wave's in-order LDS queue)
     if (mine && rank - kb < (uint32_t)kBwdGroup) {
       float4 *d = reinterpret_cast<float4 *>(&s_wrec[6 * (rank - kb)]);
       d[0] = c0;
       d[1] = c1;
       d[2] = c2;
     }
     asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the staged records, for every lane
     const char *cb = reinterpret_cast<const char *>(s_wrec);
     // unrolled: the group row k is a compile-time LDS offset
#pragma unroll
     for (int kk = 0; kk < kBwdGroup; ++kk) {
      if (kk > 0 && !m) break;
      const uint32_t bit = (uint32_t)__builtin_ctzll(m);
      m &= m - 1ull;
      cm |= 1ull << bit;
      // two b128 broadcasts and a b64: (mx my h00 h11) (ho o r g) (b z), h = -q/2;
      // pq = (h00, h11), po = (ho, opacity)
      const float4 r0v = reinterpret_cast<const float4 *>(cb + 48 * kk)[0];
      const float4 r1v = reinterpret_cast<const float4 *>(cb + 48 * kk)[1];
      const float2 pbz = reinterpret_cast<const float2 *>(cb + 48 * kk)[4];
      const float2 pm = make_float2(r0v.x, r0v.y), pq = make_float2(r0v.z, r0v.w);
      const float2 po = make_float2(r1v.x, r1v.y), prg = make_float2(r1v.z, r1v.w);
      const float dx = fx - pm.x, dy = fy - pm.y;
      const float tq = conic_s(dx, dy, pq.x, po.x, pq.y);  // -s/2, as in the forward
      // the w < 1e-5 skip on s, as in the forward (NaN falls through); `run`
      // is the forward's "A < 0.995 before this entry", carried from the
      // previous entry's own test -- the same decisions as i < n_eval
      const bool live = run && !(tq < kSkipT);
      uint32_t n_run = 0;
      if constexpr (kStats) n_run = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(run));
      const float X = __builtin_fmaf(gR0, prg.x, __builtin_fmaf(gR1, prg.y, __builtin_fmaf(gR2, pbz.x, gD * pbz.y)));
      const bool simple = kAllSimple || ((simple_w >> bit) & 1ull);
      float dop, cw;
      if (simple) {
        // Fast path (simple_entry): e = exp(-s/2) lies in [0, 1] (s >= 0) and
        // u = o w in [0, 1], so both clamps are identities and pass their
        // gradients -- the general path below with its clamp tests removed,
        // the same values.  wv = 0 exactly where the pair is skipped.
        const float w = exp_blend(tq);
        const float wv = live ? w : 0.f;
        const float trans = T1;
        const float c = trans * (po.y * wv);
        A = A + c;
        PG = __builtin_fmaf(c, X, PG);
        T1 = 1.f - A;
        const float inv = __builtin_amdgcn_rcpf(T1);  // v_rcp_f32 (1 ulp): a gradient factor, no decision
        const float d_live = __builtin_fmaf(inv, PG, X);
        // the terminating contributor has nothing behind it: (1-A_total)/T_{i+1} = 1
        const bool stop = !(A < kAlphaStop);
        const float dal = trans * (stop ? X + gA : d_live);
        run = run && !stop;
        dop = dal * wv;
        cw = c;
      } else {
        const float e = exp_blend(tq);
        const float w = sat01(e);
        const float u = po.y * w;
        const float ai = sat01(u);
        const float trans = T1;
        // the forward's skips folded into the weight exactly as there: c is
        // +0 for a skipped pair and > 0 for an accepted one (take <=> c > 0)
        const float c = trans * (live ? ai : 0.f);
        A = A + c;
        PG = __builtin_fmaf(c, X, PG);
        const bool term = !(A < kAlphaStop);
        T1 = 1.f - A;
        // both arms computed, then a select: no divergent branch per entry
        const float inv = __builtin_amdgcn_rcpf(T1);
        const float d_live = __builtin_fmaf(inv, PG, X);
        const float dal = trans * (term ? X + gA : d_live);
        run = run && !term;
        // u = o*w >= 0, so "u in [0,1]" (the clamp passes the gradient) is ai == u;
        // e = exp(.) >= 0, so "e in [0,1]" is w == e (both false for NaN)
        const float g = (ai == u) ? dal * w : 0.f;
        dop = (c > 0.f) ? g : 0.f;
        cw = (w == e) ? c : -c;  // c == +0 when skipped
      }
      s_dc[kk][lane] = make_float2(dop, cw);
      k = kk + 1;
      if constexpr (kStats) {
        const uint32_t n_con = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(cw != 0.f));
        if (lane == 0) {
          atomicAdd(&s_hist[n_run], 1u);
          atomicAdd(&s_hist[65 + n_con], 1u);
        }
        n_rep += 1u;
        n_rep32 += n_run >= 32u ? 1u : 0u;
        sum_run += n_run;
        sum_con += n_con;
      }
     }
     if (kAllSimple || (simple_w & cm) == cm) phase_b(std::false_type{}, k); else phase_b(std::true_type{}, k);
     kb += (uint32_t)k;
    }
    };
    if ((simple_w & mcur) == mcur) run_word(std::true_type{}); else run_word(std::false_type{});
    mcur = mnext;
  }
  if constexpr (kStats) {
    __syncthreads();
    if (lane == 0) {
      uint32_t *pg = stats.per_group + (size_t)blockIdx.x * 4;
      pg[0] = n_rep;
      pg[1] = n_rep32;
      pg[2] = sum_run;
      pg[3] = sum_con;
    }
    for (int i = lane; i < 2 * 65; i += kWave)
      if (s_hist[i]) atomicAdd(&stats.hist[i], (unsigned long long)s_hist[i]);
  }
}

// ======================================================== project bwd =====
// Sum of each Gaussian's gradient partials: QL x HL lanes per Gaussian, lane
// (h, q) walks g's slots h, h+HL, h+2HL, ... of [pair_offset[g],
// pair_offset[g] + touches) and adds the partial groups q, q + QL, ... of
// each (ng per slot: gs_partial_groups) that slot_live flags (slot order),
// then the lane sums are added in a fixed DPP order -- bitwise reproducible.
// The q lanes of a slot read its partial record together, and consecutive
// Gaussians' slots are adjacent (index-order slots): coalesced.  Flags of up
// to kGatherNB slots are loaded at once, then their partials: two round trips
// per kGatherNB x HL slots of g (the mean is 4.4 on C3).  Partials are 40 B, 8-B aligned:
// read as float2.
__device__ __forceinline__ float quad_sum(float v) {
  v += dpp_row<0xB1>(v);  // quad_perm [1,0,3,2]
  v += dpp_row<0x4E>(v);  // quad_perm [2,3,0,1]
  asm volatile("" : "+v"(v));
  return v;
}
template <int LPG>
__device__ __forceinline__ float lanes_sum(float v) {
  if constexpr (LPG == 8) return oct_sum(v);
  if constexpr (LPG == 4) return quad_sum(v);
  if constexpr (LPG == 2) {
    v += dpp_row<0xB1>(v);
    asm volatile("" : "+v"(v));
    return v;
  }
  return v;
}

constexpr int kGatherHL1 = 4;  // slot lanes per Gaussian with one partial group per slot

constexpr int kF2 = GS_PAIR_GRAD_FLOATS / 2;

// Gaussian g's partials summed by its QL x HL lanes (lane (h, q) of g at
// t % LPG); every one of the LPG lanes returns the sum in acc.
// Slots per lane per round trip: 3 (56 VGPRs, 8 waves per SIMD) against 4
// (71, 7 waves): 110.9 -> 105.9 us at C3 (profiles/r05/gather_nb_ab/); the
// lane's slot order, and so every sum, is the same for any batch size.
#ifndef GS_GATHER_NB
#define GS_GATHER_NB 3
#endif
constexpr int kGatherNB = GS_GATHER_NB;
// Gather mode (compile time: a runtime test costs the latency-bound gather
// ~5 us at C3, measured for a status word's scalar load on every wave's path):
// kGatherOrder -- the Gaussians walked in gs_project_bwd_args.order.  (A
// failed device-resident frame needs no test here: its emission cleared the
// rectangles, so every Gaussian gathers zero slots, gs_bin_args.device_counts.)
constexpr int kGatherOrder = 2;
template <int QL, int HL, int kNG, int kMode>
__device__ __forceinline__ void gather_slots(const gs_project_bwd_args &a, uint32_t ng, long long t, int g,
                                             float2 acc[kF2]) {
  constexpr int LPG = QL * HL;
  static_assert(LPG == 2 || LPG == 4 || LPG == 8, "lanes per Gaussian");
  const int h = (int)((t % LPG) / QL), q = (int)(t % QL);
#pragma unroll
  for (int k = 0; k < kF2; ++k) acc[k] = make_float2(0.f, 0.f);
  // vis, rect and first slot in one round trip (the empty asm keeps the
  // slot load beside the others: used only under the branch, the compiler
  // would issue it after the vis test, a second round trip)
  const bool valid = g < a.g.n;
  const uint32_t gi = valid ? (uint32_t)g : 0u;
  const uint32_t visb = a.vis[gi];
  int tx0, tx1, ty0, ty1;
  unpack_rect(a.rects, gi, tx0, tx1, ty0, ty1);
  uint32_t off32 = a.pair_offset[gi];
  asm volatile("" : "+v"(off32));
  const uint32_t cnt = (valid && visb) ? rect_touches(tx0, tx1, ty0, ty1) : 0u;
  // lane q sums partial groups q, q + QL, ... of a slot's ng (one pass when ng <= QL)
  for (uint32_t qc = (uint32_t)q; cnt > (uint32_t)h && qc < ng; qc += QL) {
    const size_t off = off32;
    const uint8_t *flag = a.slot_live + off * ng + qc;  // (slot e, group qc) at flag[ng e]
    // group-qc partial of slot e at part + e * ng * GS_PARTIAL_STRIDE (dense 40-B records)
    const float2 *part = reinterpret_cast<const float2 *>(a.pair_grads + (off * ng + qc) * GS_PARTIAL_STRIDE);
    for (uint32_t e0 = (uint32_t)h; e0 < cnt; e0 += kGatherNB * HL) {
      // the batch's flags in one round trip: unconditional loads (past the end
      // the clamped index re-reads slot e0), masked after
      uint32_t f[kGatherNB];
#pragma unroll
      for (int i = 0; i < kGatherNB; ++i) {
        const uint32_t e = e0 + HL * i;
        f[i] = flag[(size_t)ng * (e < cnt ? e : e0)];
      }
      // all the batch's flags tested before any partial is requested: the partial
      // loads are conditional, so a wait for a later flag placed between them
      // would have to count them out conservatively and drain them
      uint32_t fm = 0;
#pragma unroll
      for (int i = 0; i < kGatherNB; ++i) fm |= (e0 + HL * i < cnt && f[i]) ? 1u << i : 0u;
      asm volatile("" : "+v"(fm));
#pragma unroll
      for (int i = 0; i < kGatherNB; ++i) f[i] = (fm >> i) & 1u;
      f4_u8 va[kGatherNB], vb[kGatherNB];
      f2_u8 vc[kGatherNB];
#pragma unroll
      for (int i = 0; i < kGatherNB; ++i) {
        const float *src = reinterpret_cast<const float *>(part + (size_t)(e0 + HL * i) * ng * kF2);
        // (non-temporal loads, for data read once, measured +10 us: profiles/r03/experiments.md)
        va[i] = f[i] ? *reinterpret_cast<const f4_u8 *>(src) : f4_u8{0.f, 0.f, 0.f, 0.f};
        vb[i] = f[i] ? *reinterpret_cast<const f4_u8 *>(src + 4) : f4_u8{0.f, 0.f, 0.f, 0.f};
        vc[i] = f[i] ? *reinterpret_cast<const f2_u8 *>(src + 8) : f2_u8{0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < kGatherNB; ++i) {
        if (!f[i]) continue;
        acc[0].x += va[i].x; acc[0].y += va[i].y; acc[1].x += va[i].z; acc[1].y += va[i].w;
        acc[2].x += vb[i].x; acc[2].y += vb[i].y; acc[3].x += vb[i].z; acc[3].y += vb[i].w;
        acc[4].x += vc[i].x; acc[4].y += vc[i].y;
      }
    }
  }
  // the lane sums in a fixed DPP order, on every lane of the Gaussian's LPG
#pragma unroll
  for (int k = 0; k < kF2; ++k) {
    acc[k].x = lanes_sum<LPG>(acc[k].x);
    acc[k].y = lanes_sum<LPG>(acc[k].y);
  }
}

// accumulate: grad_sums = grad_sums + this batch's sums (the cell batches of
// one backward, added in batch order: deterministic), else grad_sums = them.
template <int QL, int HL, int kNG = 0, int kMode = 0>  // kNG > 0: the partial groups per slot at compile time (else ng)
__global__ __launch_bounds__(kBlock) void k_gather_slots(gs_project_bwd_args a, uint32_t ng_rt, int accumulate) {
  constexpr int LPG = QL * HL;
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  int g = (int)(t / LPG);
  if ((kMode & kGatherOrder) && g < a.g.n) g = (int)a.order[g];  // (gs_project_bwd_args.order)
  float2 acc[kF2];
  gather_slots<QL, HL, kNG, kMode>(a, kNG > 0 ? (uint32_t)kNG : ng_rt, t, g, acc);
  if ((t % LPG) == 0 && g < a.g.n) {
    float2 *out = reinterpret_cast<float2 *>(a.grad_sums) + (size_t)g * kF2;
    if (accumulate) {
#pragma unroll
      for (int k = 0; k < kF2; ++k) {
        const float2 o = out[k];
        out[k] = make_float2(o.x + acc[k].x, o.y + acc[k].y);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kF2; ++k) out[k] = acc[k];
    }
  }
}

// Gaussian g's chain rule from its summed blend gradients: sums(acc) fills
// acc[10] (from k_gather_slots' [n, 10] sums, or the fused gather's LDS)
// Where project_bwd_one's gradients go: out(tensor, g, k, gradient,
// parameter value) for element k of Gaussian g's row -- the gradient arrays
// (GradsOut), or, with the optimizer fused into the backward, a register
// buffer whose Adam update flush() applies once the row is complete
// (AdamOut).
enum : int { kOutXyz = 0, kOutColor = 1, kOutOpacity = 2, kOutScaling = 3, kOutRotation = 4, kOutCov = 5 };
struct GradsOut {
  const gs_project_bwd_args &a;
  __device__ __forceinline__ void operator()(int t, int g, int k, float grad, float) const {
    switch (t) {
      case kOutXyz: a.d_xyz[3 * (size_t)g + k] = grad; break;
      case kOutColor: a.d_color_logits[3 * (size_t)g + k] = grad; break;
      case kOutOpacity: a.d_opacity[g] = grad; break;
      case kOutScaling: a.d_scaling[3 * (size_t)g + k] = grad; break;
      case kOutRotation: a.d_rotation[4 * (size_t)g + k] = grad; break;
      default: a.d_cov3d[9 * (size_t)g + k] = grad; break;
    }
  }
};

// gs_project_backward_adam: FusedAdam's update (k_adam's arithmetic, the same
// fp32 operations in the same order) applied to the 14 parameters of a
// Gaussian once its gradients are formed; the parameter value is the one the
// chain rule read.  Tensors in the kOut* order; skip: a failed
// device-resident frame updates nothing.
struct FusedAdamArgs {
  float *param_out[5], *exp_avg[5], *exp_avg_sq[5];
  float lr[5], bc1[5], bc2s[5];
  float beta1, beta2, eps;
  const uint32_t *skip_flag;
  const float *hyper;        // [row][GS_ADAM_MAX_TENSORS][3] (gs_adam_args.hyper) or NULL
  const uint32_t *hyper_row;
  int hyper_slot[5];         // the tensor's slot in a hyper row
};
constexpr int kAdamRow[5] = {3, 3, 1, 3, 4};   // floats per Gaussian, kOut* order
constexpr int kAdamOff[6] = {0, 3, 6, 7, 10, 14};
struct AdamOut {
  float gv[14], pv[14];  // the row's gradients and parameter values (registers after unrolling)
  __device__ __forceinline__ void operator()(int t, int, int k, float grad, float p) {
    if (t > kOutRotation) return;  // (no covariance input on the fused path)
    gv[kAdamOff[t] + k] = grad;
    pv[kAdamOff[t] + k] = p;
  }
  // every m and v of the row requested in one round trip, then the updates
  __device__ __forceinline__ void flush(const FusedAdamArgs &f, int g) const {
    const uint32_t row = f.hyper ? *f.hyper_row : 0u;
    float m[14], v[14];
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int k = 0; k < kAdamRow[t]; ++k) {
        const size_t i = (size_t)kAdamRow[t] * g + k;
        m[kAdamOff[t] + k] = f.exp_avg[t][i];
        v[kAdamOff[t] + k] = f.exp_avg_sq[t][i];
      }
    const float om1 = 1.f - f.beta1, om2 = 1.f - f.beta2;
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      float lr = f.lr[t], bc1 = f.bc1[t], b2s = f.bc2s[t];
      if (f.hyper) {
        const float *h = f.hyper + ((size_t)row * GS_ADAM_MAX_TENSORS + f.hyper_slot[t]) * 3;
        lr = h[0];
        bc1 = h[1];
        b2s = h[2];
      }
      const float step = lr / bc1;
#pragma unroll
      for (int k = 0; k < kAdamRow[t]; ++k) {
        const int j = kAdamOff[t] + k;
        const size_t i = (size_t)kAdamRow[t] * g + k;
        const float gr = gv[j];
        const float mm = m[j] + om1 * (gr - m[j]);
        const float vv = f.beta2 * v[j] + om2 * (gr * gr);
        f.param_out[t][i] = pv[j] - step * (mm / (sqrtf(vv) / b2s + f.eps));
        f.exp_avg[t][i] = mm;
        f.exp_avg_sq[t][i] = vv;
      }
    }
  }
};

template <bool kHot, typename Sums, typename Out>
__device__ __forceinline__ void project_bwd_one(const gs_project_bwd_args &a, int g, Sums sums, Out &out) {
  float scl_pre[3] = {0.f, 0.f, 0.f}, rot_pre[4] = {0.f, 0.f, 0.f, 0.f}, op_pre = 0.f;
  if constexpr (kHot) {
#pragma unroll
    for (int k = 0; k < 3; ++k) scl_pre[k] = a.g.scaling[(int64_t)g * 3 + k];
#pragma unroll
    for (int k = 0; k < 4; ++k) rot_pre[k] = a.g.rotation[(int64_t)g * 4 + k];
    op_pre = a.g.opacity[(int64_t)g * a.g.opacity_stride];
  }
  const float4 Qf = reinterpret_cast<const float4 *>(a.conics)[g];
  float acc[GS_PAIR_GRAD_FLOATS];
  sums(acc);
  float dm0 = acc[0], dm1 = acc[1];
  float G[4] = {acc[2], acc[3], acc[3], acc[4]};
  if (!kHot && a.g_means2d) {
    dm0 += a.g_means2d[2 * (size_t)g];
    dm1 += a.g_means2d[2 * (size_t)g + 1];
  }
  if (!kHot && a.g_conics) {
#pragma unroll
    for (int k = 0; k < 4; ++k) G[k] += a.g_conics[4 * (size_t)g + k];
  }
  // colour: sigmoid chain (renderer.py:90), and the SH terms when enabled
  const float *X3 = a.g.xyz + (int64_t)g * a.g.xyz_stride;
  float cl[3], dir[3], inv_norm;
  // (the position kept in registers: read again after the stores below, it
  // would be re-loaded -- the outputs may alias it as far as the compiler knows)
  const float xw = X3[0], yw = X3[1], zw = X3[2];
  color_logits(a.g, a.cam, g, xw, yw, zw, cl, dir, inv_norm);
  float dlg[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float c = 1.f / (1.f + expf(-cl[k]));
    dlg[k] = acc[6 + k] * c * (1.f - c);
    out(kOutColor, g, k, dlg[k], cl[k]);
  }
  // SH: d rest_k = Y_k dlogit; the view direction's gradient reaches xyz
  // through dir = v / |v| (added to d_xyz below)
  float dxyz_sh[3] = {0.f, 0.f, 0.f};
  if (!kHot && a.g.sh_degree > 0) {
    const int nb = sh_rest_count(a.g.sh_degree);
    const float *r = a.g.sh_rest + (int64_t)g * a.g.sh_rest_stride;
    float Y[15], wY[15];
    sh_basis(dir[0], dir[1], dir[2], Y);
    float *dr = a.d_sh_rest + (size_t)g * 3 * 15;
    for (int k = 0; k < 15; ++k) {
      const bool on = k < nb;
      dr[3 * k] = on ? Y[k] * dlg[0] : 0.f;
      dr[3 * k + 1] = on ? Y[k] * dlg[1] : 0.f;
      dr[3 * k + 2] = on ? Y[k] * dlg[2] : 0.f;
      wY[k] = on ? (r[3 * k] * dlg[0] + r[3 * k + 1] * dlg[1]) + r[3 * k + 2] * dlg[2] : 0.f;
    }
    float dd[3];
    sh_basis_vjp(dir[0], dir[1], dir[2], wY, nb, dd);
    const float dot = (dir[0] * dd[0] + dir[1] * dd[1]) + dir[2] * dd[2];
#pragma unroll
    for (int j = 0; j < 3; ++j) dxyz_sh[j] = (dd[j] - dir[j] * dot) * inv_norm;
  }
  float dop = acc[5];
  if (a.g.opacity_is_logit) {  // through get_opacity's sigmoid, as torch's sigmoid_backward
    const float o = 1.f / (1.f + expf(-(kHot ? op_pre : a.g.opacity[(int64_t)g * a.g.opacity_stride])));
    dop = (dop * (1.f - o)) * o;
  }
  out(kOutOpacity, g, 0, dop, op_pre);
  const bool any = dm0 != 0.f || dm1 != 0.f || G[0] != 0.f || G[1] != 0.f || G[2] != 0.f ||
                   G[3] != 0.f || acc[9] != 0.f;
  const bool raw = kHot || a.g.cov3d == nullptr;
  if (!any) {
    const float xv[3] = {xw, yw, zw};
#pragma unroll
    for (int k = 0; k < 3; ++k) out(kOutXyz, g, k, dxyz_sh[k], xv[k]);
    if (raw) {
#pragma unroll
      for (int k = 0; k < 3; ++k) out(kOutScaling, g, k, 0.f, scl_pre[k]);
#pragma unroll
      for (int k = 0; k < 4; ++k) out(kOutRotation, g, k, 0.f, rot_pre[k]);
    } else {
#pragma unroll
      for (int k = 0; k < 9; ++k) out(kOutCov, g, k, 0.f, 0.f);
    }
    return;
  }
  // The screen-space part (conic inverse backward, dL/dJ, dL/dmean) runs in
  // double: for needle Gaussians Q = inv(cov2d) has condition numbers ~1e6
  // and dV = -Q G Q cancels against J C in dL/dJ.  The 3D part (J^T dV J,
  // Rv^T dC Rv, scale/rotation) is plain fp32 with the triple products
  // factored -- f64 exp/div/sqrt and 81-term sums made this kernel 3x slower.
  const gs_camera &c = a.cam;
  const float *R = c.view;  // rows [R | t]
  auto dot3 = [](float a0, float a1, float a2, float b0, float b1, float b2) {
    return __builtin_fmaf(a0, b0, __builtin_fmaf(a1, b1, a2 * b2));
  };
  float Sf[9];
  if (!raw) {
#pragma unroll
    for (int k = 0; k < 9; ++k) Sf[k] = a.g.cov3d[9 * (size_t)g + k];
  } else {
    cov_from_raw(kHot ? scl_pre : a.g.scaling + (int64_t)g * 3, kHot ? rot_pre : a.g.rotation + (int64_t)g * 4, Sf);
  }
  double Xc[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    Xc[i] = (double)xw * R[i * 4] + (double)yw * R[i * 4 + 1] + (double)zw * R[i * 4 + 2] + R[i * 4 + 3];
  const double X = Xc[0], Y = Xc[1], Z = Xc[2];
  const double fx = c.fx, fy = c.fy;
  double RS[9], C[9];  // C = Rv Sigma Rv^T
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      RS[i * 3 + j] = (double)R[i * 4] * Sf[j] + (double)R[i * 4 + 1] * Sf[3 + j] + (double)R[i * 4 + 2] * Sf[6 + j];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      C[i * 3 + j] = RS[i * 3] * R[j * 4] + RS[i * 3 + 1] * R[j * 4 + 1] + RS[i * 3 + 2] * R[j * 4 + 2];
  const double iz = 1.0 / Z, iz2 = iz * iz, iz3 = iz2 * iz;
  const double Jd[6] = {fx * iz, 0.0, -fx * X * iz2, 0.0, -fy * iz, fy * Y * iz2};
  const double Q[4] = {Qf.x, Qf.y, Qf.z, Qf.w};
  // d cov2d = -Q^T G Q^T (inverse backward)
  const double QG0 = Q[0] * G[0] + Q[2] * G[2], QG1 = Q[0] * G[1] + Q[2] * G[3];
  const double QG2 = Q[1] * G[0] + Q[3] * G[2], QG3 = Q[1] * G[1] + Q[3] * G[3];
  const double dVd[4] = {-(QG0 * Q[0] + QG1 * Q[1]), -(QG0 * Q[2] + QG1 * Q[3]), -(QG2 * Q[0] + QG3 * Q[1]),
                         -(QG2 * Q[2] + QG3 * Q[3])};
  double JCt[6], JCn[6];  // J C^T, J C
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      JCt[i * 3 + j] = Jd[i * 3] * C[j * 3] + Jd[i * 3 + 1] * C[j * 3 + 1] + Jd[i * 3 + 2] * C[j * 3 + 2];
      JCn[i * 3 + j] = Jd[i * 3] * C[j] + Jd[i * 3 + 1] * C[3 + j] + Jd[i * 3 + 2] * C[6 + j];
    }
  double dJ[6];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      dJ[i * 3 + j] = dVd[i * 2] * JCt[j] + dVd[i * 2 + 1] * JCt[3 + j] + dVd[i] * JCn[j] + dVd[2 + i] * JCn[3 + j];
  const double dX = dm0 * fx * iz + dJ[2] * (-fx * iz2);
  const double dY = dm1 * (-fy * iz) + dJ[5] * (fy * iz2);
  const double dZ = dm0 * (-fx * X * iz2) + dm1 * (fy * Y * iz2) + dJ[0] * (-fx * iz2) +
                    dJ[2] * (2.0 * fx * X * iz3) + dJ[4] * (fy * iz2) + dJ[5] * (-2.0 * fy * Y * iz3) +
                    (double)acc[9];
  {
    const float xv[3] = {xw, yw, zw};
#pragma unroll
    for (int j = 0; j < 3; ++j)
      out(kOutXyz, g, j, (float)(R[j] * dX + R[4 + j] * dY + R[8 + j] * dZ + (double)dxyz_sh[j]), xv[j]);
  }
  float J[6], dV[4];
#pragma unroll
  for (int k = 0; k < 6; ++k) J[k] = (float)Jd[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) dV[k] = (float)dVd[k];
  float dVJ[6], dC[9];  // dC = J^T dV J
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int j = 0; j < 3; ++j) dVJ[k * 3 + j] = __builtin_fmaf(dV[k * 2], J[j], dV[k * 2 + 1] * J[3 + j]);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) dC[i * 3 + j] = __builtin_fmaf(J[i], dVJ[j], J[3 + i] * dVJ[3 + j]);
  float dCR[9], dS[9];  // dS = Rv^T dC Rv
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int j = 0; j < 3; ++j) dCR[k * 3 + j] = dot3(dC[k * 3], dC[k * 3 + 1], dC[k * 3 + 2], R[j], R[4 + j], R[8 + j]);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) dS[i * 3 + j] = dot3(R[i], R[4 + i], R[8 + i], dCR[j], dCR[3 + j], dCR[6 + j]);
  if (!raw) {
#pragma unroll
    for (int k = 0; k < 9; ++k) out(kOutCov, g, k, dS[k], 0.f);
    return;
  }
  // raw path: Sigma = M M^T, M = R(q) diag(s), s = exp(scaling), q = normalize(rotation)
  const float *sc = kHot ? scl_pre : a.g.scaling + (int64_t)g * 3, *rq = kHot ? rot_pre : a.g.rotation + (int64_t)g * 4;
  float qn = sqrtf(dot3(rq[0], rq[1], rq[2], rq[0], rq[1], rq[2]) + rq[3] * rq[3]);
  qn = qn < 1e-12f ? 1e-12f : qn;
  const float iq = 1.f / qn;
  const float w = rq[0] * iq, x = rq[1] * iq, y = rq[2] * iq, z = rq[3] * iq;
  const float Rq[9] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y - w * z), 2.f * (x * z + w * y),
                       2.f * (x * y + w * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - w * x),
                       2.f * (x * z - w * y), 2.f * (y * z + w * x), 1.f - 2.f * (x * x + y * y)};
  const float s3[3] = {expf(sc[0]), expf(sc[1]), expf(sc[2])};
  float Ss[9];  // dS + dS^T
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k) Ss[i * 3 + k] = dS[i * 3 + k] + dS[k * 3 + i];
  float dR[9];  // dL/dRq = (dS + dS^T) Rq diag(s)^2
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      dR[i * 3 + j] = dot3(Ss[i * 3], Ss[i * 3 + 1], Ss[i * 3 + 2], Rq[j], Rq[3 + j], Rq[6 + j]) * (s3[j] * s3[j]);
#pragma unroll
  for (int j = 0; j < 3; ++j)  // dL/ds_j s_j: (dR / s_j) . Rq column j, times s_j
    out(kOutScaling, g, j, dot3(dR[j], dR[3 + j], dR[6 + j], Rq[j], Rq[3 + j], Rq[6 + j]), sc[j]);
  const float dw = 2.f * ((-z * dR[1] + y * dR[2]) + (z * dR[3] - x * dR[5]) + (-y * dR[6] + x * dR[7]));
  const float dx = 2.f * ((y * dR[1] + z * dR[2]) + (y * dR[3] - 2.f * x * dR[4]) + (-w * dR[5] + z * dR[6]) +
                          (w * dR[7] - 2.f * x * dR[8]));
  const float dy = 2.f * ((-2.f * y * dR[0] + x * dR[1]) + (w * dR[2] + x * dR[3]) + (z * dR[5] - w * dR[6]) +
                          (z * dR[7] - 2.f * y * dR[8]));
  const float dz = 2.f * ((-2.f * z * dR[0] - w * dR[1]) + (x * dR[2] + w * dR[3]) + (-2.f * z * dR[4] + y * dR[5]) +
                          (x * dR[6] + y * dR[7]));
  const float dot = __builtin_fmaf(dw, w, __builtin_fmaf(dx, x, __builtin_fmaf(dy, y, dz * z)));
  out(kOutRotation, g, 0, (dw - w * dot) * iq, rq[0]);
  out(kOutRotation, g, 1, (dx - x * dot) * iq, rq[1]);
  out(kOutRotation, g, 2, (dy - y * dot) * iq, rq[2]);
  out(kOutRotation, g, 3, (dz - z * dot) * iq, rq[3]);
}

// kHot: partials present, no viewspace/conic cotangents, raw scale/rotation,
// DC colour -- the training configuration.  Its loads are all issued up
// front (a load under a runtime branch is waited for at the branch's join,
// which serialised six round trips per thread in the generic instantiation).
// kAdam (gs_project_backward_adam, kHot only): the parameters' Adam update
// fused in, no gradient arrays written.
template <bool kHot, bool kAdam = false>
__global__ __launch_bounds__(kBlock) void k_project_bwd(gs_project_bwd_args a, FusedAdamArgs fa = {}) {
  const int k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= a.g.n) return;
  if (kAdam && fa.skip_flag && *fa.skip_flag) return;  // (the replayed step's frame failed)
  // in depth order, consecutive threads own adjacent slot ranges
  const int g = (!kHot && a.order) ? (int)a.order[k] : k;
  auto sums = [&](float acc[GS_PAIR_GRAD_FLOATS]) {
#pragma unroll
    for (int k = 0; k < GS_PAIR_GRAD_FLOATS; ++k) acc[k] = 0.f;
    if (kHot || a.grad_sums) {  // g's partials summed (k_gather_slots)
      const float2 *gs = reinterpret_cast<const float2 *>(a.grad_sums) + (size_t)g * kF2;
#pragma unroll
      for (int k = 0; k < kF2; ++k) {
        const float2 v = gs[k];
        acc[2 * k] = v.x;
        acc[2 * k + 1] = v.y;
      }
    }
  };
  if constexpr (kAdam) {
    AdamOut out;
    project_bwd_one<kHot>(a, g, sums, out);
    out.flush(fa, g);
  } else {
    GradsOut out{a};
    project_bwd_one<kHot>(a, g, sums, out);
  }
}

// tile coordinates are packed in 12 bits (record word 11): images up to 65536 px a side

// ======================================================== Adam ============
// One launch for all tensors: block b -> (tensor, chunk of kAdamChunk floats)
// through a prefix table in the kernel arguments; float4 streaming.
constexpr int kAdamChunk = kBlock * 4 * 4;  // 4096 floats per block

__global__ __launch_bounds__(kBlock) void k_adam(gs_adam_args a, int4 firsts0, int4 firsts1) {
  const int starts[GS_ADAM_MAX_TENSORS + 1] = {firsts0.x, firsts0.y, firsts0.z, firsts0.w,
                                               firsts1.x, firsts1.y, firsts1.z, firsts1.w, 0x7fffffff};
  int ti = 0;
#pragma unroll
  for (int k = 1; k < GS_ADAM_MAX_TENSORS; ++k) ti += (int)blockIdx.x >= starts[k] ? 1 : 0;
  const gs_adam_tensor &t = a.t[ti];
  if (!t.grad) return;
  // a replayed step whose frame failed on the device updates nothing (the
  // caller redoes it); a replayed step's per-step scalars come from its row
  if (a.skip_flag && *a.skip_flag) return;
  float lr = t.lr, bc1 = t.bias_correction1, bc2s = t.bias_correction2_sqrt;
  if (a.hyper) {
    const float *h = a.hyper + ((size_t)*a.hyper_row * GS_ADAM_MAX_TENSORS + ti) * 3;
    lr = h[0];
    bc1 = h[1];
    bc2s = h[2];
  }
  float *const pout = t.param_out ? t.param_out : t.param;  // (in place unless an output is given)
  const int64_t base = (int64_t)(blockIdx.x - starts[ti]) * kAdamChunk;
  const float b1 = a.beta1, b2 = a.beta2, om1 = 1.f - b1, om2 = 1.f - b2;
  const float step = lr / bc1;
  const bool vec = ((reinterpret_cast<uintptr_t>(t.param) | reinterpret_cast<uintptr_t>(t.grad) |
                     reinterpret_cast<uintptr_t>(t.exp_avg) | reinterpret_cast<uintptr_t>(t.exp_avg_sq) |
                     reinterpret_cast<uintptr_t>(pout)) & 15) == 0;
  if (vec && base + kAdamChunk <= t.numel) {
    // whole chunk in range (all but a tensor's last block): the four rounds'
    // loads issued together, no branch between them -- under the per-round
    // branches below the compiler waited for each round's loads in turn
    float4 p[4], g[4], m[4], v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t i0 = base + ((int64_t)r * kBlock + threadIdx.x) * 4;
      p[r] = *reinterpret_cast<const float4 *>(t.param + i0);
      g[r] = *reinterpret_cast<const float4 *>(t.grad + i0);
      m[r] = *reinterpret_cast<const float4 *>(t.exp_avg + i0);
      v[r] = *reinterpret_cast<const float4 *>(t.exp_avg_sq + i0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t i0 = base + ((int64_t)r * kBlock + threadIdx.x) * 4;
#define GS_ADAM_1(c)                                                          \
      m[r].c = m[r].c + om1 * (g[r].c - m[r].c);                              \
      v[r].c = b2 * v[r].c + om2 * (g[r].c * g[r].c);                         \
      p[r].c -= step * (m[r].c / (sqrtf(v[r].c) / bc2s + a.eps));
      GS_ADAM_1(x) GS_ADAM_1(y) GS_ADAM_1(z) GS_ADAM_1(w)
#undef GS_ADAM_1
      *reinterpret_cast<float4 *>(pout + i0) = p[r];
      *reinterpret_cast<float4 *>(t.exp_avg + i0) = m[r];
      *reinterpret_cast<float4 *>(t.exp_avg_sq + i0) = v[r];
    }
    return;
  }
  for (int r = 0; r < 4; ++r) {
    const int64_t i0 = base + ((int64_t)r * kBlock + threadIdx.x) * 4;
    if (i0 >= t.numel) break;
    if (vec && i0 + 4 <= t.numel) {
      float4 p = *reinterpret_cast<const float4 *>(t.param + i0);
      const float4 g = *reinterpret_cast<const float4 *>(t.grad + i0);
      float4 m = *reinterpret_cast<const float4 *>(t.exp_avg + i0);
      float4 v = *reinterpret_cast<const float4 *>(t.exp_avg_sq + i0);
#define GS_ADAM_1(c)                                              \
      m.c = m.c + om1 * (g.c - m.c);                              \
      v.c = b2 * v.c + om2 * (g.c * g.c);                         \
      p.c -= step * (m.c / (sqrtf(v.c) / bc2s + a.eps));
      GS_ADAM_1(x) GS_ADAM_1(y) GS_ADAM_1(z) GS_ADAM_1(w)
#undef GS_ADAM_1
      *reinterpret_cast<float4 *>(pout + i0) = p;
      *reinterpret_cast<float4 *>(t.exp_avg + i0) = m;
      *reinterpret_cast<float4 *>(t.exp_avg_sq + i0) = v;
    } else {
      for (int64_t i = i0; i < i0 + 4 && i < t.numel; ++i) {
        const float g = t.grad[i];
        const float m = t.exp_avg[i] + om1 * (g - t.exp_avg[i]);
        const float v = b2 * t.exp_avg_sq[i] + om2 * (g * g);
        t.exp_avg[i] = m;
        t.exp_avg_sq[i] = v;
        pout[i] = t.param[i] - step * (m / (sqrtf(v) / bc2s + a.eps));
      }
    }
  }
}

int cells_per_tile(int tile_size) {
  const int qx = (tile_size + GS_QUAD - 1) / GS_QUAD;
  return qx * qx;
}


// tile_size in range, image non-empty, tile coordinates fit 12 bits
bool cam_ok(const gs_camera &c) {
  if (c.tile_size < 1 || c.tile_size > GS_MAX_TILE || c.image_width <= 0 || c.image_height <= 0) return false;
  return div_up(c.image_width, c.tile_size) <= GS_MAX_TILES_AXIS && div_up(c.image_height, c.tile_size) <= GS_MAX_TILES_AXIS;
}
const char *kCamMsg = "%s: tile_size must be in [1, 16384], the image non-empty with at most 4096 tiles per axis";

// A Gaussian's rectangle is at most 2 floor(r) + 1 <= 2 floor(radius_max) + 1
// pixels wide (renderer.py:278-293), clipped to the image: its tile width
// minus one must fit the record's 8-bit field (GS_MAX_RECT_TILES).
bool rect_ok(const gs_camera &c) {
  if (!(c.radius_max >= 0.f) || !(c.radius_max < 1e9f) || !(c.radius_min <= c.radius_max)) return false;
  const long long tiles_x = div_up(c.image_width, c.tile_size);
  const long long span = (2LL * (long long)c.radius_max + 1 + c.tile_size - 1) / c.tile_size + 1;
  return (span < tiles_x ? span : tiles_x) <= GS_MAX_RECT_TILES;
}

bool tiles_match(const gs_camera &c, int tiles_x, int tiles_y) {
  return tiles_x == (int)div_up(c.image_width, c.tile_size) && tiles_y == (int)div_up(c.image_height, c.tile_size);
}

}  // namespace

gs_status gs_internal_fail(gs_status s, const char *fmt, const char *what) { return fail(s, fmt, what); }
gs_status gs_internal_check_launch(const char *what) { return check_launch(what); }

// ============================================================ C ABI =======
extern "C" {

int32_t gs_abi_version(void) { return GS_ABI_VERSION; }

const char *gs_last_error(void) { return g_err; }

gs_status gs_project_forward(const gs_project_args *a, gs_stream_t stream) {
  if (!a) return fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_project_forward");
  if (!cam_ok(a->cam)) return fail(GS_ERR_UNSUPPORTED, kCamMsg, "gs_project_forward");
  if (!rect_ok(a->cam))
    return fail(GS_ERR_UNSUPPORTED, "%s: radius_min <= radius_max, finite, with rectangles of at most 256 tiles in x "
                "(GS_MAX_RECT_TILES)", "gs_project_forward");
  if (a->key_bits < 1 || a->key_bits > 32) return fail(GS_ERR_INVALID_ARG, "%s: key_bits must be 1..32", "gs_project_forward");
  if (a->g.n < 0) return fail(GS_ERR_INVALID_ARG, "%s: bad n", "gs_project_forward");
  hipStream_t s = (hipStream_t)stream;
  if (a->g.n == 0) return GS_OK;
  if (!a->g.xyz || !a->g.color_logits || !a->g.opacity || !a->means2d || !a->conics || !a->radii ||
      !a->vis || !a->records || !a->rects || !a->depth_keys || !a->key_minmax)
    return fail(GS_ERR_INVALID_ARG, "%s: null pointer", "gs_project_forward");
  if (!a->g.cov3d && (!a->g.scaling || !a->g.rotation))
    return fail(GS_ERR_INVALID_ARG, "%s: need cov3d or scaling+rotation", "gs_project_forward");
  if (a->g.sh_degree < 0 || a->g.sh_degree > 3 || (a->g.sh_degree > 0 && !a->g.sh_rest))
    return fail(GS_ERR_INVALID_ARG, "%s: sh_degree must be 0..3, with sh_rest when > 0", "gs_project_forward");
  if (!a->g.cov3d && a->g.sh_degree == 0)
    k_project_fwd<true><<<div_up(a->g.n, kBlock), kBlock, 0, s>>>(*a);
  else
    k_project_fwd<false><<<div_up(a->g.n, kBlock), kBlock, 0, s>>>(*a);
  return check_launch("gs_project_forward");
}

size_t gs_radix_sort_workspace_bytes(int32_t n) {
  const size_t nb = n > 0 ? div_up(n, kSortChunk) : 1;
  return sizeof(uint32_t) * (kRadix * nb + kRadix) + 256;
}

gs_status gs_radix_sort_pairs(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt,
                              int32_t n, int32_t begin_bit, int32_t end_bit, int32_t vals_are_iota,
                              void *workspace, size_t workspace_bytes, int32_t *result_in_alt,
                              gs_stream_t stream) {
  return gs_internal_radix_sort_pairs(keys, vals, keys_alt, vals_alt, n, begin_bit, end_bit, vals_are_iota,
                                      workspace, workspace_bytes, result_in_alt, 0, nullptr, stream);
}

}  // extern "C"

gs_status gs_internal_radix_sort_pairs(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt,
                                       int32_t n, int32_t begin_bit, int32_t end_bit, int32_t vals_are_iota,
                                       void *workspace, size_t workspace_bytes, int32_t *result_in_alt,
                                       int32_t first_counts_ready, const uint32_t *n_dev, gs_stream_t stream) {
  if (!result_in_alt) return fail(GS_ERR_INVALID_ARG, "%s: null result_in_alt", "gs_radix_sort_pairs");
  if (begin_bit < 0 || end_bit > 32 || begin_bit >= end_bit || n < 0)
    return fail(GS_ERR_INVALID_ARG, "%s: bad bit range / n", "gs_radix_sort_pairs");
  const int passes = (end_bit - begin_bit + kRadixBits - 1) / kRadixBits;
  *result_in_alt = passes & 1;
  if (n == 0) return GS_OK;
  if (!keys || !vals || !keys_alt || !vals_alt || !workspace ||
      workspace_bytes < gs_radix_sort_workspace_bytes(n))
    return fail(GS_ERR_INVALID_ARG, "%s: null buffer or workspace too small", "gs_radix_sort_pairs");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)div_up(n, kSortChunk);
  uint32_t *counts = (uint32_t *)workspace;
  uint32_t *totals = counts + (size_t)kRadix * nb;
  uint32_t *kin = keys, *vin = vals, *kout = keys_alt, *vout = vals_alt;
  // the bits spread evenly over the passes, the narrower digit first (13-bit
  // tile ids: 6 + 7, not 8 + 5): the first pass's scatter writes are the least
  // coalesced (its input is in emission order), so it gets the fewer, longer
  // digit runs per block (7 + 6 measured 0.9 us slower per scatter,
  // profiles/r05/sort_ab/)
  int shift = begin_bit;
  for (int p = 0; p < passes; ++p) {
    const int nbits = (end_bit - shift) / (passes - p);
    if (p > 0 || !first_counts_ready) k_radix_hist<<<nb, kBlock, 0, s>>>(kin, n, shift, nbits, counts, nb, n_dev);
    k_radix_scan<<<1 << nbits, kBlock, 0, s>>>(counts, totals, nb, n_dev);
    if (p == 0 && vals_are_iota)
      k_radix_scatter<true><<<nb, kBlock, 0, s>>>(kin, nullptr, kout, vout, n, shift, nbits, counts, totals, nb,
                                                   n_dev);
    else
      k_radix_scatter<false><<<nb, kBlock, 0, s>>>(kin, vin, kout, vout, n, shift, nbits, counts, totals, nb,
                                                    n_dev);
    gs_status st = check_launch("gs_radix_sort_pairs");
    if (st) return st;
    shift += nbits;
    uint32_t *tk = kin, *tv = vin;
    kin = kout;
    vin = vout;
    kout = tk;
    vout = tv;
  }
  return GS_OK;
}

int32_t gs_internal_small_sort_max(void) { return kMsdCap; }

gs_status gs_internal_small_sort(const uint32_t *keys, const uint32_t *vals, uint32_t *keys_out, uint32_t *vals_out,
                                 int32_t n, int32_t bits, const uint32_t *n_dev, gs_stream_t stream) {
  if (n < 0 || n > kMsdCap || bits < 1 || bits > 32 || (n > 0 && (!keys || !keys_out || !vals_out)))
    return fail(GS_ERR_INVALID_ARG, "%s: bad args", "gs_internal_small_sort");
  if (n == 0) return GS_OK;
  k_msd_bucket_sort<true><<<1, kMsdThreads, 0, (hipStream_t)stream>>>(
      const_cast<uint32_t *>(keys), const_cast<uint32_t *>(vals), nullptr, bits, nullptr, (uint32_t)n, keys_out,
      vals_out, n_dev);
  return check_launch("gs_internal_small_sort");
}

int32_t gs_internal_first_pass_bits(int32_t begin_bit, int32_t end_bit) {
  const int passes = (end_bit - begin_bit + kRadixBits - 1) / kRadixBits;
  return passes > 0 ? (end_bit - begin_bit) / passes : 0;  // (the narrower digit first, as the sort)
}

gs_status gs_internal_bin_count_hist(const gs_bin_args *a, uint32_t *tile_counts, int32_t bits, gs_stream_t stream) {
  if (!a || !a->counters || a->n <= 0 || !a->workspace || a->workspace_bytes < gs_bin_workspace_bytes(a->n))
    return fail(GS_ERR_INVALID_ARG, "%s: bad args", "gs_internal_bin_count_hist");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)div_up(a->n, kBinChunk);
  uint32_t *partials = (uint32_t *)a->workspace;
  const uint32_t zero = tile_counts ? (uint32_t)((1u << bits) * div_up(a->capacity > 0 ? a->capacity : 0, kSortChunk))
                                    : 0u;
  k_bin_partials<<<nb, kBlock, 0, s>>>(*a, partials, nb, TileHist{tile_counts, zero, 0});
  k_bin_scan_partials<<<1, kBlock, 0, s>>>(*a, partials, nb);
  return check_launch("gs_bin_count");
}

gs_status gs_internal_bin_emit_hist(const gs_bin_args *a, uint32_t *tile_counts, int32_t bits, gs_stream_t stream) {
  if (!a || a->n <= 0 || !tile_counts || bits < 1 || bits > kRadixBits)
    return fail(GS_ERR_INVALID_ARG, "%s: bad args", "gs_internal_bin_emit_hist");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)div_up(a->n, kBinChunk);
  k_bin_emit<true><<<nb, kBlock, 0, s>>>(*a, (const uint32_t *)a->workspace, TileHist{tile_counts, 0u, bits});
  return check_launch("gs_bin_emit");
}

extern "C" {

gs_status gs_depth_sort_msd(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt, int32_t n,
                            int32_t key_bits, void *workspace, size_t workspace_bytes, uint32_t *overflow_word,
                            int32_t *result_in_alt, gs_stream_t stream) {
  if (!result_in_alt) return fail(GS_ERR_INVALID_ARG, "%s: null result_in_alt", "gs_depth_sort_msd");
  if (key_bits < 9 || key_bits > 32 || n < 0)
    return fail(GS_ERR_UNSUPPORTED, "%s: key_bits must be 9..32", "gs_depth_sort_msd");
  *result_in_alt = 1;
  if (n == 0) return GS_OK;
  if (!keys || !vals || !keys_alt || !vals_alt || !workspace || !overflow_word ||
      workspace_bytes < gs_radix_sort_workspace_bytes(n))
    return fail(GS_ERR_INVALID_ARG, "%s: null buffer or workspace too small", "gs_depth_sort_msd");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)div_up(n, kSortChunk);
  uint32_t *counts = (uint32_t *)workspace;
  uint32_t *totals = counts + (size_t)kRadix * nb;
  const int shift = key_bits - kRadixBits;
  k_radix_hist<<<nb, kBlock, 0, s>>>(keys, n, shift, kRadixBits, counts, nb);
  k_radix_scan<<<kRadix, kBlock, 0, s>>>(counts, totals, nb);
  k_radix_scatter<true><<<nb, kBlock, 0, s>>>(keys, nullptr, keys_alt, vals_alt, n, shift, kRadixBits, counts,
                                               totals, nb);
  k_msd_bucket_sort<false><<<kRadix - 1, kMsdThreads, 0, s>>>(keys_alt, vals_alt, totals, shift, overflow_word);
  return check_launch("gs_depth_sort_msd");
}

size_t gs_bin_workspace_bytes(int32_t n) {
  const size_t nb = n > 0 ? div_up(n, kBinChunk) : 1;
  return sizeof(uint32_t) * ((5 * nb + 3) & ~(size_t)3) + sizeof(uint32_t) * 2 * (size_t)(n > 0 ? n : 0) + 256;
}

gs_status gs_bin_count(const gs_bin_args *a, gs_stream_t stream) {
  if (!a || !a->counters) return fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_bin_count");
  if (a->n <= 0) return GS_OK;
  if (!a->sorted_ids || !a->rects || !a->vis || !a->pair_offset || !a->workspace || !a->key_minmax ||
      a->workspace_bytes < gs_bin_workspace_bytes(a->n))
    return fail(GS_ERR_INVALID_ARG, "%s: null buffer or workspace too small", "gs_bin_count");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)div_up(a->n, kBinChunk);
  uint32_t *partials = (uint32_t *)a->workspace;
  k_bin_partials<<<nb, kBlock, 0, s>>>(*a, partials, nb, TileHist{nullptr, 0u, 0});
  k_bin_scan_partials<<<1, kBlock, 0, s>>>(*a, partials, nb);
  return check_launch("gs_bin_count");
}

gs_status gs_bin_emit(const gs_bin_args *a, gs_stream_t stream) {
  if (!a) return fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_bin_emit");
  if (a->n <= 0) return GS_OK;
  if (!a->sorted_ids || !a->rects || !a->counters || !a->workspace || !a->tile_keys || !a->pair_gauss ||
      !a->pair_offset || !a->records)
    return fail(GS_ERR_INVALID_ARG, "%s: null buffer", "gs_bin_emit");
  if (a->workspace_bytes < gs_bin_workspace_bytes(a->n))
    return fail(GS_ERR_INVALID_ARG, "%s: workspace too small", "gs_bin_emit");
  if (a->capacity < 0) return fail(GS_ERR_INVALID_ARG, "%s: negative capacity", "gs_bin_emit");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)div_up(a->n, kBinChunk);
  k_bin_emit<false><<<nb, kBlock, 0, s>>>(*a, (const uint32_t *)a->workspace, TileHist{nullptr, 0u, 0});
  return check_launch("gs_bin_emit");
}

gs_status gs_tile_ranges(const gs_range_args *a, gs_stream_t stream) {
  if (!a || !a->ranges) return fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_tile_ranges");
  hipStream_t s = (hipStream_t)stream;
  if (a->num_pairs < 0 || a->num_tiles < 0) return fail(GS_ERR_INVALID_ARG, "%s: negative size", "gs_tile_ranges");
  if (a->num_tiles == 0) return GS_OK;
  if (a->num_pairs > 0 && !a->sorted_keys) return fail(GS_ERR_INVALID_ARG, "%s: null buffer", "gs_tile_ranges");
  if (a->slot_live && (a->cells < 1 || (a->cells == 4 && (reinterpret_cast<uintptr_t>(a->slot_live) & 3u))))
    return fail(GS_ERR_INVALID_ARG, "%s: slot_live needs cells >= 1 (4-B aligned at 4 cells)", "gs_tile_ranges");
  // four positions per thread where the flags are 4-B words (the default
  // tile) and the keys 16-B aligned
  if (GS_RANGES_X4 && (!a->slot_live || a->cells == 4) && (reinterpret_cast<uintptr_t>(a->sorted_keys) & 15u) == 0 &&
      (reinterpret_cast<uintptr_t>(a->slot_live) & 15u) == 0)
    k_tile_ranges4<<<div_up(a->num_pairs / 4 + 1, kBlock), kBlock, 0, s>>>(*a);
  else
    k_tile_ranges<<<div_up(a->num_pairs + 1, kBlock), kBlock, 0, s>>>(*a);
  return check_launch("gs_tile_ranges");
}

int32_t gs_tile_quads(int32_t tile_size) {
  return (tile_size < 1 || tile_size > GS_MAX_TILE) ? 0 : cells_per_tile(tile_size);
}

int32_t gs_partial_groups(int32_t tile_size) {
  // one partial per 8x8 cell (a wave combining a tile's cells wrote fewer and
  // replayed slower: tools/variants/README.md)
  return (tile_size < 1 || tile_size > GS_MAX_TILE) ? 0 : cells_per_tile(tile_size);
}

size_t gs_blend_live_words(int32_t num_pairs, int32_t num_tiles) {
  if (num_pairs < 0 || num_tiles < 0) return 0;
  return (size_t)num_pairs / 64u + (size_t)num_tiles + 2u;
}

gs_status gs_blend_forward(const gs_blend_fwd_args *a, gs_stream_t stream) {
  if (!a) return fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_blend_forward");
  if (!cam_ok(a->cam)) return fail(GS_ERR_UNSUPPORTED, kCamMsg, "gs_blend_forward");
  if (!tiles_match(a->cam, a->tiles_x, a->tiles_y))
    return fail(GS_ERR_INVALID_ARG, "%s: tiles_x/tiles_y do not match the image", "gs_blend_forward");
  if (!a->ranges || !a->records || !a->image || !a->alpha || !a->depth || !a->pix_flags || !a->cell_neval ||
      (a->live_bits && a->live_words <= 0) || (a->num_pairs > 0 && !a->sorted_gauss))
    return fail(GS_ERR_INVALID_ARG, "%s: null buffer", "gs_blend_forward");
  if (a->num_pairs < 0) return fail(GS_ERR_INVALID_ARG, "%s: negative num_pairs", "gs_blend_forward");
  hipStream_t s = (hipStream_t)stream;
  const bool t16 = a->cam.tile_size == GS_DEFAULT_TILE;
  const long long cblocks = (long long)div_up((long long)a->tiles_x * a->tiles_y, 8) * 8LL * cells_per_tile(a->cam.tile_size);
  // (a launch's work-items, workgroups x 64, must stay below 2^32)
  if (cblocks * kWave > 0xffffffffLL) return fail(GS_ERR_UNSUPPORTED, "%s: too many tiles", "gs_blend_forward");
  if (a->pair_counts)
    k_blend_fwd<true, false><<<(unsigned)cblocks, kWave, 0, s>>>(*a);
  else if (t16)
    k_blend_fwd<false, true><<<(unsigned)cblocks, kWave, 0, s>>>(*a);
  else
    k_blend_fwd<false, false><<<(unsigned)cblocks, kWave, 0, s>>>(*a);
  return check_launch("gs_blend_forward");
}

gs_status gs_blend_backward(const gs_blend_bwd_args *a, gs_stream_t stream) {
  if (!a) return fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_blend_backward");
  if (!cam_ok(a->cam)) return fail(GS_ERR_UNSUPPORTED, kCamMsg, "gs_blend_backward");
  if (!tiles_match(a->cam, a->tiles_x, a->tiles_y))
    return fail(GS_ERR_INVALID_ARG, "%s: tiles_x/tiles_y do not match the image", "gs_blend_backward");
  if (!a->ranges || !a->sorted_gauss || !a->records || !a->image || !a->alpha || !a->depth || !a->pix_flags ||
      !a->cell_neval || !a->g_image ||
      !a->pair_grads || !a->slot_live || (a->live_bits && a->live_words <= 0))
    return fail(GS_ERR_INVALID_ARG, "%s: null buffer", "gs_blend_backward");
  if (a->num_pairs < 0) return fail(GS_ERR_INVALID_ARG, "%s: negative num_pairs", "gs_blend_backward");
  const int cells = cells_per_tile(a->cam.tile_size);
  gs_blend_bwd_args b = *a;
  if (b.cell_count == 0 && b.cell_begin == 0) b.cell_count = cells;  // (0: every cell, one batch)
  if (b.cell_begin < 0 || b.cell_count < 1 || b.cell_begin + b.cell_count > cells)
    return fail(GS_ERR_INVALID_ARG, "%s: the cell batch [cell_begin, cell_begin + cell_count) must lie in "
                "[0, gs_tile_quads(tile_size))", "gs_blend_backward");
  hipStream_t s = (hipStream_t)stream;
  const int num_tiles = b.tiles_x * b.tiles_y;
  if (num_tiles <= 0) return GS_OK;
  const long long blocks = (long long)div_up(num_tiles, 8) * 8LL * b.cell_count;
  if (blocks * kWave > 0xffffffffLL) return fail(GS_ERR_UNSUPPORTED, "%s: too many tiles", "gs_blend_backward");
  if (b.cam.tile_size == GS_DEFAULT_TILE && b.cell_count == cells)
    k_blend_bwd<true><<<(unsigned)blocks, kWave, 0, s>>>(b);
  else
    k_blend_bwd<false><<<(unsigned)blocks, kWave, 0, s>>>(b);
  return check_launch("gs_blend_backward");
}

int64_t gs_blend_backward_groups(int32_t tiles_x, int32_t tiles_y, int32_t cell_count) {
  if (tiles_x <= 0 || tiles_y <= 0 || cell_count <= 0) return 0;
  return (int64_t)div_up(tiles_x * tiles_y, 8) * 8LL * cell_count;
}

gs_status gs_blend_backward_lane_stats(const gs_blend_bwd_args *a, uint64_t *hist, uint32_t *per_group,
                                       gs_stream_t stream) {
  if (!a || !hist || !per_group) return fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_blend_backward_lane_stats");
  if (a->cam.tile_size != GS_DEFAULT_TILE || !(a->cell_begin == 0 && (a->cell_count == 0 || a->cell_count == 4)))
    return fail(GS_ERR_UNSUPPORTED, "%s: the default tile, one batch", "gs_blend_backward_lane_stats");
  if (!a->ranges || !a->sorted_gauss || !a->records || !a->image || !a->alpha || !a->depth || !a->pix_flags ||
      !a->cell_neval || !a->g_image ||
      !a->pair_grads || !a->slot_live || !tiles_match(a->cam, a->tiles_x, a->tiles_y))
    return fail(GS_ERR_INVALID_ARG, "%s: bad buffers", "gs_blend_backward_lane_stats");
  gs_blend_bwd_args b = *a;
  b.cell_begin = 0;
  b.cell_count = 4;
  const int64_t blocks = gs_blend_backward_groups(b.tiles_x, b.tiles_y, 4);
  if (blocks <= 0) return GS_OK;
  hipStream_t s = (hipStream_t)stream;
  k_blend_bwd<true, true><<<(unsigned)blocks, kWave, 0, s>>>(
      b, BwdStats{reinterpret_cast<unsigned long long *>(hist), per_group});
  return check_launch("gs_blend_backward_lane_stats");
}

namespace {
gs_status launch_gather(const gs_project_bwd_args *a, int accumulate, hipStream_t s) {
  const uint32_t ng = (uint32_t)a->partial_groups;
  const unsigned gb = div_up(8LL * a->g.n, kBlock);
  if (a->order) {  // (a walk in another order: the default tile only, a probe's)
    if (ng != 4)
      return fail(GS_ERR_UNSUPPORTED, "%s: order needs the default tile's 4 partial groups", "gs_gather_partials");
    k_gather_slots<4, 2, 4, kGatherOrder><<<gb, kBlock, 0, s>>>(*a, ng, accumulate);
    return check_launch("gs_gather_partials");
  }
  if (ng == 1)
    k_gather_slots<1, kGatherHL1><<<div_up((long long)kGatherHL1 * a->g.n, kBlock), kBlock, 0, s>>>(*a, ng, accumulate);
  else if (ng == 2)
    k_gather_slots<2, 2><<<div_up(4LL * a->g.n, kBlock), kBlock, 0, s>>>(*a, ng, accumulate);
  else if (ng == 4)  // the default tile's four cells
    k_gather_slots<4, 2, 4><<<div_up(8LL * a->g.n, kBlock), kBlock, 0, s>>>(*a, ng, accumulate);
  else
    k_gather_slots<4, 2><<<div_up(8LL * a->g.n, kBlock), kBlock, 0, s>>>(*a, ng, accumulate);
  return check_launch("gs_gather_partials");
}
}  // namespace

gs_status gs_gather_partials(const gs_project_bwd_args *a, int32_t accumulate, gs_stream_t stream) {
  if (!a) return fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_gather_partials");
  if (a->g.n <= 0) return GS_OK;
  if (!a->pair_grads || !a->slot_live || !a->grad_sums || !a->vis || !a->rects || !a->pair_offset ||
      a->partial_groups < 1)
    return fail(GS_ERR_INVALID_ARG, "%s: null buffer or partial_groups < 1", "gs_gather_partials");
  return launch_gather(a, accumulate, (hipStream_t)stream);
}

gs_status gs_project_backward(const gs_project_bwd_args *a, gs_stream_t stream) {
  if (!a) return fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_project_backward");
  if (a->g.n <= 0) return GS_OK;
  const bool raw = a->g.cov3d == nullptr;
  if (!a->g.xyz || !a->g.color_logits || !a->means2d || !a->conics || !a->vis || !a->rects ||
      !a->pair_offset || !a->d_xyz || !a->d_color_logits || !a->d_opacity ||
      (raw ? (!a->g.scaling || !a->g.rotation || !a->d_scaling || !a->d_rotation) : !a->d_cov3d) ||
      (a->pair_grads && (!a->grad_sums || !a->slot_live || a->partial_groups < 1)))
    return fail(GS_ERR_INVALID_ARG, "%s: null buffer", "gs_project_backward");
  if (a->g.sh_degree < 0 || a->g.sh_degree > 3 || (a->g.sh_degree > 0 && (!a->g.sh_rest || !a->d_sh_rest)))
    return fail(GS_ERR_INVALID_ARG, "%s: sh_degree must be 0..3, with sh_rest and d_sh_rest when > 0",
                "gs_project_backward");
  if (a->pair_grads && !cam_ok(a->cam)) return fail(GS_ERR_UNSUPPORTED, kCamMsg, "gs_project_backward");
  hipStream_t s = (hipStream_t)stream;
  const bool hot = a->grad_sums && !a->g_means2d && !a->g_conics && !a->g.cov3d && a->g.sh_degree == 0 && !a->order;
  if (a->pair_grads) {  // (NULL with grad_sums: the sums are there already, gs_gather_partials)
    gs_status st = launch_gather(a, 0, s);
    if (st) return st;
  }
  if (hot)
    k_project_bwd<true><<<div_up(a->g.n, kBlock), kBlock, 0, s>>>(*a);
  else
    k_project_bwd<false><<<div_up(a->g.n, kBlock), kBlock, 0, s>>>(*a);
  return check_launch("gs_project_backward");
}

gs_status gs_project_backward_adam(const gs_project_bwd_args *a, const gs_adam_args *adam, gs_stream_t stream) {
  static const char *what = "gs_project_backward_adam";
  if (!a || !adam) return fail(GS_ERR_INVALID_ARG, "%s: null args", what);
  if (a->g.n <= 0) return GS_OK;
  // the training configuration only (k_project_bwd<kHot>): raw scale /
  // rotation, DC colour, blend sums, no viewspace / conic cotangents
  if (a->g.cov3d || a->g.sh_degree != 0 || a->g_means2d || a->g_conics || a->order || !a->grad_sums ||
      !a->g.scaling || !a->g.rotation || !a->g.opacity_is_logit)
    return fail(GS_ERR_UNSUPPORTED, "%s: raw scaling / rotation, opacity logit, DC colour, blend sums, no "
                "viewspace / conic cotangents", what);
  if (!a->g.xyz || !a->g.color_logits || !a->means2d || !a->conics || !a->vis || !a->rects || !a->pair_offset ||
      (a->pair_grads && (!a->slot_live || a->partial_groups < 1)) || adam->num_tensors != 5 ||
      (adam->hyper && !adam->hyper_row) || !cam_ok(a->cam))
    return fail(GS_ERR_INVALID_ARG, "%s: null buffer, or adam->num_tensors != 5", what);
  // the tensors in the kOut* order, each the parameter the projection reads
  const float *params[5] = {a->g.xyz, a->g.color_logits, a->g.opacity, a->g.scaling, a->g.rotation};
  const int64_t rows[5] = {3, 3, 1, 3, 4};
  FusedAdamArgs f;
  memset(&f, 0, sizeof(f));
  for (int t = 0; t < 5; ++t) {
    const gs_adam_tensor &x = adam->t[t];
    if (x.param != params[t] || !x.exp_avg || !x.exp_avg_sq || x.numel != rows[t] * a->g.n)
      return fail(GS_ERR_INVALID_ARG, "%s: adam->t[0..4] must be xyz, colour logits, opacity, scaling, rotation "
                  "(the projection's own parameter arrays, dense)", what);
    f.param_out[t] = x.param_out ? x.param_out : x.param;
    f.exp_avg[t] = x.exp_avg;
    f.exp_avg_sq[t] = x.exp_avg_sq;
    f.lr[t] = x.lr;
    f.bc1[t] = x.bias_correction1;
    f.bc2s[t] = x.bias_correction2_sqrt;
    f.hyper_slot[t] = t;
  }
  if (a->g.xyz_stride != 3 || a->g.color_stride != 3 || a->g.opacity_stride != 1)
    return fail(GS_ERR_INVALID_ARG, "%s: dense parameter rows", what);
  f.beta1 = adam->beta1;
  f.beta2 = adam->beta2;
  f.eps = adam->eps;
  f.skip_flag = adam->skip_flag;
  f.hyper = adam->hyper;
  f.hyper_row = adam->hyper_row;
  hipStream_t s = (hipStream_t)stream;
  if (a->pair_grads) {
    gs_status st = launch_gather(a, 0, s);
    if (st) return st;
  }
  k_project_bwd<true, true><<<div_up(a->g.n, kBlock), kBlock, 0, s>>>(*a, f);
  return check_launch(what);
}

gs_status gs_adam_step(const gs_adam_args *a, gs_stream_t stream) {
  if (!a || a->num_tensors < 0 || a->num_tensors > GS_ADAM_MAX_TENSORS || (a->hyper && !a->hyper_row))
    return fail(GS_ERR_INVALID_ARG, "%s: bad args", "gs_adam_step");
  int starts[GS_ADAM_MAX_TENSORS] = {0};
  long long nblk = 0;
  for (int i = 0; i < GS_ADAM_MAX_TENSORS; ++i) {
    starts[i] = (int)nblk;
    if (i < a->num_tensors) {
      const gs_adam_tensor &t = a->t[i];
      if (t.grad && (!t.param || !t.exp_avg || !t.exp_avg_sq || t.numel < 0))
        return fail(GS_ERR_INVALID_ARG, "%s: null buffer", "gs_adam_step");
      nblk += t.grad ? (t.numel + kAdamChunk - 1) / kAdamChunk : 0;
    }
  }
  if (nblk == 0) return GS_OK;
  if (nblk > 0x7fffffffLL) return fail(GS_ERR_UNSUPPORTED, "%s: too many elements", "gs_adam_step");
  // tensors without grad get no blocks: zero-length ranges in the table
  gs_adam_args c = *a;
  for (int i = a->num_tensors; i < GS_ADAM_MAX_TENSORS; ++i) c.t[i].grad = nullptr;
  k_adam<<<(unsigned)nblk, kBlock, 0, (hipStream_t)stream>>>(
      c, make_int4(starts[0], starts[1], starts[2], starts[3]), make_int4(starts[4], starts[5], starts[6], starts[7]));
  return check_launch("gs_adam_step");
}

}  // extern "C"
