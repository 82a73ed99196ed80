// gs_loss.hip -- fused L1 + D-SSIM photometric loss, forward and backward
// (include/gsplat_mi355x.h, "Photometric loss").
//
// Forward, one 256-thread workgroup per 16x16 output tile of one channel:
// the (16+2R)^2 patch of pred and target goes to LDS (zero outside the
// image = the reference's conv2d zero padding), a horizontal pass forms the
// five windowed sums (x, y, x^2, y^2, xy) per patch row, a vertical pass the
// per-pixel statistics.  Each pixel then has its SSIM, |x - y| and the three
// partial derivatives of its clamped SSIM with respect to (mu_x, E[x^2],
// E[xy]); the workgroup writes its two partial sums (fixed-order tree), and
// a one-workgroup kernel reduces them in fixed order, in double.
// Backward: dL/dx_p = blur(m1)(p) + 2 x_p blur(m2)(p) + y_p blur(m3)(p)
// (the window is symmetric, so the adjoint of the zero-padded blur is the
// same blur), scaled by -lambda / (CHW), plus (1 - lambda) sign(x - y) / (CHW).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gs_internal.h"
#include "gsplat_mi355x.h"

namespace {

constexpr int kT = 16;                       // output tile edge
constexpr int kThreads = kT * kT;            // 256
constexpr int kMaxR = GS_LOSS_MAX_WINDOW / 2;
constexpr int kP = kT + 2 * kMaxR;           // patch edge at the largest window

struct Window {
  float w[GS_LOSS_MAX_WINDOW];
  int r;  // radius: window = 2r + 1
};

__device__ __forceinline__ float block_sum(float v, float *s_red) {
  // fixed-order: wave shuffle tree, then the 4 wave sums in order
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  const int wave = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s_red[wave] = v;
  __syncthreads();
  return (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

__global__ __launch_bounds__(kThreads) void k_loss_fwd(gs_loss_args a, Window win, float2 *partials) {
  __shared__ float sx[kP][kP + 1], sy[kP][kP + 1];
  __shared__ float sh[5][kP][kT + 1];
  __shared__ float s_red[4];
  const int H = a.height, W = a.width, c = blockIdx.z, R = win.r, P = kT + 2 * R;
  const int x0 = blockIdx.x * kT, y0 = blockIdx.y * kT;
  const size_t plane = (size_t)H * W;
  const float *px = a.pred + c * plane, *py = a.target + c * plane;
  for (int i = threadIdx.x; i < P * P; i += kThreads) {
    const int r = i / P, q = i % P, gy = y0 - R + r, gx = x0 - R + q;
    const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
    sx[r][q] = in ? px[(size_t)gy * W + gx] : 0.f;
    sy[r][q] = in ? py[(size_t)gy * W + gx] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P * kT; i += kThreads) {  // horizontal pass
    const int r = i / kT, q = i % kT;
    float h0 = 0.f, h1 = 0.f, h2 = 0.f, h3 = 0.f, h4 = 0.f;
    for (int k = 0; k <= 2 * R; ++k) {
      const float w = win.w[k], u = sx[r][q + k], v = sy[r][q + k];
      h0 = __builtin_fmaf(w, u, h0);
      h1 = __builtin_fmaf(w, v, h1);
      h2 = __builtin_fmaf(w, u * u, h2);
      h3 = __builtin_fmaf(w, v * v, h3);
      h4 = __builtin_fmaf(w, u * v, h4);
    }
    sh[0][r][q] = h0; sh[1][r][q] = h1; sh[2][r][q] = h2; sh[3][r][q] = h3; sh[4][r][q] = h4;
  }
  __syncthreads();
  const int oy = threadIdx.x / kT, ox = threadIdx.x % kT, gy = y0 + oy, gx = x0 + ox;
  float mx = 0.f, my = 0.f, exx = 0.f, eyy = 0.f, exy = 0.f;
  for (int k = 0; k <= 2 * R; ++k) {  // vertical pass
    const float w = win.w[k];
    mx = __builtin_fmaf(w, sh[0][oy + k][ox], mx);
    my = __builtin_fmaf(w, sh[1][oy + k][ox], my);
    exx = __builtin_fmaf(w, sh[2][oy + k][ox], exx);
    eyy = __builtin_fmaf(w, sh[3][oy + k][ox], eyy);
    exy = __builtin_fmaf(w, sh[4][oy + k][ox], exy);
  }
  float ssim_c = 0.f, l1 = 0.f;
  if (gy < H && gx < W) {
    const float x = sx[oy + R][ox + R], y = sy[oy + R][ox + R];
    l1 = fabsf(x - y);
    // loss.py:33-38
    const float sxx = exx - mx * mx, syy = eyy - my * my, sxy = exy - mx * my;
    const float A1 = 2.f * mx * my + a.c1, A2 = 2.f * sxy + a.c2;
    const float B1 = mx * mx + my * my + a.c1, B2 = sxx + syy + a.c2;
    const float D = B1 * B2, S = (A1 * A2) / D;
    ssim_c = fminf(fmaxf(S, 0.f), 1.f);  // loss.py:39 (NaN -> 0 here; torch would keep NaN)
    if (a.maps) {
      // d clamp(S)/dS: 1 on [0,1] (torch clamp_backward, boundary-inclusive), else 0
      const float g = (S >= 0.f && S <= 1.f) ? 1.f : 0.f;
      const float iD = 1.f / D;
      const float d_mu = g * 2.f * iD * (my * (A2 - A1) - S * mx * (B2 - B1));
      const float d_exx = g * (-S / B2);
      const float d_exy = g * 2.f * A1 * iD;
      const size_t o = c * plane + (size_t)gy * W + gx, n = (size_t)a.channels * plane;
      a.maps[o] = d_mu;
      a.maps[n + o] = d_exx;
      a.maps[2 * n + o] = d_exy;
    }
  }
  const float ss = block_sum(ssim_c, s_red);
  const float sl = block_sum(l1, s_red);
  if (threadIdx.x == 0)
    partials[((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = make_float2(ss, sl);
}

__global__ __launch_bounds__(1024) void k_loss_final(gs_loss_args a, const float2 *partials, int nb) {
  __shared__ double s_a[1024], s_b[1024];
  double sa = 0.0, sb = 0.0;
  for (int i = threadIdx.x; i < nb; i += 1024) {
    sa += (double)partials[i].x;
    sb += (double)partials[i].y;
  }
  s_a[threadIdx.x] = sa;
  s_b[threadIdx.x] = sb;
  __syncthreads();
  for (int d = 512; d >= 1; d >>= 1) {
    if ((int)threadIdx.x < d) {
      s_a[threadIdx.x] += s_a[threadIdx.x + d];
      s_b[threadIdx.x] += s_b[threadIdx.x + d];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double n = (double)a.channels * a.height * a.width;
    const float l1 = (float)(s_b[0] / n), dssim = (float)(1.0 - s_a[0] / n);
    a.out[0] = (1.f - a.lambda_dssim) * l1 + a.lambda_dssim * dssim;  // loss.py:58
    a.out[1] = l1;
    a.out[2] = dssim;
  }
}

__global__ __launch_bounds__(kThreads) void k_loss_bwd(gs_loss_args a, Window win) {
  __shared__ float sm[3][kP][kP + 1];
  __shared__ float sh[3][kP][kT + 1];
  const int H = a.height, W = a.width, c = blockIdx.z, R = win.r, P = kT + 2 * R;
  const int x0 = blockIdx.x * kT, y0 = blockIdx.y * kT;
  const size_t plane = (size_t)H * W, n = (size_t)a.channels * plane;
  const float *m = a.maps + c * plane;
  for (int i = threadIdx.x; i < P * P; i += kThreads) {
    const int r = i / P, q = i % P, gy = y0 - R + r, gx = x0 - R + q;
    const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
    const size_t o = (size_t)gy * W + gx;
    sm[0][r][q] = in ? m[o] : 0.f;
    sm[1][r][q] = in ? m[n + o] : 0.f;
    sm[2][r][q] = in ? m[2 * n + o] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P * kT; i += kThreads) {
    const int r = i / kT, q = i % kT;
    float h0 = 0.f, h1 = 0.f, h2 = 0.f;
    for (int k = 0; k <= 2 * R; ++k) {
      const float w = win.w[k];
      h0 = __builtin_fmaf(w, sm[0][r][q + k], h0);
      h1 = __builtin_fmaf(w, sm[1][r][q + k], h1);
      h2 = __builtin_fmaf(w, sm[2][r][q + k], h2);
    }
    sh[0][r][q] = h0; sh[1][r][q] = h1; sh[2][r][q] = h2;
  }
  __syncthreads();
  const int oy = threadIdx.x / kT, ox = threadIdx.x % kT, gy = y0 + oy, gx = x0 + ox;
  if (gy >= H || gx >= W) return;
  float b0 = 0.f, b1 = 0.f, b2 = 0.f;
  for (int k = 0; k <= 2 * R; ++k) {
    const float w = win.w[k];
    b0 = __builtin_fmaf(w, sh[0][oy + k][ox], b0);
    b1 = __builtin_fmaf(w, sh[1][oy + k][ox], b1);
    b2 = __builtin_fmaf(w, sh[2][oy + k][ox], b2);
  }
  const size_t o = c * plane + (size_t)gy * W + gx;
  const float x = a.pred[o], y = a.target[o];
  const float inv_n = 1.f / (float)n;
  const float gt = a.g_total ? *a.g_total : 1.f;
  const float sgn = x > y ? 1.f : (x < y ? -1.f : 0.f);  // abs backward (sign, 0 at 0)
  const float d_ssim = b0 + 2.f * x * b1 + y * b2;     // d(sum of clamped SSIM)/dx
  a.d_pred[o] = gt * (((1.f - a.lambda_dssim) * inv_n) * sgn - (a.lambda_dssim * inv_n) * d_ssim);
}

bool window_of(int k, Window &win) {
  if (k < 1 || k > GS_LOSS_MAX_WINDOW || (k & 1) == 0) return false;
  // loss.py:20-23: x = arange(K) - (K-1)/2; g = exp(-x^2 / (2 (K/6)^2)); g /= sum
  double g[GS_LOSS_MAX_WINDOW], s = 0.0;
  const double sig = k / 6.0;
  for (int i = 0; i < k; ++i) {
    const double x = i - (k - 1) / 2.0;
    g[i] = exp(-x * x / (2.0 * sig * sig));
    s += g[i];
  }
  for (int i = 0; i < GS_LOSS_MAX_WINDOW; ++i) win.w[i] = i < k ? (float)(g[i] / s) : 0.f;
  win.r = k / 2;
  return true;
}

inline unsigned blocks_of(int v) { return (unsigned)((v + kT - 1) / kT); }

}  // namespace

extern "C" size_t gs_loss_workspace_bytes(int32_t channels, int32_t height, int32_t width) {
  if (channels <= 0 || height <= 0 || width <= 0) return 0;
  return sizeof(float2) * (size_t)blocks_of(width) * blocks_of(height) * channels;
}

extern "C" gs_status gs_loss_forward(const gs_loss_args *a, gs_stream_t stream) {
  if (!a) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_loss_forward");
  Window win;
  if (!window_of(a->window, win)) return gs_internal_fail(GS_ERR_UNSUPPORTED, "%s: window must be odd, 1..11", "gs_loss_forward");
  if (a->channels <= 0 || a->height <= 0 || a->width <= 0 || a->height > 65535 * kT || a->channels > 65535)
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: bad shape", "gs_loss_forward");
  if (!a->pred || !a->target || !a->out || !a->workspace ||
      a->workspace_bytes < gs_loss_workspace_bytes(a->channels, a->height, a->width))
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null buffer or small workspace", "gs_loss_forward");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(blocks_of(a->width), blocks_of(a->height), a->channels);
  float2 *partials = (float2 *)a->workspace;
  k_loss_fwd<<<grid, kThreads, 0, s>>>(*a, win, partials);
  k_loss_final<<<1, 1024, 0, s>>>(*a, partials, (int)(grid.x * grid.y * grid.z));
  return gs_internal_check_launch("gs_loss_forward");
}

extern "C" gs_status gs_loss_backward(const gs_loss_args *a, gs_stream_t stream) {
  if (!a) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_loss_backward");
  Window win;
  if (!window_of(a->window, win)) return gs_internal_fail(GS_ERR_UNSUPPORTED, "%s: window must be odd, 1..11", "gs_loss_backward");
  if (a->channels <= 0 || a->height <= 0 || a->width <= 0 || a->height > 65535 * kT || a->channels > 65535)
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: bad shape", "gs_loss_backward");
  if (!a->pred || !a->target || !a->maps || !a->d_pred)
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null buffer", "gs_loss_backward");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(blocks_of(a->width), blocks_of(a->height), a->channels);
  k_loss_bwd<<<grid, kThreads, 0, s>>>(*a, win);
  return gs_internal_check_launch("gs_loss_backward");
}
