// gs_loss.hip -- fused L1 + D-SSIM photometric loss, forward and backward
// (include/gsplat_mi355x.h, "Photometric loss").
//
// Forward, one 256-thread workgroup per 32x32 output tile of one channel:
// the (32+2R)^2 patch of pred and target goes to LDS (zero outside the
// image = the reference's conv2d zero padding).  A horizontal pass forms the
// five windowed sums (x, y, x^2, y^2, xy) per patch row, each thread item
// sliding over 4 adjacent outputs from registers; a vertical pass gives every
// thread one column of 4 output rows, again from registers.  The taps of
// every sum are accumulated in window order (fma), as a single-output loop
// would.  Each pixel then has its SSIM, |x - y| and the three partial
// derivatives of its clamped SSIM with respect to (mu_x, E[x^2], E[xy]); the
// workgroup writes its two partial sums (fixed-order tree), and a
// one-workgroup kernel reduces them in fixed order, in double.
// Backward: dL/dx_p = blur(m1)(p) + 2 x_p blur(m2)(p) + y_p blur(m3)(p)
// (the window is symmetric, so the adjoint of the zero-padded blur is the
// same blur), scaled by -lambda / (CHW), plus (1 - lambda) sign(x - y) / (CHW).
// Kernels are instantiated per window radius (taps unrolled, weights in
// registers).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gs_internal.h"
#include "gsplat_mi355x.h"

namespace {

constexpr int kTW = 32;                      // output tile width
constexpr int kTH = 32;                      // output tile height
constexpr int kThreads = 256;
constexpr int kRows = kTW * kTH / kThreads;  // vertical pass: output rows per thread
constexpr int kSeg = 4;                      // horizontal pass: outputs per thread item
constexpr int kSegs = kTW / kSeg;
constexpr int kMaxR = GS_LOSS_MAX_WINDOW / 2;
static_assert(kThreads % kTW == 0 && kRows * kThreads == kTW * kTH, "tile / block shape");

typedef float f2 __attribute__((ext_vector_type(2)));

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

// Output tiles in (channel, row, column) order; tile t's partial sums go to
// partials[t].  Workgroups go to the 8 XCDs round-robin by linear id, and
// each XCD has its own L2: block b is given tile
//   (b mod 8) * floor(n/8) + min(b mod 8, n mod 8) + floor(b/8),
// so each XCD works through one contiguous run of tile rows and the halo
// rows a tile shares with its neighbours are fetched from HBM once per run
// rather than once per tile (measured: the default order fetched every
// patch whole, ~1.7x the image per plane).
struct Tile {
  int x0, y0, c;
};
struct Tiles {
  int tx, per_c, n;
  __device__ explicit Tiles(const gs_loss_args &a)
      : tx((a.width + kTW - 1) / kTW), per_c(tx * ((a.height + kTH - 1) / kTH)), n(per_c * a.channels) {}
  __device__ int of_block(int b) const {
    const int x = b & 7, per = n >> 3, rem = n & 7;
    return x * per + (x < rem ? x : rem) + (b >> 3);
  }
  __device__ Tile at(int t) const {
    const int c = t / per_c, r = t - c * per_c, y = r / tx;
    return Tile{(r - y * tx) * kTW, y * kTH, c};
  }
};

template <int R>
__global__ __launch_bounds__(kThreads) void k_loss_fwd(gs_loss_args a, Window win, float2 *partials) {
  constexpr int K = 2 * R + 1, PH = kTH + 2 * R, PW = kTW + 2 * R;
  // The patch is held as (x, y) pairs and the row sums as (x, y), (x^2, y^2)
  // pairs plus xy, so two of every three sums advance by one packed fp32 FMA
  // (each half an ordinary fp32 fma: the same values as scalar code).  The
  // patch and the row sums share one LDS buffer: the row sums wait in
  // registers until every thread has read its patch rows.
  constexpr int kPatch = 2 * PH * (PW + 1), kSums = 5 * PH * (kTW + 1);
  __shared__ __attribute__((aligned(16))) float smem[kPatch > kSums ? kPatch : kSums];
  __shared__ float s_red[4];
  auto sxy = reinterpret_cast<f2(*)[PW + 1]>(smem);
  auto s01 = reinterpret_cast<f2(*)[kTW + 1]>(smem);
  auto s23 = reinterpret_cast<f2(*)[kTW + 1]>(smem + 2 * PH * (kTW + 1));
  auto s4 = reinterpret_cast<float(*)[kTW + 1]>(smem + 4 * PH * (kTW + 1));
  float w[K];
#pragma unroll
  for (int k = 0; k < K; ++k) w[k] = win.w[k];
  const int H = a.height, W = a.width;
  const Tiles tl(a);
  const int t = tl.of_block(blockIdx.x);
  const Tile tc = tl.at(t);
  const int c = tc.c, x0 = tc.x0, y0 = tc.y0;
  const size_t plane = (size_t)H * W;
  const float *px = a.pred + c * plane, *py = a.target + c * plane;
  // patch load: every load of the thread in flight before the first LDS store
  constexpr int kLoads = (PH * PW + kThreads - 1) / kThreads;
  f2 lxy[kLoads];
#pragma unroll
  for (int it = 0; it < kLoads; ++it) {
    const int i = threadIdx.x + it * kThreads, r = i / PW, q = i - r * PW, gy = y0 - R + r, gx = x0 - R + q;
    const bool in = i < PH * PW && gy >= 0 && gy < H && gx >= 0 && gx < W;
    lxy[it].x = in ? px[(size_t)gy * W + gx] : 0.f;
    lxy[it].y = in ? py[(size_t)gy * W + gx] : 0.f;
  }
#pragma unroll
  for (int it = 0; it < kLoads; ++it) {
    const int i = threadIdx.x + it * kThreads, r = i / PW, q = i - r * PW;
    if (i < PH * PW) sxy[r][q] = lxy[it];
  }
  __syncthreads();
  constexpr int kItems = (PH * kSegs + kThreads - 1) / kThreads;
  f2 hm[kItems][kSeg], hq[kItems][kSeg];  // (sum x, sum y), (sum x^2, sum y^2)
  float hp[kItems][kSeg];                  // sum xy
#pragma unroll
  for (int it = 0; it < kItems; ++it) {  // horizontal pass
    const int i = threadIdx.x + it * kThreads, r = i / kSegs, q0 = (i % kSegs) * kSeg;
    if (i >= PH * kSegs) break;
    f2 v[kSeg + 2 * R], sq[kSeg + 2 * R];
    float pr[kSeg + 2 * R];
#pragma unroll
    for (int j = 0; j < kSeg + 2 * R; ++j) {
      v[j] = sxy[r][q0 + j];
      sq[j] = v[j] * v[j];
      pr[j] = v[j].x * v[j].y;
    }
#pragma unroll
    for (int o = 0; o < kSeg; ++o) {
      f2 m = {0.f, 0.f}, q2 = {0.f, 0.f};
      float pp = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const f2 wk = {w[k], w[k]};
        m = __builtin_elementwise_fma(wk, v[o + k], m);
        q2 = __builtin_elementwise_fma(wk, sq[o + k], q2);
        pp = __builtin_fmaf(w[k], pr[o + k], pp);
      }
      hm[it][o] = m; hq[it][o] = q2; hp[it][o] = pp;
    }
  }
  const int col = threadIdx.x % kTW, r0 = (threadIdx.x / kTW) * kRows, gx = x0 + col;
  float xc[kRows], yc[kRows];  // this thread's output pixels, fetched while the row sums settle
#pragma unroll
  for (int o = 0; o < kRows; ++o) {
    const int gy = y0 + r0 + o;
    const bool in = gy < H && gx < W;
    xc[o] = in ? px[(size_t)gy * W + gx] : 0.f;
    yc[o] = in ? py[(size_t)gy * W + gx] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const int i = threadIdx.x + it * kThreads, r = i / kSegs, q0 = (i % kSegs) * kSeg;
    if (i >= PH * kSegs) break;
#pragma unroll
    for (int o = 0; o < kSeg; ++o) {
      s01[r][q0 + o] = hm[it][o];
      s23[r][q0 + o] = hq[it][o];
      s4[r][q0 + o] = hp[it][o];
    }
  }
  __syncthreads();
  f2 am[kRows], aq[kRows];
  float ap[kRows];
#pragma unroll
  for (int o = 0; o < kRows; ++o) {
    am[o] = aq[o] = (f2){0.f, 0.f};
    ap[o] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < kRows + 2 * R; ++j) {  // vertical pass: row j feeds output o at tap j - o
    const f2 m = s01[r0 + j][col], q2 = s23[r0 + j][col];
    const float pp = s4[r0 + j][col];
#pragma unroll
    for (int o = 0; o < kRows; ++o) {
      const int k = j - o;
      if (k >= 0 && k < K) {
        const f2 wk = {w[k], w[k]};
        am[o] = __builtin_elementwise_fma(wk, m, am[o]);
        aq[o] = __builtin_elementwise_fma(wk, q2, aq[o]);
        ap[o] = __builtin_fmaf(w[k], pp, ap[o]);
      }
    }
  }
  const size_t n = (size_t)a.channels * plane;
  float ss = 0.f, sl = 0.f;
#pragma unroll
  for (int o = 0; o < kRows; ++o) {
    const int gy = y0 + r0 + o;
    if (gy >= H || gx >= W) continue;
    const float mx = am[o].x, my = am[o].y, exx = aq[o].x, eyy = aq[o].y, exy = ap[o];
    const float x = xc[o], y = yc[o];
    sl += fabsf(x - y);
    // loss.py:33-38
    const float sxx = exx - mx * mx, syy = eyy - my * my, sxy = exy - mx * my;
    const float A1 = 2.f * mx * my + a.c1, A2 = 2.f * sxy + a.c2;
    const float B1 = mx * mx + my * my + a.c1, B2 = sxx + syy + a.c2;
    const float D = B1 * B2, S = (A1 * A2) / D;
    ss += fminf(fmaxf(S, 0.f), 1.f);  // loss.py:39 (NaN -> 0 here; torch would keep NaN)
    if (a.maps) {
      // d clamp(S)/dS: 1 on [0,1] (torch clamp_backward, boundary-inclusive), else 0
      const float g = (S >= 0.f && S <= 1.f) ? 1.f : 0.f;
      const float iD = 1.f / D;
      const size_t p = c * plane + (size_t)gy * W + gx;
      a.maps[p] = g * 2.f * iD * (my * (A2 - A1) - S * mx * (B2 - B1));  // d/d mu_x
      a.maps[n + p] = g * (-S / B2);                                     // d/d E[x^2]
      a.maps[2 * n + p] = g * 2.f * A1 * iD;                             // d/d E[xy]
    }
  }
  ss = block_sum(ss, s_red);
  sl = block_sum(sl, s_red);
  if (threadIdx.x == 0) partials[t] = make_float2(ss, sl);
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

template <int R>
__global__ __launch_bounds__(kThreads) void k_loss_bwd(gs_loss_args a, Window win) {
  constexpr int K = 2 * R + 1, PH = kTH + 2 * R, PW = kTW + 2 * R;
  // maps 1 and 2 travel as a pair (packed fp32 FMA), map 3 alone; patch and
  // row sums share LDS, as in the forward
  constexpr int kPatch = 3 * PH * (PW + 1), kSums = 3 * PH * (kTW + 1);
  __shared__ __attribute__((aligned(16))) float smem[kPatch > kSums ? kPatch : kSums];
  auto sp = reinterpret_cast<f2(*)[PW + 1]>(smem);
  auto s2 = reinterpret_cast<float(*)[PW + 1]>(smem + 2 * PH * (PW + 1));
  auto hp = reinterpret_cast<f2(*)[kTW + 1]>(smem);
  auto h2 = reinterpret_cast<float(*)[kTW + 1]>(smem + 2 * PH * (kTW + 1));
  float w[K];
#pragma unroll
  for (int k = 0; k < K; ++k) w[k] = win.w[k];
  const int H = a.height, W = a.width;
  const Tiles tl(a);
  const Tile tc = tl.at(tl.of_block(blockIdx.x));
  const int c = tc.c, x0 = tc.x0, y0 = tc.y0;
  const size_t plane = (size_t)H * W, n = (size_t)a.channels * plane;
  const float *m = a.maps + c * plane;
  constexpr int kLoads = (PH * PW + kThreads - 1) / kThreads;  // all in flight, as in the forward
  f2 l01[kLoads];
  float l2[kLoads];
#pragma unroll
  for (int it = 0; it < kLoads; ++it) {
    const int i = threadIdx.x + it * kThreads, r = i / PW, q = i - r * PW, gy = y0 - R + r, gx = x0 - R + q;
    const bool in = i < PH * PW && gy >= 0 && gy < H && gx >= 0 && gx < W;
    const size_t o = (size_t)gy * W + gx;
    l01[it].x = in ? m[o] : 0.f;
    l01[it].y = in ? m[n + o] : 0.f;
    l2[it] = in ? m[2 * n + o] : 0.f;
  }
#pragma unroll
  for (int it = 0; it < kLoads; ++it) {
    const int i = threadIdx.x + it * kThreads, r = i / PW, q = i - r * PW;
    if (i < PH * PW) {
      sp[r][q] = l01[it];
      s2[r][q] = l2[it];
    }
  }
  __syncthreads();
  constexpr int kItems = (PH * kSegs + kThreads - 1) / kThreads;
  f2 hs01[kItems][kSeg];
  float hs2[kItems][kSeg];
#pragma unroll
  for (int it = 0; it < kItems; ++it) {  // horizontal pass
    const int i = threadIdx.x + it * kThreads, r = i / kSegs, q0 = (i % kSegs) * kSeg;
    if (i >= PH * kSegs) break;
    f2 u01[kSeg + 2 * R];
    float u2[kSeg + 2 * R];
#pragma unroll
    for (int j = 0; j < kSeg + 2 * R; ++j) {
      u01[j] = sp[r][q0 + j];
      u2[j] = s2[r][q0 + j];
    }
#pragma unroll
    for (int o = 0; o < kSeg; ++o) {
      f2 b01 = {0.f, 0.f};
      float b2 = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        b01 = __builtin_elementwise_fma((f2){w[k], w[k]}, u01[o + k], b01);
        b2 = __builtin_fmaf(w[k], u2[o + k], b2);
      }
      hs01[it][o] = b01;
      hs2[it][o] = b2;
    }
  }
  const int col = threadIdx.x % kTW, r0 = (threadIdx.x / kTW) * kRows, gx = x0 + col;
  float xc[kRows], yc[kRows];  // this thread's output pixels, fetched while the row sums settle
#pragma unroll
  for (int o = 0; o < kRows; ++o) {
    const int gy = y0 + r0 + o;
    const bool in = gy < H && gx < W;
    const size_t p = c * plane + (size_t)gy * W + gx;
    xc[o] = in ? a.pred[p] : 0.f;
    yc[o] = in ? a.target[p] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const int i = threadIdx.x + it * kThreads, r = i / kSegs, q0 = (i % kSegs) * kSeg;
    if (i >= PH * kSegs) break;
#pragma unroll
    for (int o = 0; o < kSeg; ++o) {
      hp[r][q0 + o] = hs01[it][o];
      h2[r][q0 + o] = hs2[it][o];
    }
  }
  __syncthreads();
  f2 a01[kRows];
  float a2[kRows];
#pragma unroll
  for (int o = 0; o < kRows; ++o) {
    a01[o] = (f2){0.f, 0.f};
    a2[o] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < kRows + 2 * R; ++j) {
    const f2 b01 = hp[r0 + j][col];
    const float b2 = h2[r0 + j][col];
#pragma unroll
    for (int o = 0; o < kRows; ++o) {
      const int k = j - o;
      if (k >= 0 && k < K) {
        a01[o] = __builtin_elementwise_fma((f2){w[k], w[k]}, b01, a01[o]);
        a2[o] = __builtin_fmaf(w[k], b2, a2[o]);
      }
    }
  }
  const float inv_n = 1.f / (float)n;
  const float gt = a.g_total ? *a.g_total : 1.f;
#pragma unroll
  for (int o = 0; o < kRows; ++o) {
    const int gy = y0 + r0 + o;
    if (gy >= H || gx >= W) continue;
    const size_t p = c * plane + (size_t)gy * W + gx;
    const float x = xc[o], y = yc[o];
    const float sgn = x > y ? 1.f : (x < y ? -1.f : 0.f);  // abs backward (sign, 0 at 0)
    const float d_ssim = a01[o].x + 2.f * x * a01[o].y + y * a2[o];  // d(sum of clamped SSIM)/dx
    a.d_pred[p] = gt * (((1.f - a.lambda_dssim) * inv_n) * sgn - (a.lambda_dssim * inv_n) * d_ssim);
  }
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

inline unsigned blocks_of(int v, int t) { return (unsigned)((v + t - 1) / t); }

inline int tiles_of(const gs_loss_args &a) {
  return (int)(blocks_of(a.width, kTW) * blocks_of(a.height, kTH)) * a.channels;
}

template <int R>
void launch_fwd(const gs_loss_args &a, const Window &win, float2 *partials, hipStream_t s) {
  k_loss_fwd<R><<<tiles_of(a), kThreads, 0, s>>>(a, win, partials);
}

template <int R>
void launch_bwd(const gs_loss_args &a, const Window &win, hipStream_t s) {
  k_loss_bwd<R><<<tiles_of(a), kThreads, 0, s>>>(a, win);
}

using FwdLaunch = void (*)(const gs_loss_args &, const Window &, float2 *, hipStream_t);
using BwdLaunch = void (*)(const gs_loss_args &, const Window &, hipStream_t);
static_assert(kMaxR == 5, "one instantiation per window radius 0..kMaxR");
constexpr FwdLaunch kFwd[kMaxR + 1] = {launch_fwd<0>, launch_fwd<1>, launch_fwd<2>,
                                       launch_fwd<3>, launch_fwd<4>, launch_fwd<5>};
constexpr BwdLaunch kBwd[kMaxR + 1] = {launch_bwd<0>, launch_bwd<1>, launch_bwd<2>,
                                       launch_bwd<3>, launch_bwd<4>, launch_bwd<5>};

}  // namespace

extern "C" size_t gs_loss_workspace_bytes(int32_t channels, int32_t height, int32_t width) {
  if (channels <= 0 || height <= 0 || width <= 0) return 0;
  return sizeof(float2) * (size_t)blocks_of(width, kTW) * blocks_of(height, kTH) * channels;
}

extern "C" gs_status gs_loss_forward(const gs_loss_args *a, gs_stream_t stream) {
  if (!a) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_loss_forward");
  Window win;
  if (!window_of(a->window, win)) return gs_internal_fail(GS_ERR_UNSUPPORTED, "%s: window must be odd, 1..11", "gs_loss_forward");
  if (a->channels <= 0 || a->height <= 0 || a->width <= 0 || (double)blocks_of(a->width, kTW) * blocks_of(a->height, kTH) * a->channels > 2147483647.0)
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: bad shape", "gs_loss_forward");
  if (!a->pred || !a->target || !a->out || !a->workspace ||
      a->workspace_bytes < gs_loss_workspace_bytes(a->channels, a->height, a->width))
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null buffer or small workspace", "gs_loss_forward");
  hipStream_t s = (hipStream_t)stream;
  float2 *partials = (float2 *)a->workspace;
  kFwd[win.r](*a, win, partials, s);
  k_loss_final<<<1, 1024, 0, s>>>(*a, partials, tiles_of(*a));
  return gs_internal_check_launch("gs_loss_forward");
}

extern "C" gs_status gs_loss_backward(const gs_loss_args *a, gs_stream_t stream) {
  if (!a) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null args", "gs_loss_backward");
  Window win;
  if (!window_of(a->window, win)) return gs_internal_fail(GS_ERR_UNSUPPORTED, "%s: window must be odd, 1..11", "gs_loss_backward");
  if (a->channels <= 0 || a->height <= 0 || a->width <= 0 || (double)blocks_of(a->width, kTW) * blocks_of(a->height, kTH) * a->channels > 2147483647.0)
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: bad shape", "gs_loss_backward");
  if (!a->pred || !a->target || !a->maps || !a->d_pred)
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null buffer", "gs_loss_backward");
  hipStream_t s = (hipStream_t)stream;
  kBwd[win.r](*a, win, s);
  return gs_internal_check_launch("gs_loss_backward");
}
