// gs_densify.hip -- split / clone / prune of the Gaussian set in one
// compaction pass, with the Adam moments remapped (include/gsplat_mi355x.h,
// "Densification").
//
// Count: one thread per Gaussian classifies it (keep / split / clone, each
// output subject to the opacity prune) and every 256-Gaussian block writes
// its four category counts.  Scan: one workgroup turns them into per-block
// bases (fixed order).  Emit: the same classification, block-local
// exclusive scans and the bases give every output row its index; outputs are
// grouped [kept | split - | split + | clones], index order within each.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gs_internal.h"
#include "gsplat_mi355x.h"

namespace {

constexpr int kB = 256;

struct Cls {
  bool keep, split, clone;  // outputs this Gaussian produces (after the prune)
  float smean;              // mean(exp(scaling))
  float child_op;           // split children's opacity logit
};

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

__device__ Cls classify(const gs_densify_args &a, int i) {
  Cls c{};
  const float *sc = a.in.scaling + 3 * (size_t)i;
  c.smean = ((expf(sc[0]) + expf(sc[1])) + expf(sc[2])) / 3.f;  // get_scaling.mean(dim=-1)
  const float op = a.in.opacity[i];
  const bool prune = (a.flags & GS_DENSIFY_PRUNE) != 0;
  const bool alive = !prune || sigmoidf_(op) > a.min_opacity;  // optimizer.py:64
  bool split = false, clone = false;
  if (a.xyz_grad) {
    const float *g = a.xyz_grad + 3 * (size_t)i;
    const float gn = sqrtf((g[0] * g[0] + g[1] * g[1]) + g[2] * g[2]);  // .norm(dim=-1)
    const bool hot = gn > a.grad_threshold;
    split = (a.flags & GS_DENSIFY_SPLIT) && hot && c.smean > a.split_size * a.scene_extent;   // :137
    clone = (a.flags & GS_DENSIFY_CLONE) && hot && c.smean < a.clone_size * a.scene_extent;   // :166
  }
  // children: clamp(logit(get_opacity), -6, 6) (:150)
  const float o = sigmoidf_(op);
  c.child_op = fminf(fmaxf(logf(o / (1.f - o)), -6.f), 6.f);
  const bool child_alive = !prune || sigmoidf_(c.child_op) > a.min_opacity;
  c.keep = !split && alive;
  c.split = split && child_alive;
  c.clone = clone && alive;
  return c;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// standard normal from (seed, i, k): Box-Muller on two 24-bit uniforms
__device__ float normal_of(uint64_t seed, uint32_t i, uint32_t k) {
  const uint64_t h = mix64(seed ^ mix64((uint64_t)i * 4u + k));
  const float u1 = (float)((h >> 40) + 1ull) * 0x1p-24f;  // (0, 1]
  const float u2 = (float)((h >> 16) & 0xFFFFFFull) * 0x1p-24f;
  return sqrtf(-2.f * logf(u1)) * cosf(6.283185307179586f * u2);
}

__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *s_tmp, uint32_t *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  if (lane == 63) s_tmp[wave] = incl;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kB / 64; ++w) {
    const uint32_t x = s_tmp[w];
    base += (w < wave) ? x : 0u;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

__global__ __launch_bounds__(kB) void k_densify_count(gs_densify_args a, uint32_t *part) {
  __shared__ uint32_t s_tmp[4];
  const int i = blockIdx.x * kB + threadIdx.x;
  Cls c{};
  if (i < a.n) c = classify(a, i);
  uint32_t t0, t1, t2;
  block_exscan(c.keep, s_tmp, &t0);
  block_exscan(c.split, s_tmp, &t1);
  block_exscan(c.clone, s_tmp, &t2);
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x] = t0;
    part[3 * blockIdx.x + 1] = t1;
    part[3 * blockIdx.x + 2] = t2;
  }
}

// exclusive scan of the per-block counts of each category, in place
__global__ __launch_bounds__(kB) void k_densify_scan(uint32_t *part, int nb, uint32_t *counters) {
  __shared__ uint32_t s_tmp[4];
  uint32_t tot[3];
  for (int c = 0; c < 3; ++c) {
    uint32_t carry = 0;
    for (int b0 = 0; b0 < nb; b0 += kB) {
      const int b = b0 + threadIdx.x;
      const uint32_t v = b < nb ? part[3 * b + c] : 0u;
      uint32_t t;
      const uint32_t e = block_exscan(v, s_tmp, &t);
      if (b < nb) part[3 * b + c] = carry + e;
      carry += t;
    }
    tot[c] = carry;
  }
  if (threadIdx.x == 0) {
    counters[0] = tot[0];
    counters[1] = tot[1];
    counters[2] = tot[2];
    counters[3] = tot[0] + 2u * tot[1] + tot[2];
  }
}

__device__ __forceinline__ void copy_row(const float *src, float *dst, int n) {
  if (!src || !dst) return;
  for (int k = 0; k < n; ++k) dst[k] = src[k];
}
__device__ __forceinline__ void zero_row(float *dst, int n) {
  if (!dst) return;
  for (int k = 0; k < n; ++k) dst[k] = 0.f;
}

// one output row: params (from p / explicit values) and, if remapped, Adam moments
__device__ void write_moments(const gs_densify_args &a, int i, size_t o, bool carry) {
  const gs_model_arrays *mi[2] = {&a.adam_m_in, &a.adam_v_in};
  const gs_model_arrays *mo[2] = {&a.adam_m_out, &a.adam_v_out};
  for (int t = 0; t < 2; ++t) {
    const gs_model_arrays &I = *mi[t];
    const gs_model_arrays &O = *mo[t];
    if (carry) {
      copy_row(I.xyz ? I.xyz + 3 * (size_t)i : nullptr, O.xyz ? O.xyz + 3 * o : nullptr, 3);
      copy_row(I.features_dc ? I.features_dc + 3 * (size_t)i : nullptr, O.features_dc ? O.features_dc + 3 * o : nullptr, 3);
      copy_row(I.features_rest ? I.features_rest + (size_t)a.rest_floats * i : nullptr,
               O.features_rest ? O.features_rest + (size_t)a.rest_floats * o : nullptr, a.rest_floats);
      copy_row(I.scaling ? I.scaling + 3 * (size_t)i : nullptr, O.scaling ? O.scaling + 3 * o : nullptr, 3);
      copy_row(I.rotation ? I.rotation + 4 * (size_t)i : nullptr, O.rotation ? O.rotation + 4 * o : nullptr, 4);
      copy_row(I.opacity ? I.opacity + i : nullptr, O.opacity ? O.opacity + o : nullptr, 1);
    } else {
      zero_row(O.xyz ? O.xyz + 3 * o : nullptr, 3);
      zero_row(O.features_dc ? O.features_dc + 3 * o : nullptr, 3);
      zero_row(O.features_rest ? O.features_rest + (size_t)a.rest_floats * o : nullptr, a.rest_floats);
      zero_row(O.scaling ? O.scaling + 3 * o : nullptr, 3);
      zero_row(O.rotation ? O.rotation + 4 * o : nullptr, 4);
      zero_row(O.opacity ? O.opacity + o : nullptr, 1);
    }
  }
}

__global__ __launch_bounds__(kB) void k_densify_emit(gs_densify_args a, const uint32_t *part) {
  __shared__ uint32_t s_tmp[4];
  const int i = blockIdx.x * kB + threadIdx.x;
  Cls c{};
  if (i < a.n) c = classify(a, i);
  uint32_t t;
  const uint32_t lk = block_exscan(c.keep, s_tmp, &t);
  const uint32_t ls = block_exscan(c.split, s_tmp, &t);
  const uint32_t lc = block_exscan(c.clone, s_tmp, &t);
  if (i >= a.n) return;
  const uint32_t nk = a.counters[0], ns = a.counters[1];
  const gs_model_arrays &in = a.in, &out = a.out;
  const int R = a.rest_floats;
  const float *xyz = in.xyz + 3 * (size_t)i, *fdc = in.features_dc + 3 * (size_t)i;
  const float *frest = in.features_rest ? in.features_rest + (size_t)R * i : nullptr;
  const float *scl = in.scaling + 3 * (size_t)i, *rot = in.rotation + 4 * (size_t)i;
  auto put = [&](size_t o, const float *p3, const float *s3, const float *q4, float op) {
    for (int k = 0; k < 3; ++k) out.xyz[3 * o + k] = p3[k];
    copy_row(fdc, out.features_dc + 3 * o, 3);
    if (frest && out.features_rest) copy_row(frest, out.features_rest + (size_t)R * o, R);
    for (int k = 0; k < 3; ++k) out.scaling[3 * o + k] = s3[k];
    for (int k = 0; k < 4; ++k) out.rotation[4 * o + k] = q4[k];
    out.opacity[o] = op;
  };
  if (c.keep) {
    const size_t o = part[3 * blockIdx.x] + lk;
    put(o, xyz, scl, rot, in.opacity[i]);
    write_moments(a, i, o, true);
  }
  if (c.split) {
    // normalize(q) (F.normalize, eps 1e-12) and R(q)[:, 0] (math_utils.py:20-24)
    const float nq = fmaxf(sqrtf(((rot[0] * rot[0] + rot[1] * rot[1]) + rot[2] * rot[2]) + rot[3] * rot[3]), 1e-12f);
    const float q[4] = {rot[0] / nq, rot[1] / nq, rot[2] / nq, rot[3] / nq};
    const float w = q[0], x = q[1], y = q[2], z = q[3];
    const float dir[3] = {1.f - 2.f * (y * y + z * z), 2.f * (x * y + w * z), 2.f * (x * z - w * y)};
    const float h = c.smean * 0.5f;  // (:145)
    float s3[3];
    for (int k = 0; k < 3; ++k) s3[k] = logf(expf(scl[k]) * 0.75f);  // log(scale * 0.75) (:149)
    float pm[3], pp[3];
    for (int k = 0; k < 3; ++k) {
      const float off = dir[k] * h;
      pm[k] = xyz[k] - off;
      pp[k] = xyz[k] + off;
    }
    const size_t om = nk + part[3 * blockIdx.x + 1] + ls, op_ = om + ns;
    put(om, pm, s3, q, c.child_op);
    put(op_, pp, s3, q, c.child_op);
    write_moments(a, i, om, false);
    write_moments(a, i, op_, false);
  }
  if (c.clone) {
    const float h = c.smean * 0.5f;  // (:169)
    float p3[3];
    for (int k = 0; k < 3; ++k) p3[k] = xyz[k] + normal_of(a.seed, (uint32_t)i, (uint32_t)k) * h;
    const size_t o = nk + 2u * ns + part[3 * blockIdx.x + 2] + lc;
    put(o, p3, scl, rot, in.opacity[i]);
    write_moments(a, i, o, false);
  }
}

inline unsigned nblocks(int n) { return (unsigned)((n + kB - 1) / kB); }

gs_status check_args(const gs_densify_args *a, const char *what) {
  if (!a) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null args", what);
  if (a->n < 0 || a->rest_floats < 0) return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: bad size", what);
  if (a->n > 0 && (!a->in.xyz || !a->in.features_dc || !a->in.scaling || !a->in.rotation || !a->in.opacity ||
                   (a->rest_floats > 0 && !a->in.features_rest) || !a->counters || !a->workspace ||
                   a->workspace_bytes < gs_densify_workspace_bytes(a->n)))
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null buffer or small workspace", what);
  return GS_OK;
}

}  // namespace

extern "C" size_t gs_densify_workspace_bytes(int32_t n) {
  return n > 0 ? sizeof(uint32_t) * 3 * (size_t)nblocks(n) : 0;
}

extern "C" gs_status gs_densify_count(const gs_densify_args *a, gs_stream_t stream) {
  const gs_status st = check_args(a, "gs_densify_count");
  if (st != GS_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  if (a->n == 0) {
    if (a->counters && hipMemsetAsync(a->counters, 0, 4 * sizeof(uint32_t), s) != hipSuccess)
      return gs_internal_fail(GS_ERR_LAUNCH, "%s: memset failed", "gs_densify_count");
    return GS_OK;
  }
  uint32_t *part = (uint32_t *)a->workspace;
  k_densify_count<<<nblocks(a->n), kB, 0, s>>>(*a, part);
  k_densify_scan<<<1, kB, 0, s>>>(part, (int)nblocks(a->n), a->counters);
  return gs_internal_check_launch("gs_densify_count");
}

extern "C" gs_status gs_densify_emit(const gs_densify_args *a, gs_stream_t stream) {
  const gs_status st = check_args(a, "gs_densify_emit");
  if (st != GS_OK) return st;
  if (a->n == 0) return GS_OK;
  if (!a->out.xyz || !a->out.features_dc || !a->out.scaling || !a->out.rotation || !a->out.opacity)
    return gs_internal_fail(GS_ERR_INVALID_ARG, "%s: null output", "gs_densify_emit");
  hipStream_t s = (hipStream_t)stream;
  k_densify_emit<<<nblocks(a->n), kB, 0, s>>>(*a, (const uint32_t *)a->workspace);
  return gs_internal_check_launch("gs_densify_emit");
}
