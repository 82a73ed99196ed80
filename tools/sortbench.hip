// Sort microbenchmark: this library's gs_radix_sort_pairs against rocPRIM's
// radix_sort_pairs (onesweep) on the two sorts of a C3 frame: 1M 32-bit depth
// keys with iota values, and 4.4M 13-bit tile keys with 32-bit values.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/sortbench.hip \
//          -L mini-3d-gaussian-splatting_amd -lgsplat_mi355x -Wl,-rpath,$PWD/mini-3d-gaussian-splatting_amd -o build/sortbench
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "gsplat_mi355x.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static void run(int n, int bits, int iota) {
  std::vector<uint32_t> hk(n), hv(n);
  srand(1);
  for (int i = 0; i < n; ++i) { hk[i] = ((uint32_t)rand() << 16 ^ (uint32_t)rand()) & (bits == 32 ? 0xFFFFFFFFu : ((1u << bits) - 1)); hv[i] = i; }
  uint32_t *k0, *v0, *k1, *v1, *kin, *vin;
  CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&k1, n * 4)); CK(hipMalloc(&v1, n * 4));
  CK(hipMalloc(&kin, n * 4)); CK(hipMalloc(&vin, n * 4));
  CK(hipMemcpy(kin, hk.data(), n * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(vin, hv.data(), n * 4, hipMemcpyHostToDevice));
  size_t ws_gs = gs_radix_sort_workspace_bytes(n), ws_rp = 0;
  CK(rocprim::radix_sort_pairs(nullptr, ws_rp, kin, k1, vin, v1, n, 0, bits));
  void *ws; CK(hipMalloc(&ws, ws_gs > ws_rp ? ws_gs : ws_rp));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int iters = 20;
  float t_gs = 0, t_rp = 0;
  for (int it = 0; it < iters + 2; ++it) {
    CK(hipMemcpy(k0, kin, n * 4, hipMemcpyDeviceToDevice)); CK(hipMemcpy(v0, vin, n * 4, hipMemcpyDeviceToDevice));
    int32_t alt = 0; float ms;
    CK(hipEventRecord(a, 0));
    if (gs_radix_sort_pairs(k0, v0, k1, v1, n, 0, bits, iota, ws, ws_gs, &alt, 0) != GS_OK) { printf("gs sort failed\n"); exit(1); }
    CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    if (it >= 2) t_gs += ms;
    CK(hipEventRecord(a, 0));
    CK(rocprim::radix_sort_pairs(ws, ws_rp, kin, k1, vin, v1, n, 0, bits));
    CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    if (it >= 2) t_rp += ms;
  }
  printf("n=%d bits=%d: gs_radix_sort_pairs %.1f us, rocprim::radix_sort_pairs %.1f us\n", n, bits,
         1000.f * t_gs / iters, 1000.f * t_rp / iters);
  hipFree(k0); hipFree(v0); hipFree(k1); hipFree(v1); hipFree(kin); hipFree(vin); hipFree(ws);
}

// gs_depth_sort_msd (one 8-bit MSD pass + per-bucket LDS sorts) on n keys of
// `bits` bits below 255 << (bits - 8) (the top bucket is the sentinel's),
// against gs_radix_sort_pairs on the same keys: the estimate for an MSD tile
// sort (round-3 review item 6; 13-bit tile keys, buckets of n / 255 <= 16K)
static void run_msd(int n, int bits) {
  std::vector<uint32_t> hk(n), hv(n);
  srand(2);
  const uint32_t lim = 255u << (bits - 8);
  for (int i = 0; i < n; ++i) { hk[i] = ((uint32_t)rand() << 16 ^ (uint32_t)rand()) % lim; hv[i] = i; }
  uint32_t *k0, *v0, *k1, *v1, *kin, *ovf;
  CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&k1, n * 4)); CK(hipMalloc(&v1, n * 4));
  CK(hipMalloc(&kin, n * 4)); CK(hipMalloc(&ovf, 4));
  CK(hipMemcpy(kin, hk.data(), n * 4, hipMemcpyHostToDevice));
  size_t ws_gs = gs_radix_sort_workspace_bytes(n);
  void *ws; CK(hipMalloc(&ws, ws_gs));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int iters = 20;
  float t_msd = 0, t_lsd = 0;
  uint32_t ov = 0;
  for (int it = 0; it < iters + 2; ++it) {
    CK(hipMemcpy(k0, kin, n * 4, hipMemcpyDeviceToDevice)); CK(hipMemset(ovf, 0, 4));
    int32_t alt = 0; float ms;
    CK(hipEventRecord(a, 0));
    if (gs_depth_sort_msd(k0, v0, k1, v1, n, bits, ws, ws_gs, ovf, &alt, 0) != GS_OK) { printf("msd failed\n"); exit(1); }
    CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    if (it >= 2) t_msd += ms;
    CK(hipMemcpy(&ov, ovf, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(k0, kin, n * 4, hipMemcpyDeviceToDevice));
    CK(hipEventRecord(a, 0));
    if (gs_radix_sort_pairs(k0, v0, k1, v1, n, 0, bits, 1, ws, ws_gs, &alt, 0) != GS_OK) { printf("lsd failed\n"); exit(1); }
    CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
    if (it >= 2) t_lsd += ms;
  }
  printf("n=%d bits=%d (buckets ~%d keys, overflow %s): gs_depth_sort_msd %.1f us, gs_radix_sort_pairs %.1f us\n", n,
         bits, n / 255, ov ? "YES" : "no", 1000.f * t_msd / iters, 1000.f * t_lsd / iters);
  hipFree(k0); hipFree(v0); hipFree(k1); hipFree(v1); hipFree(kin); hipFree(ovf); hipFree(ws);
}

int main() {
  run(1000000, 32, 1);
  run(1000000, 24, 1);  // the depth sort over its key window (C3: 24 bits)
  run(4400000, 13, 0);
  run_msd(1000000, 13);
  run_msd(2000000, 13);
  run_msd(3800000, 13);  // ~14.9K keys per bucket: the C3 tile sort's size at 16K LDS capacity
  return 0;
}
