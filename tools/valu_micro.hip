// VALU issue-rate microbenchmark: scalar v_fma_f32 vs packed v_pk_fma_f32 /
// v_pk_mul_f32 / v_pk_add_f32, and v_exp_f32, on gfx950.  Each lane runs 8
// independent chains; the kernel reports cycles per wave-instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_micro.hip -o /tmp/valu_micro
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

__global__ void k_fma(float *out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pkfma(float *out, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = (f2){threadIdx.x * 1e-3f + i, threadIdx.x * 2e-3f + i};
  const f2 av = {a, a * 0.5f}, bv = {b, b * 0.25f};
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(av), "v"(bv));
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pkmul(float *out, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = (f2){threadIdx.x * 1e-3f + i, threadIdx.x * 2e-3f + i};
  const f2 av = {a, a * 0.5f};
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(av));
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul(float *out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_exp(float *out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-6f - i * 1e-3f;
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_cnd(float *out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(a) : "vcc");
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(float *, float, float);
int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  const int waves_per_simd = 8, threads = 256;
  const int blocks = cus * 4 * waves_per_simd / (threads / 64);
  float *out;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  struct { const char *name; kfn f; int instrs; } ks[] = {
      {"v_fma_f32", k_fma, 8}, {"v_pk_fma_f32", k_pkfma, 8}, {"v_mul_f32", k_mul, 8},
      {"v_pk_mul_f32", k_pkmul, 8}, {"v_exp_f32", k_exp, 8}, {"v_cndmask_b32", k_cnd, 8}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("CUs %d, clock %d kHz, %d waves/SIMD\n", cus, clk, waves_per_simd);
  for (auto &k : ks) {
    k.f<<<blocks, threads>>>(out, 0.999f, 0.001f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k.f<<<blocks, threads>>>(out, 0.999f, 0.001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double t = ms / 5 * 1e-3;
    const double wave_instr_per_simd = (double)waves_per_simd * kIters * k.instrs;
    const double cyc = t * clk * 1e3;  // at the reported clock
    printf("%-20s %8.3f ms  %.2f cycles per wave-instruction per SIMD (at %d MHz)\n", k.name, ms / 5,
           cyc / wave_instr_per_simd, clk / 1000);
  }
  return 0;
}
