// Per-instruction issue cost in shader cycles (s_memtime inside the kernel),
// at 1/2/4/8 waves per SIMD: v_fma_f32, v_pk_fma_f32, v_exp_f32,
// v_cndmask_b32, v_cmp_lt_f32, ds_read_b64 (broadcast) -- one instruction
// kind per kernel, 8 independent chains per lane, 256 instructions per
// timed loop iteration.
//   hipcc --offload-arch=gfx950 -O3 -w tools/valu_cycles.hip -o tools/valu_cycles.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 256;

#define BODY8(ASM, T)                                                                  \
  _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(ASM : "+v"(x[i]) : "v"(a), "v"(b));

template <int KIND>
__global__ void kern(float *out, long long *cyc, float a0, float b0) {
  float x[8];
  f2 xp[8];
  for (int i = 0; i < 8; ++i) {
    x[i] = threadIdx.x * 1e-3f + i;
    xp[i] = (f2){x[i], x[i] + 1.f};
  }
  float a = a0, b = b0;
  f2 ap = {a0, a0}, bp = {b0, b0};
  unsigned long long msk = 0x5555555555555555ull ^ (unsigned long long)blockIdx.x, mk[8];
  __shared__ float2 lds[64];
  if (threadIdx.x < 64) lds[threadIdx.x] = make_float2(threadIdx.x, 1.f);
  __syncthreads();
  const long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (KIND == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
      } else if (KIND == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(xp[i]) : "v"(ap), "v"(bp));
      } else if (KIND == 2) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
      } else if (KIND == 3) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "s"(msk));
      } else if (KIND == 4) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_cmp_lt_f32 %0, %1, %2" : "=s"(mk[i]) : "v"(x[i]), "v"(a));
      } else if (KIND == 5) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
      } else if (KIND == 6) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_max_f32 %0, %0, %0 clamp" : "+v"(x[i]));
      } else if (KIND == 7) {
        float2 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          typedef __attribute__((address_space(3))) const volatile unsigned long long u64l;
          unsigned long long q = *(u64l *)&lds[(it + i) & 63];
          v[i] = make_float2(__uint_as_float((uint32_t)q), __uint_as_float((uint32_t)(q >> 32)));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] += v[i].x;
      }
    }
  }
  const long long t1 = __builtin_readcyclecounter();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i] + xp[i].x + xp[i].y;
  if (KIND == 4)
    for (int i = 0; i < 8; ++i) s += (float)(mk[i] & 1);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

typedef void (*kfn)(float *, long long *, float, float);
int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const char *names[] = {"v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "v_cndmask_b32", "v_cmp_lt_f32(sgpr)",
                         "v_mul_f32", "v_max_f32 clamp", "ds_read_b64+v_add"};
  kfn fs[] = {kern<0>, kern<1>, kern<2>, kern<3>, kern<4>, kern<5>, kern<6>, kern<7>};
  float *out;
  long long *cyc;
  hipMalloc(&out, sizeof(float) * cus * 4 * 8 * 64);
  hipMalloc(&cyc, sizeof(long long) * cus * 4 * 8);
  long long *h = (long long *)malloc(sizeof(long long) * cus * 4 * 8);
  printf("cycles per wave-instruction per SIMD (s_memtime), 8 chains x 4 x %d per wave\n", kIters);
  for (int k = 0; k < 8; ++k) {
    printf("%-22s", names[k]);
    for (int wps : {1, 2, 4, 8}) {
      const int threads = 64 * wps, blocks = cus * 4;  // one block per SIMD (4 per CU)
      fs[k]<<<blocks, threads>>>(out, cyc, 0.999f, 0.001f);
      hipDeviceSynchronize();
      fs[k]<<<blocks, threads>>>(out, cyc, 0.999f, 0.001f);
      hipMemcpy(h, cyc, sizeof(long long) * blocks * wps, hipMemcpyDeviceToHost);
      double mx = 0;
      for (int i = 0; i < blocks * wps; ++i) mx = h[i] > mx ? h[i] : mx;
      const double instr_per_wave = 8.0 * 4 * kIters;
      printf("  %dw: %6.2f", wps, mx / (instr_per_wave * wps));
    }
    printf("\n");
  }
  return 0;
}
