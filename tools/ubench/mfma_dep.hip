// MFMA dependency probe (gfx950): time per v_mfma_f32_32x32x16_bf16 per SIMD when each wave accumulates
// into NACC accumulators round-robin (NACC = 1: every MFMA depends on the previous one), at 1 or 2 waves
// per SIMD (workgroups of 256 / 512 threads, one per CU).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/mfma_dep.hip -o tools/ubench/mfma_dep && tools/ubench/mfma_dep
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int NACC>
__global__ void __launch_bounds__(512) kdep(float* out, int iters) {
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(float)(threadIdx.x & 7);
    b[i] = (__bf16)(float)(i + 1);
  }
  f32x16 acc[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      acc[k % NACC] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[k % NACC], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NACC; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[j][i];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  float* out;
  hipMalloc(&out, (size_t)ncu * 512 * 4);
  const int iters = 2000;
#define RUN(NACC, THREADS)                                                                         \
  {                                                                                                \
    hipEvent_t e0, e1;                                                                             \
    hipEventCreate(&e0); hipEventCreate(&e1);                                                      \
    hipLaunchKernelGGL(kdep<NACC>, dim3(ncu), dim3(THREADS), 0, 0, out, 50);                       \
    hipEventRecord(e0);                                                                            \
    hipLaunchKernelGGL(kdep<NACC>, dim3(ncu), dim3(THREADS), 0, 0, out, iters);                    \
    hipEventRecord(e1);                                                                            \
    hipEventSynchronize(e1);                                                                       \
    float ms; hipEventElapsedTime(&ms, e0, e1);                                                    \
    const double n = (THREADS / 256.0) * iters * 16;   /* MFMAs per SIMD */                        \
    printf("NACC=%d waves/SIMD=%d: %6.2f ns per MFMA per SIMD (%5.1f cyc @2.4GHz)\n", NACC,        \
           THREADS / 256, ms * 1e6 / n, ms * 1e6 / n * 2.4);                                       \
  }
  RUN(1, 256) RUN(2, 256) RUN(4, 256) RUN(8, 256)
  RUN(1, 512) RUN(2, 512) RUN(4, 512) RUN(8, 512)
  return 0;
}
