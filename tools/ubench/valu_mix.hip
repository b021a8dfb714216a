// Cost of VALU fillers BESIDE MFMAs (gfx950): each wave runs a loop of one v_mfma_f32_32x32x16_bf16
// (two alternating accumulators) followed by a block of independent VALU fillers, two waves per SIMD.
// Fillers: 16 x v_fma_f32, 8 x v_pk_fma_f32 (same element work), 8 x v_pk_fma_f16 (same element count),
// 4 x v_exp_f32, and none (MFMA only).  Prints ns per loop iteration per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/valu_mix.hip -o tools/ubench/valu_mix
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned long long u64;
typedef unsigned int u32;

#define MF(ACC) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(ACC) : "v"(fa), "v"(fb));
#define F1(INS, X) asm volatile(INS : "+v"(X) : "v"(b), "v"(c));
#define F8(INS, T)                                                                                  \
  F1(INS, a0) F1(INS, a1) F1(INS, a2) F1(INS, a3) F1(INS, a4) F1(INS, a5) F1(INS, a6) F1(INS, a7)

template <int MODE>
__global__ void __launch_bounds__(512) mix(float* out, int iters) {
  f32x16 acc0 = {}, acc1 = {};
  bf16x8 fa, fb;
  for (int i = 0; i < 8; ++i) { fa[i] = (__bf16)(0.01f * threadIdx.x); fb[i] = (__bf16)0.5f; }
  if constexpr (MODE == 1 || MODE == 0) {
    float a0 = threadIdx.x, a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0, b = 1.f, c = 0.f;
    for (int i = 0; i < iters; ++i) {
      MF(acc0)
      if (MODE == 1) { F8("v_fma_f32 %0, %0, %1, %2", float) F8("v_fma_f32 %0, %0, %1, %2", float) }
      MF(acc1)
      if (MODE == 1) { F8("v_fma_f32 %0, %0, %1, %2", float) F8("v_fma_f32 %0, %0, %1, %2", float) }
    }
    out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + acc0[0] + acc1[3];
  } else if constexpr (MODE == 2) {
    u64 a0 = threadIdx.x, a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0, b = 1, c = 0;
    for (int i = 0; i < iters; ++i) {
      MF(acc0) F8("v_pk_fma_f32 %0, %0, %1, %2", u64)
      MF(acc1) F8("v_pk_fma_f32 %0, %0, %1, %2", u64)
    }
    out[blockIdx.x * 512 + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7) + acc0[0] + acc1[3];
  } else if constexpr (MODE == 3) {
    u32 a0 = threadIdx.x, a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0, b = 1, c = 0;
    for (int i = 0; i < iters; ++i) {
      MF(acc0) F8("v_pk_fma_f16 %0, %0, %1, %2", u32)
      MF(acc1) F8("v_pk_fma_f16 %0, %0, %1, %2", u32)
    }
    out[blockIdx.x * 512 + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7) + acc0[0] + acc1[3];
  } else {
    float a0 = threadIdx.x, a1 = a0, a2 = a0, a3 = a0, b = 1.f, c = 0.f;
    for (int i = 0; i < iters; ++i) {
      MF(acc0) F1("v_exp_f32 %0, %0", a0) F1("v_exp_f32 %0, %0", a1) F1("v_exp_f32 %0, %0", a2) F1("v_exp_f32 %0, %0", a3)
      MF(acc1) F1("v_exp_f32 %0, %0", a0) F1("v_exp_f32 %0, %0", a1) F1("v_exp_f32 %0, %0", a2) F1("v_exp_f32 %0, %0", a3)
    }
    out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3 + acc0[0] + acc1[3];
  }
}

template <int MODE>
void run(const char* name, float* out, int ncu) {
  const int iters = 2000;
  hipLaunchKernelGGL(mix<MODE>, dim3(ncu), dim3(512), 0, 0, out, 50);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(mix<MODE>, dim3(ncu), dim3(512), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // per SIMD: 2 waves x iters x 2 MFMAs
  printf("%-34s %8.3f ms  %7.2f ns per MFMA-slot per SIMD\n", name, ms, ms * 1e6 / (2.0 * iters * 2));
}

int main() {
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  float* out;
  (void)hipMalloc(&out, (size_t)ncu * 512 * 4);
  run<0>("MFMA only", out, ncu);
  run<1>("MFMA + 16 v_fma_f32", out, ncu);
  run<2>("MFMA + 8 v_pk_fma_f32 (16 FMAs)", out, ncu);
  run<3>("MFMA + 8 v_pk_fma_f16 (16 FMAs)", out, ncu);
  run<4>("MFMA + 4 v_exp_f32", out, ncu);
  return 0;
}
