// VALU issue-rate probe (gfx950): cycles per wave-instruction per SIMD for the instruction forms the pool
// kernels could use (fp32 scalar, packed fp16, packed fp32, transcendentals, dot2).  Each wave runs 8
// independent chains of one instruction; 2 waves per SIMD (512-thread workgroups, one per CU).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CH8(INS)                                                                                \
  asm volatile(INS : "+v"(a0) : "v"(b), "v"(c));                                                \
  asm volatile(INS : "+v"(a1) : "v"(b), "v"(c));                                                \
  asm volatile(INS : "+v"(a2) : "v"(b), "v"(c));                                                \
  asm volatile(INS : "+v"(a3) : "v"(b), "v"(c));                                                \
  asm volatile(INS : "+v"(a4) : "v"(b), "v"(c));                                                \
  asm volatile(INS : "+v"(a5) : "v"(b), "v"(c));                                                \
  asm volatile(INS : "+v"(a6) : "v"(b), "v"(c));                                                \
  asm volatile(INS : "+v"(a7) : "v"(b), "v"(c));

#define KERN(NAME, T, INS)                                                                       \
  __global__ void __launch_bounds__(512) NAME(T* out, int iters) {                               \
    T a0 = (T)threadIdx.x, a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0;        \
    T b = (T)1, c = (T)0;                                                                         \
    for (int i = 0; i < iters; ++i) { CH8(INS) CH8(INS) }                                         \
    out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                 \
  }

typedef unsigned int u32;
typedef unsigned long long u64;
KERN(k_fma_f32, float, "v_fma_f32 %0, %0, %1, %2")
KERN(k_mul_f32, float, "v_mul_f32 %0, %0, %1")
KERN(k_pk_fma_f16, u32, "v_pk_fma_f16 %0, %0, %1, %2")
KERN(k_pk_mul_f16, u32, "v_pk_mul_f16 %0, %0, %1")
KERN(k_pk_fma_f32, u64, "v_pk_fma_f32 %0, %0, %1, %2")
KERN(k_exp_f32, float, "v_exp_f32 %0, %0")
KERN(k_rcp_f32, float, "v_rcp_f32 %0, %0")
KERN(k_exp_f16, u32, "v_exp_f16 %0, %0")
KERN(k_rcp_f16, u32, "v_rcp_f16 %0, %0")
KERN(k_dot2_f32_f16, u32, "v_dot2_f32_f16 %0, %1, %2, %0")
KERN(k_cvt_pkrtz, u32, "v_cvt_pkrtz_f16_f32 %0, %0, %1")
KERN(k_cvt_pk_bf16, u32, "v_cvt_pk_bf16_f32 %0, %0, %1")

int main() {
  int dev = 0, ncu = 0, clk = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  void* out;
  hipMalloc(&out, (size_t)ncu * 512 * 8);
  const int iters = 4000;
  struct K { const char* n; void (*f)(void*, int); };
#define RUN(NAME, T)                                                                               \
  {                                                                                                \
    hipEvent_t e0, e1;                                                                             \
    hipEventCreate(&e0); hipEventCreate(&e1);                                                      \
    hipLaunchKernelGGL(NAME, dim3(ncu), dim3(512), 0, 0, (T*)out, 100);                            \
    hipEventRecord(e0);                                                                            \
    hipLaunchKernelGGL(NAME, dim3(ncu), dim3(512), 0, 0, (T*)out, iters);                          \
    hipEventRecord(e1);                                                                            \
    hipEventSynchronize(e1);                                                                       \
    float ms; hipEventElapsedTime(&ms, e0, e1);                                                    \
    /* per SIMD: 2 waves x iters x 16 instructions */                                              \
    const double ins = 2.0 * iters * 16;                                                           \
    printf("%-18s %8.3f ms  %6.2f ns per wave-instr per SIMD  (%5.2f cyc @2.4GHz)\n", #NAME, ms,   \
           ms * 1e6 / ins, ms * 1e6 / ins * 2.4);                                                  \
  }
  RUN(k_fma_f32, float) RUN(k_mul_f32, float) RUN(k_pk_fma_f16, u32) RUN(k_pk_mul_f16, u32)
  RUN(k_pk_fma_f32, u64) RUN(k_exp_f32, float) RUN(k_rcp_f32, float) RUN(k_exp_f16, u32)
  RUN(k_rcp_f16, u32) RUN(k_dot2_f32_f16, u32) RUN(k_cvt_pkrtz, u32) RUN(k_cvt_pk_bf16, u32)
  return 0;
}
