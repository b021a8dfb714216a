// GELU throughput microbenchmark: each thread evaluates ITER x 16 GELUs on register data (no memory
// traffic in the loop); prints ns per element per CU-equivalent and cycles per wave-element.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../proteinbert_pytorch_replication_amd/ops/csrc/common.h"

constexpr int ITER = 4096;

template <int MODE>
__global__ void __launch_bounds__(256) kgelu(float* out, float seed) {
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = seed * (threadIdx.x + i) * 1e-3f - 2.0f;
  float acc = 0.f;
  for (int it = 0; it < ITER; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc += gelu_f(v[i]);
    } else if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2 g = gelu2_fast((f32x2){v[i], v[i + 1]});
        acc += g.x + g.y;
      }
    } else if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < 16; i += 8) {
        const f32x2 x[4] = {(f32x2){v[i], v[i + 1]}, (f32x2){v[i + 2], v[i + 3]}, (f32x2){v[i + 4], v[i + 5]},
                            (f32x2){v[i + 6], v[i + 7]}};
        f32x2 g[4];
        gelu2_fast_n<4, false>(x, g);
        const f32x2 s = (g[0] + g[1]) + (g[2] + g[3]);
        acc += s.x + s.y;
      }
    } else if (MODE == 3) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc += v[i] * v[i] + 1.0f;   // baseline: 2 VALU per element
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] += 1e-7f;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE>
void run(const char* name, float* d, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kgelu<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kgelu<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double elems = 5.0 * blocks * 256.0 * ITER * 16.0;
  // per SIMD (1024 SIMDs), per wave64 element-vector: cycles at an assumed 2.4 GHz
  const double cyc = ms * 1e-3 * 2.4e9 * 1024.0 / (elems / 64.0);
  printf("%-28s %8.3f ms  %7.2f Gelem/s  %6.2f cyc per wave-element per SIMD (2.4 GHz)\n", name, ms / 5,
         elems / (ms * 1e-3) / 1e9, cyc);
}

int main() {
  float* d;
  const int blocks = 256 * 8;   // 8 waves per CU... x4 -> 2048 blocks of 4 waves = 8 waves/CU
  hipMalloc(&d, blocks * 256 * sizeof(float));
  run<3>("baseline fma", d, blocks);
  run<0>("scalar gelu_f", d, blocks);
  run<1>("packed gelu2_fast", d, blocks);
  run<2>("packed gelu2_fast_n<4>", d, blocks);
  hipFree(d);
  return 0;
}
