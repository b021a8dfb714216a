// GELU throughput microbenchmark: each thread evaluates ITER x 16 GELUs on register data (no memory
// traffic in the loop); prints ns per element per CU-equivalent and cycles per wave-element.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include "../../proteinbert_pytorch_replication_amd/ops/csrc/common.h"

constexpr int ITER = 4096;

// table-driven GELU / GELU' (cubic Hermite per interval of [-R, R], coefficients of Phi and GELU'
// interleaved so one v_pk_fma evaluates both polynomials): see csrc/common.h gelu_both_tab
constexpr int TAB_N = 64;
constexpr float TAB_R = 6.0f;
__device__ __forceinline__ void tab_both(float x, const unsigned char* tab, float& g, float& gd) {
  const float xc = __builtin_amdgcn_fmed3f(x, -TAB_R, TAB_R * 0.999999f);
  const float u = fmaf(xc, TAB_N / (2.0f * TAB_R), TAB_N * 0.5f);
  const int i = (int)u;
  const float t = u - (float)i;
  const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(tab + i * 32);
  const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(tab + i * 32 + 16);
  const f32x2 tt = {t, t};
  f32x2 p = __builtin_elementwise_fma(tt, (f32x2){hi[2], hi[3]}, (f32x2){hi[0], hi[1]});
  p = __builtin_elementwise_fma(tt, p, (f32x2){lo[2], lo[3]});
  p = __builtin_elementwise_fma(tt, p, (f32x2){lo[0], lo[1]});
  g = x * p.x;
  gd = p.y;
}

template <int MODE>
__global__ void __launch_bounds__(256) kgelu(float* out, float seed, const float* gtab) {
  __shared__ __attribute__((aligned(16))) unsigned char tab[TAB_N * 32];
  if (MODE >= 5) {
    for (int k = threadIdx.x; k < TAB_N * 8; k += 256) reinterpret_cast<float*>(tab)[k] = gtab[k];
    __syncthreads();
  }
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
    } else if (MODE == 4) {         // GELU and GELU' from the shared core (attention pool forward)
#pragma unroll
      for (int i = 0; i < 16; i += 8) {
        const f32x2 x[4] = {(f32x2){v[i], v[i + 1]}, (f32x2){v[i + 2], v[i + 3]}, (f32x2){v[i + 4], v[i + 5]},
                            (f32x2){v[i + 6], v[i + 7]}};
        f32x2 g[4], gd[4];
        gelu2_both_n<4>(x, g, gd);
        const f32x2 s = (g[0] + g[1]) + (g[2] + g[3]) + (gd[0] + gd[1]) + (gd[2] + gd[3]);
        acc += s.x + s.y;
      }
    } else if (MODE == 5) {         // table-driven GELU and GELU'
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float g, gd;
        tab_both(v[i], tab, g, gd);
        acc += g + gd;
      }
    } else if (MODE == 6) {         // table-driven GELU only (g)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float g, gd;
        tab_both(v[i], tab, g, gd);
        acc += g;
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
void run(const char* name, float* d, int blocks, const float* tab) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kgelu<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1.0f, tab);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kgelu<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1.0f, tab);
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
  // Hermite coefficients of Phi and GELU' on TAB_N intervals of [-R, R], interleaved (Phi_k, G'_k)
  float h_tab[TAB_N * 8];
  const double h = 2.0 * TAB_R / TAB_N;
  auto phi = [](double x) { return 0.3989422804014327 * exp(-0.5 * x * x); };
  auto Phi = [](double x) { return 0.5 * erfc(-x / sqrt(2.0)); };
  for (int k = 0; k < TAB_N; ++k) {
    const double x0 = -TAB_R + k * h, x1 = x0 + h;
    const double f[2][2] = {{Phi(x0), Phi(x1)}, {Phi(x0) + x0 * phi(x0), Phi(x1) + x1 * phi(x1)}};
    const double df[2][2] = {{phi(x0), phi(x1)}, {phi(x0) * (2 - x0 * x0), phi(x1) * (2 - x1 * x1)}};
    for (int q = 0; q < 2; ++q) {
      const double c0 = f[q][0], c1 = h * df[q][0];
      const double c2 = 3 * (f[q][1] - f[q][0]) - 2 * h * df[q][0] - h * df[q][1];
      const double c3 = 2 * (f[q][0] - f[q][1]) + h * df[q][0] + h * df[q][1];
      h_tab[k * 8 + q] = (float)c0;
      h_tab[k * 8 + 2 + q] = (float)c1;
      h_tab[k * 8 + 4 + q] = (float)c2;
      h_tab[k * 8 + 6 + q] = (float)c3;
    }
  }
  float* tab;
  hipMalloc(&tab, sizeof(h_tab));
  hipMemcpy(tab, h_tab, sizeof(h_tab), hipMemcpyHostToDevice);
  run<3>("baseline fma", d, blocks, tab);
  run<0>("scalar gelu_f", d, blocks, tab);
  run<1>("packed gelu2_fast", d, blocks, tab);
  run<2>("packed gelu2_fast_n<4>", d, blocks, tab);
  run<4>("packed gelu2_both_n<4>", d, blocks, tab);
  run<5>("table GELU+GELU'", d, blocks, tab);
  run<6>("table GELU only", d, blocks, tab);
  hipFree(d);
  return 0;
}
