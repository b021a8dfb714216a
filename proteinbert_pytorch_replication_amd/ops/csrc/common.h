// Shared helpers for the pbx CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PBX_EXPORT extern "C" __attribute__((visibility("default")))

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // 8 bf16 = one MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) short bf16x4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

// bf16 <-> f32.  f32 -> bf16 is the language cast, which hipcc lowers to the gfx950 hardware
// convert v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN kept NaN, two values per instruction when
// adjacent conversions pair up) instead of ~6 integer VALU ops + a NaN select per value.
__device__ __forceinline__ float bf2f(unsigned short h) {
  return __uint_as_float(((unsigned int)h) << 16);
}
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}

// GELU (nn.GELU default, erf form) and its derivative, branch-free: erf via Abramowitz-Stegun
// 7.1.26 (|err| <= 1.5e-7) sharing exp(-x^2/2) with the Gaussian pdf.  The libm erff inlines a
// piecewise polynomial with divergent branches, which dominated the epilogues of the fused kernels.
__device__ __forceinline__ void gelu_parts(float x, float& cdf, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float e = __expf(-z * z);
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  const float erfz = fmaf(-poly, e, 1.0f);
  cdf = fmaf(0.5f, copysignf(erfz, x), 0.5f);
  pdf = 0.3989422804014327f * e;
}
__device__ __forceinline__ float gelu_f(float x) {
  float c, p;
  gelu_parts(x, c, p);
  return x * c;
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  float c, p;
  gelu_parts(x, c, p);
  return fmaf(x, p, c);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// The fused kernels' GELU cores come in two builds of the same sources (ops/build.py):
//   libpbx_hip.so        the fitted logistic core below (max |err| 2.9e-4 in GELU, 7.8e-4 in GELU', below the
//                        bf16 rounding of every stored value; 7 / 11 VALU per GELU / GELU + GELU')
//   libpbx_hip_exact.so  -DPBX_GELU_EXACT: the A&S 7.1.26 erf core (|err| <= 1.5e-7, the reference's exact
//                        nn.GELU() up to fp32 rounding; 14 / 15 VALU), selected at run time by PBX_GELU=exact
//                        or the `kernel.gelu=exact` config key
#ifndef PBX_GELU_EXACT
#define PBX_GELU_EXACT 0
#endif

// A&S 7.1.26 erf core on 2N independent scalars, stage by stage (every stage of all values before the
// next, so the transcendental latencies and dependent-op slots are filled).  Scalar on purpose: beside
// in-flight MFMAs a v_pk_*_f32 costs far more than its two scalar halves (MI355X_MICROARCH.md constants
// table), and the build passes -fno-slp-vectorize so the halves stay scalar.
template <int N, int MODE>   // MODE 0: GELU, 1: GELU', 2: both (g and gd)
__device__ __forceinline__ void gelu_scalar_n(const f32x2* x, f32x2* g, f32x2* gd) {
  constexpr int M = 2 * N;
  float xs[M], t[M], e[M], pl[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    xs[i] = (i & 1) ? x[i >> 1].y : x[i >> 1].x;
    t[i] = fmaf(fabsf(xs[i]), 0.23164190f, 1.0f);
    // MODE 0: e = exp(-x^2/2); MODE 1/2: e = phi(x) = exp(-x^2/2) / sqrt(2 pi) (Zelen-Severo form:
    // Phi(|x|) = 1 - phi(x) t B(t), the same A&S 7.1.26 polynomial rescaled), so GELU' = Phi + x e is one fma
    e[i] = MODE == 0 ? (xs[i] * -0.72134752044448170f) * xs[i]
                     : fmaf(xs[i] * xs[i], -0.72134752044448170f, -1.3257480647361592f);
  }
#pragma unroll
  for (int i = 0; i < M; ++i) {
    t[i] = __builtin_amdgcn_rcpf(t[i]);
    e[i] = __builtin_amdgcn_exp2f(e[i]);
  }
  constexpr float c5 = MODE == 0 ? -0.5307027145f : -1.3302744295891233f;
  constexpr float c4 = MODE == 0 ? 0.7265760135f : 1.8212559791077754f;
  constexpr float c3 = MODE == 0 ? -0.7107068705f : -1.7814779365698128f;
  constexpr float c2 = MODE == 0 ? 0.142248368f : 0.3565637812489156f;
  constexpr float c1 = MODE == 0 ? -0.127414796f : -0.31938153025994087f;
#pragma unroll
  for (int i = 0; i < M; ++i) pl[i] = fmaf(t[i], c5, c4);
#pragma unroll
  for (int i = 0; i < M; ++i) pl[i] = fmaf(t[i], pl[i], c3);
#pragma unroll
  for (int i = 0; i < M; ++i) pl[i] = fmaf(t[i], pl[i], c2);
#pragma unroll
  for (int i = 0; i < M; ++i) pl[i] = fmaf(t[i], pl[i], c1);
#pragma unroll
  for (int i = 0; i < M; ++i) pl[i] = fmaf(pl[i] * t[i], e[i], 0.5f);   // h = 0.5 erf(|x| / sqrt 2)
#pragma unroll
  for (int i = 0; i < M; ++i) {
    float gv = 0.f, dv = 0.f;
    if (MODE == 0) {
      gv = fmaf(fabsf(xs[i]), pl[i], xs[i] * 0.5f);
    } else {
      const float Phi = copysignf(pl[i], xs[i]) + 0.5f;
      if (MODE == 2) gv = xs[i] * Phi;
      dv = fmaf(xs[i], e[i], Phi);
    }
    if (i & 1) {
      if (MODE != 1) g[i >> 1].y = gv;
      if (MODE != 0) gd[i >> 1].y = dv;
    } else {
      if (MODE != 1) g[i >> 1].x = gv;
      if (MODE != 0) gd[i >> 1].x = dv;
    }
  }
}

// Fitted logistic GELU core: GELU(x) ~ x s, s = sigma(x k(t)), k(t) = 1.59934 + 0.0696829 t, t = x^2 (minimax
// fit to the erf GELU on [-14, 14]: max |err| 2.9e-4 in GELU, 7.8e-4 in GELU' = s + x s (1 - s) (k + 2 t k1),
// both below the bf16 rounding of the stored values), evaluated as s = 1 / (1 + exp2(-log2(e) x k(t))):
// 7 VALU per GELU, 11 for GELU and GELU' together (the A&S erf form above: 14 / 15).  Saturates cleanly:
// x -> -inf gives s = 0 (exp2 -> inf), x -> +inf gives s = 1.
template <int N, int MODE>   // MODE 0: GELU, 1: GELU', 2: both (g and gd)
__device__ __forceinline__ void gelu_logistic_n(const f32x2* x, f32x2* g, f32x2* gd) {
  constexpr int M = 2 * N;
  float xs[M], t[M], s[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    xs[i] = (i & 1) ? x[i >> 1].y : x[i >> 1].x;
    t[i] = xs[i] * xs[i];
    s[i] = fmaf(t[i], -0.10053117f, -2.3073633f) * xs[i];      // -log2(e) x k(t)
  }
#pragma unroll
  for (int i = 0; i < M; ++i) s[i] = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(s[i]) + 1.0f);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    float gv = 0.f, dv = 0.f;
    if (MODE != 1) gv = xs[i] * s[i];
    if (MODE != 0) {
      const float kd = fmaf(t[i], 0.20904868f, 1.59934236f);   // k + 2 t k1
      dv = fmaf(xs[i] * fmaf(-s[i], s[i], s[i]), kd, s[i]);
    }
    if (i & 1) {
      if (MODE != 1) g[i >> 1].y = gv;
      if (MODE != 0) gd[i >> 1].y = dv;
    } else {
      if (MODE != 1) g[i >> 1].x = gv;
      if (MODE != 0) gd[i >> 1].x = dv;
    }
  }
}

// The build's GELU core on N independent pairs (MODE 0: GELU, 1: GELU', 2: both)
template <int N, int MODE>
__device__ __forceinline__ void gelu_n(const f32x2* x, f32x2* g, f32x2* gd) {
  if constexpr (PBX_GELU_EXACT) gelu_scalar_n<N, MODE>(x, g, gd);
  else gelu_logistic_n<N, MODE>(x, g, gd);
}
template <int N, bool GRAD>
__device__ __forceinline__ void gelu2_fast_n(const f32x2* x, f32x2* out) {
  if (GRAD) gelu_n<N, 1>(x, nullptr, out);
  else gelu_n<N, 0>(x, out, nullptr);
}
template <int N>
__device__ __forceinline__ void gelu2_both_n(const f32x2* x, f32x2* g, f32x2* gd) {
  gelu_n<N, 2>(x, g, gd);
}

__device__ __forceinline__ float wave_reduce_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_reduce_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// counter-based RNG (splitmix64 finaliser of (seed, stream, index)); uniform in [0, 1)
__device__ __forceinline__ unsigned long long pbx_mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float pbx_uniform(unsigned long long seed, unsigned long long stream,
                                             unsigned long long idx) {
  unsigned long long h = pbx_mix64(seed ^ pbx_mix64(stream * 0xD1B54A32D192ED03ull + idx));
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}

static inline int pbx_launch_status() { return (int)hipGetLastError(); }
