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

// Packed (2-wide) versions on v_pk_fma_f32 / v_pk_mul_f32: the polynomial, the squares and the
// final products run two lanes' values per instruction; rcp / exp2 stay scalar (transcendental).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gelu_parts2(f32x2 x, f32x2& cdf, f32x2& pdf) {
  const f32x2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f32x2 den = z * 0.3275911f + 1.0f;
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 pl = __builtin_elementwise_fma(t, (f32x2){1.061405429f, 1.061405429f}, (f32x2){-1.453152027f, -1.453152027f});
  pl = __builtin_elementwise_fma(t, pl, (f32x2){1.421413741f, 1.421413741f});
  pl = __builtin_elementwise_fma(t, pl, (f32x2){-0.284496736f, -0.284496736f});
  pl = __builtin_elementwise_fma(t, pl, (f32x2){0.254829592f, 0.254829592f});
  pl = pl * t;
  const f32x2 q = (z * z) * -1.4426950408889634f;          // -z^2 log2(e)
  const f32x2 e = {__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  const f32x2 erfz = __builtin_elementwise_fma(-pl, e, (f32x2){1.0f, 1.0f});
  const f32x2 se = {copysignf(erfz.x, x.x), copysignf(erfz.y, x.y)};
  cdf = __builtin_elementwise_fma(se, (f32x2){0.5f, 0.5f}, (f32x2){0.5f, 0.5f});
  pdf = e * 0.3989422804014327f;
}
#ifndef PBX_PACKED_GELU
// Beside MFMAs packed f32 VALU is an anti-lever on gfx950 (a v_pk_fma_f32 costs ~22 cycles more per
// MFMA gap than two v_fma_f32, MI355X_MICROARCH.md): the 2-wide entry points run scalar code.
__device__ __forceinline__ f32x2 gelu2(f32x2 x) { return (f32x2){gelu_f(x.x), gelu_f(x.y)}; }
__device__ __forceinline__ f32x2 gelu_grad2(f32x2 x) { return (f32x2){gelu_grad_f(x.x), gelu_grad_f(x.y)}; }
#else
__device__ __forceinline__ f32x2 gelu2(f32x2 x) {
  f32x2 c, p;
  gelu_parts2(x, c, p);
  return x * c;
}
__device__ __forceinline__ f32x2 gelu_grad2(f32x2 x) {
  f32x2 c, p;
  gelu_parts2(x, c, p);
  return __builtin_elementwise_fma(x, p, c);
}
#endif

// Packed GELU / GELU' for VALU-bound epilogues (the attention pool: one GELU per element of a
// [rows, 512] GEMM output, ~13 VALU + 2 transcendentals each, 3-4x the MFMA time of the GEMM).
// A&S 7.1.26 erf, arranged so every non-transcendental step is one v_pk_* instruction for two
// values:  gelu(x) = 0.5 x + |x| * h,  h = 0.5 erf(|x|/sqrt2) = 0.5 - 0.5 t P(t) e  (the -0.5 is
// folded into the polynomial coefficients), e = exp(-x^2 / 2), t = 1 / (1 + p |x| / sqrt2).

// Scalar form of the interleaved cores below: the same A&S stages on 2N independent scalars, one
// v_fma_f32 per value per stage.  Beside in-flight MFMAs a v_pk_*_f32 costs far more than its two
// scalar halves (MI355X_MICROARCH.md constants table), and these cores run in the shadow of the MFMAs
// of the next tile.  (Needs -fno-slp-vectorize, or the SLP vectoriser packs the halves again.)
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

// N independent pairs evaluated stage by stage (every stage of all N before the next): the
// one-pair forms above compile to a serial dependency chain with an s_nop between dependent packed
// ops; N interleaved chains fill those slots and the transcendental latencies.
template <int N, bool GRAD>
__device__ __forceinline__ void gelu2_fast_n(const f32x2* x, f32x2* out) {
#ifdef PBX_ABL_NOGELU   // ablation builds only (tools/ubench/build_flags.sh): the cost of the GELU chains
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = x[i] * 0.5f;
  return;
#endif
#ifndef PBX_GELU_ERF   // default: the fitted logistic core (A/B builds with -DPBX_GELU_ERF keep the erf forms)
  if (GRAD) gelu_logistic_n<N, 1>(x, nullptr, out);
  else gelu_logistic_n<N, 0>(x, out, nullptr);
  return;
#endif
#ifdef PBX_SCALAR_GELU
  if (GRAD) gelu_scalar_n<N, 1>(x, nullptr, out);
  else gelu_scalar_n<N, 0>(x, out, nullptr);
  return;
#endif
  // GRAD: e = phi(x) with the Zelen-Severo coefficients (see gelu2_both_n), GELU' = Phi + x e
  constexpr float q1 = GRAD ? -1.3257480647361592f : 0.0f;
  constexpr float c5 = GRAD ? -1.3302744295891233f : -0.5307027145f;
  constexpr float c4 = GRAD ? 1.8212559791077754f : 0.7265760135f;
  constexpr float c3 = GRAD ? -1.7814779365698128f : -0.7107068705f;
  constexpr float c2 = GRAD ? 0.3565637812489156f : 0.142248368f;
  constexpr float c1 = GRAD ? -0.31938153025994087f : -0.127414796f;
  f32x2 ax[N], t[N], e[N], pl[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    ax[i] = __builtin_elementwise_abs(x[i]);
    t[i] = __builtin_elementwise_fma(ax[i], (f32x2){0.23164190f, 0.23164190f}, (f32x2){1.0f, 1.0f});
    if (GRAD)
      e[i] = __builtin_elementwise_fma(x[i] * x[i], (f32x2){-0.72134752044448170f, -0.72134752044448170f},
                                       (f32x2){q1, q1});
    else
      e[i] = (x[i] * -0.72134752044448170f) * x[i];
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    t[i] = (f32x2){__builtin_amdgcn_rcpf(t[i].x), __builtin_amdgcn_rcpf(t[i].y)};
    e[i] = (f32x2){__builtin_amdgcn_exp2f(e[i].x), __builtin_amdgcn_exp2f(e[i].y)};
  }
#pragma unroll
  for (int i = 0; i < N; ++i) pl[i] = __builtin_elementwise_fma(t[i], (f32x2){c5, c5}, (f32x2){c4, c4});
#pragma unroll
  for (int i = 0; i < N; ++i) pl[i] = __builtin_elementwise_fma(t[i], pl[i], (f32x2){c3, c3});
#pragma unroll
  for (int i = 0; i < N; ++i) pl[i] = __builtin_elementwise_fma(t[i], pl[i], (f32x2){c2, c2});
#pragma unroll
  for (int i = 0; i < N; ++i) pl[i] = __builtin_elementwise_fma(t[i], pl[i], (f32x2){c1, c1});
#pragma unroll
  for (int i = 0; i < N; ++i) pl[i] = __builtin_elementwise_fma(pl[i] * t[i], e[i], (f32x2){0.5f, 0.5f});   // h
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (GRAD) {
      const f32x2 Phi = (f32x2){copysignf(pl[i].x, x[i].x), copysignf(pl[i].y, x[i].y)} + 0.5f;
      out[i] = __builtin_elementwise_fma(x[i], e[i], Phi);
    } else {
      out[i] = __builtin_elementwise_fma(ax[i], pl[i], x[i] * 0.5f);
    }
  }
}

// GELU AND GELU' of N independent pairs from one shared erf / exp evaluation (same stages as
// gelu2_fast_n): a producer that needs the activation now and its derivative later (stored for the
// backward) pays ~5 extra packed ops per pair instead of a second core.
template <int N>
__device__ __forceinline__ void gelu2_both_n(const f32x2* x, f32x2* g, f32x2* gd) {
#ifdef PBX_ABL_NOGELU
#pragma unroll
  for (int i = 0; i < N; ++i) {
    g[i] = x[i] * 0.5f;
    gd[i] = x[i] * 0.25f;
  }
  return;
#endif
#ifndef PBX_GELU_ERF
  gelu_logistic_n<N, 2>(x, g, gd);
  return;
#endif
#ifdef PBX_SCALAR_GELU
  gelu_scalar_n<N, 2>(x, g, gd);
  return;
#endif
  // e = phi(x) (the 1/sqrt(2 pi) folded into the exponent and the polynomial: Zelen-Severo form of
  // the same A&S 7.1.26 erf), Phi = 0.5 + sign(x) h, GELU = x Phi, GELU' = Phi + x phi: 13 VALU + 2 T
  f32x2 t[N], e[N], pl[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    t[i] = __builtin_elementwise_fma(__builtin_elementwise_abs(x[i]), (f32x2){0.23164190f, 0.23164190f},
                                     (f32x2){1.0f, 1.0f});
    e[i] = __builtin_elementwise_fma(x[i] * x[i], (f32x2){-0.72134752044448170f, -0.72134752044448170f},
                                     (f32x2){-1.3257480647361592f, -1.3257480647361592f});
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    t[i] = (f32x2){__builtin_amdgcn_rcpf(t[i].x), __builtin_amdgcn_rcpf(t[i].y)};
    e[i] = (f32x2){__builtin_amdgcn_exp2f(e[i].x), __builtin_amdgcn_exp2f(e[i].y)};
  }
#pragma unroll
  for (int i = 0; i < N; ++i)
    pl[i] = __builtin_elementwise_fma(t[i], (f32x2){-1.3302744295891233f, -1.3302744295891233f},
                                      (f32x2){1.8212559791077754f, 1.8212559791077754f});
#pragma unroll
  for (int i = 0; i < N; ++i)
    pl[i] = __builtin_elementwise_fma(t[i], pl[i], (f32x2){-1.7814779365698128f, -1.7814779365698128f});
#pragma unroll
  for (int i = 0; i < N; ++i)
    pl[i] = __builtin_elementwise_fma(t[i], pl[i], (f32x2){0.3565637812489156f, 0.3565637812489156f});
#pragma unroll
  for (int i = 0; i < N; ++i)
    pl[i] = __builtin_elementwise_fma(t[i], pl[i], (f32x2){-0.31938153025994087f, -0.31938153025994087f});
#pragma unroll
  for (int i = 0; i < N; ++i) pl[i] = __builtin_elementwise_fma(pl[i] * t[i], e[i], (f32x2){0.5f, 0.5f});   // h
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const f32x2 Phi = (f32x2){copysignf(pl[i].x, x[i].x), copysignf(pl[i].y, x[i].y)} + 0.5f;
    g[i] = x[i] * Phi;
    gd[i] = __builtin_elementwise_fma(x[i], e[i], Phi);
  }
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
