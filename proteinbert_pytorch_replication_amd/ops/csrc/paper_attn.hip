// Paper-semantics global attention core (local -> global, one query per head, softmax over the
// sequence axis, pad-masked): the published ProteinBERT attention that the reference's
// GlobalAttentionHead (modules.py:49-60) was meant to compute.  The reference's own softmax runs
// over the key axis and collapses to a mean pool (reference semantics live in ln.hip's pool).
//
// (Split form, PBX_PAPER_ATTN=split: the K/V projections [B*L, C] x [C, H*(K+VD)] are one in-tree MFMA
// GEMM, csrc/gemm.hip, producing the bf16 pre-activations `pre`; the default fused form computes them
// inside csrc/paper_fused.hip.)  Everything after the projection is here:
//
//   forward   split-L flash-decoding: per (b, h, L-chunk) one workgroup of 4 waves; each wave owns
//             one position per step (lane k <-> key channel k, lane j <-> value channels 2j, 2j+1),
//             s_l = sum_k q_k tanh(pre_k) (q pre-scaled by 1/sqrt(K)), online softmax with running
//             (m, l, acc[VD]) in registers, 4 positions in flight per wave for ILP.  Partials of the
//             4 waves merge through LDS; a combine kernel merges the chunks and writes o and lse.
//   backward  one pass over the same grid: recompute s_l, p_l = exp(s_l - lse);
//             dpre_v = p dO * gelu'(pre_v), ds = p (dO.v - dO.o), dpre_k = ds q (1 - tanh^2),
//             dq partial = sum_l ds tanh(pre_k) per chunk (fixed-order, deterministic, summed by
//             the caller).  Masked positions get p = 0 and write zero gradients.
//
// Layout of a `pre` row (N = H*(K+VD) bf16): [H*K keys | H*VD values], head-major in each half.
#include "common.h"

namespace {

constexpr int PA_K = 64;      // key dim == wavefront size
constexpr int PA_VD = 128;    // value dim per head (2 per lane)
constexpr int PA_WAVES = 4;
constexpr int PA_UNROLL = 4;

__device__ __forceinline__ float tanh_f(float x) {
  // tanh(x) = 1 - 2 / (exp(2x) + 1), saturating correctly at +-inf
  const float e = __expf(2.0f * x);
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}

struct PaOnline {
  float m, l, a0, a1;
};

__global__ __launch_bounds__(256) void paper_attn_fwd_kernel(
    const unsigned short* __restrict__ pre, const float* __restrict__ qs, const unsigned char* __restrict__ mask,
    float* __restrict__ part, int L, int H, int chunk, int nsplit) {
  const int split = blockIdx.x, bh = blockIdx.y;
  const int b = bh / H, h = bh - b * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int N = H * (PA_K + PA_VD);
  const int l0 = split * chunk, l1 = min(L, l0 + chunk);
  const float q = qs[(size_t)bh * PA_K + lane];
  const unsigned short* rowk = pre + (size_t)b * L * N + h * PA_K + lane;
  const unsigned short* rowv = pre + (size_t)b * L * N + H * PA_K + h * PA_VD + 2 * lane;
  const unsigned char* mrow = mask ? mask + (size_t)b * L : nullptr;

  PaOnline st = {-INFINITY, 0.f, 0.f, 0.f};
  for (int base = l0 + wave; base < l1; base += PA_WAVES * PA_UNROLL) {
    float s[PA_UNROLL], v0[PA_UNROLL], v1[PA_UNROLL];
    bool ok[PA_UNROLL];
#pragma unroll
    for (int u = 0; u < PA_UNROLL; ++u) {
      const int l = base + u * PA_WAVES;
      const int lc = min(l, l1 - 1);                       // clamped, unconditional loads
      ok[u] = (l < l1) && (!mrow || mrow[lc]);
      const float kp = bf2f(rowk[(size_t)lc * N]);
      const unsigned int vv = *reinterpret_cast<const unsigned int*>(rowv + (size_t)lc * N);
      s[u] = q * tanh_f(kp);
      v0[u] = bf2f((unsigned short)(vv & 0xffff));
      v1[u] = bf2f((unsigned short)(vv >> 16));
    }
#pragma unroll
    for (int u = 0; u < PA_UNROLL; ++u) s[u] = wave_reduce_sum(s[u]);
#pragma unroll
    for (int u = 0; u < PA_UNROLL; ++u) {
      if (!ok[u]) continue;                                 // wave-uniform
      const float g0 = gelu_f(v0[u]), g1 = gelu_f(v1[u]);
      const float mn = fmaxf(st.m, s[u]);
      const float c = __expf(st.m - mn), p = __expf(s[u] - mn);
      st.l = fmaf(st.l, c, p);
      st.a0 = fmaf(st.a0, c, p * g0);
      st.a1 = fmaf(st.a1, c, p * g1);
      st.m = mn;
    }
  }
  // merge the 4 waves through LDS
  __shared__ float sm[PA_WAVES], sl[PA_WAVES], sa[PA_WAVES][PA_VD];
  if (lane == 0) { sm[wave] = st.m; sl[wave] = st.l; }
  sa[wave][2 * lane] = st.a0;
  sa[wave][2 * lane + 1] = st.a1;
  __syncthreads();
  if (wave == 0) {
    float M = sm[0];
#pragma unroll
    for (int w = 1; w < PA_WAVES; ++w) M = fmaxf(M, sm[w]);
    float Ls = 0.f, A0 = 0.f, A1 = 0.f;
#pragma unroll
    for (int w = 0; w < PA_WAVES; ++w) {
      const float c = (sm[w] == -INFINITY) ? 0.f : __expf(sm[w] - M);
      Ls = fmaf(sl[w], c, Ls);
      A0 = fmaf(sa[w][2 * lane], c, A0);
      A1 = fmaf(sa[w][2 * lane + 1], c, A1);
    }
    float* out = part + ((size_t)bh * nsplit + split) * (2 + PA_VD);
    if (lane == 0) { out[0] = M; out[1] = Ls; }
    out[2 + 2 * lane] = A0;
    out[3 + 2 * lane] = A1;
  }
}

// one wave per (b, h): merge the L-chunk partials -> o [B, H*VD] (fp32), lse [B*H]
__global__ __launch_bounds__(64) void paper_attn_combine_kernel(const float* __restrict__ part, float* __restrict__ o,
                                                                float* __restrict__ lse, int nsplit) {
  const int bh = blockIdx.x, lane = threadIdx.x;
  const float* p = part + (size_t)bh * nsplit * (2 + PA_VD);
  float M = -INFINITY;
  for (int i = 0; i < nsplit; ++i) M = fmaxf(M, p[i * (2 + PA_VD)]);
  float Ls = 0.f, A0 = 0.f, A1 = 0.f;
  for (int i = 0; i < nsplit; ++i) {
    const float* q = p + i * (2 + PA_VD);
    const float c = (q[0] == -INFINITY) ? 0.f : __expf(q[0] - M);
    Ls = fmaf(q[1], c, Ls);
    A0 = fmaf(q[2 + 2 * lane], c, A0);
    A1 = fmaf(q[3 + 2 * lane], c, A1);
  }
  // a fully padded row has no key: output 0 (torch's masked softmax would give NaN)
  const float inv = Ls > 0.f ? 1.0f / Ls : 0.f;
  o[(size_t)bh * PA_VD + 2 * lane] = A0 * inv;
  o[(size_t)bh * PA_VD + 2 * lane + 1] = A1 * inv;
  if (lane == 0) lse[bh] = Ls > 0.f ? M + __logf(Ls) : INFINITY;
}

__global__ __launch_bounds__(256) void paper_attn_bwd_kernel(
    const unsigned short* __restrict__ pre, const float* __restrict__ qs, const unsigned char* __restrict__ mask,
    const float* __restrict__ lse, const float* __restrict__ o, const float* __restrict__ dO,
    unsigned short* __restrict__ dpre, float* __restrict__ dq_part, int L, int H, int chunk, int nsplit) {
  const int split = blockIdx.x, bh = blockIdx.y;
  const int b = bh / H, h = bh - b * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int N = H * (PA_K + PA_VD);
  const int l0 = split * chunk, l1 = min(L, l0 + chunk);
  const float q = qs[(size_t)bh * PA_K + lane];
  const float ls = lse[bh];
  const float do0 = dO[(size_t)bh * PA_VD + 2 * lane], do1 = dO[(size_t)bh * PA_VD + 2 * lane + 1];
  const float D = wave_reduce_sum(do0 * o[(size_t)bh * PA_VD + 2 * lane] + do1 * o[(size_t)bh * PA_VD + 2 * lane + 1]);
  const size_t koff = (size_t)b * L * N + h * PA_K + lane;
  const size_t voff = (size_t)b * L * N + H * PA_K + h * PA_VD + 2 * lane;
  const unsigned char* mrow = mask ? mask + (size_t)b * L : nullptr;

  float dqa = 0.f;
  for (int base = l0 + wave; base < l1; base += PA_WAVES * PA_UNROLL) {
    float t[PA_UNROLL], s[PA_UNROLL], v0[PA_UNROLL], v1[PA_UNROLL], dp[PA_UNROLL], gd0[PA_UNROLL], gd1[PA_UNROLL];
    bool ok[PA_UNROLL];
#pragma unroll
    for (int u = 0; u < PA_UNROLL; ++u) {
      const int l = base + u * PA_WAVES;
      const int lc = min(l, l1 - 1);
      ok[u] = !mrow || mrow[lc];
      t[u] = tanh_f(bf2f(pre[koff + (size_t)lc * N]));
      const unsigned int vv = *reinterpret_cast<const unsigned int*>(pre + voff + (size_t)lc * N);
      v0[u] = bf2f((unsigned short)(vv & 0xffff));
      v1[u] = bf2f((unsigned short)(vv >> 16));
      float c, pd;
      gelu_parts(v0[u], c, pd);
      gd0[u] = fmaf(v0[u], pd, c);
      const float g0 = v0[u] * c;
      gelu_parts(v1[u], c, pd);
      gd1[u] = fmaf(v1[u], pd, c);
      const float g1 = v1[u] * c;
      s[u] = q * t[u];
      dp[u] = fmaf(do0, g0, do1 * g1);
    }
#pragma unroll
    for (int u = 0; u < PA_UNROLL; ++u) {
      s[u] = wave_reduce_sum(s[u]);
      dp[u] = wave_reduce_sum(dp[u]);
    }
#pragma unroll
    for (int u = 0; u < PA_UNROLL; ++u) {
      const int l = base + u * PA_WAVES;
      if (l >= l1) continue;                                // wave-uniform
      const float p = ok[u] ? __expf(s[u] - ls) : 0.f;
      const float ds = p * (dp[u] - D);
      const float dk = ds * q * fmaf(-t[u], t[u], 1.0f);
      dqa = fmaf(ds, t[u], dqa);
      dpre[koff + (size_t)l * N] = f2bf(dk);
      const unsigned int pk = (unsigned int)f2bf(p * do0 * gd0[u]) | ((unsigned int)f2bf(p * do1 * gd1[u]) << 16);
      *reinterpret_cast<unsigned int*>(dpre + voff + (size_t)l * N) = pk;
    }
  }
  __shared__ float sq[PA_WAVES][PA_K];
  sq[wave][lane] = dqa;
  __syncthreads();
  if (wave == 0) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < PA_WAVES; ++w) a += sq[w][lane];
    dq_part[((size_t)bh * nsplit + split) * PA_K + lane] = a;
  }
}

}  // namespace

// pre [B, L, H*(K+VD)] bf16, qs [B*H, K] fp32 (tanh(q) / sqrt(K)), mask [B, L] u8 or null,
// part [B*H, nsplit, 2+VD] fp32 workspace, o [B*H, VD] fp32, lse [B*H] fp32
PBX_EXPORT int pbx_paper_attn_fwd(const void* pre, const void* qs, const void* mask, void* part, void* o, void* lse,
                                  int B, int L, int H, int K, int VD, int nsplit, hipStream_t stream) {
  if (K != PA_K || VD != PA_VD || B <= 0 || L <= 0 || H <= 0 || nsplit <= 0 || nsplit > L) return (int)hipErrorInvalidValue;
  const int chunk = (L + nsplit - 1) / nsplit;
  if ((nsplit - 1) * chunk >= L) return (int)hipErrorInvalidValue;   // every chunk non-empty
  hipLaunchKernelGGL(paper_attn_fwd_kernel, dim3(nsplit, B * H), dim3(256), 0, stream,
                     (const unsigned short*)pre, (const float*)qs, (const unsigned char*)mask, (float*)part, L, H,
                     chunk, nsplit);
  hipLaunchKernelGGL(paper_attn_combine_kernel, dim3(B * H), dim3(64), 0, stream, (const float*)part, (float*)o,
                     (float*)lse, nsplit);
  return pbx_launch_status();
}

// dpre [B, L, H*(K+VD)] bf16 (every element written), dq_part [B*H, nsplit, K] fp32
PBX_EXPORT int pbx_paper_attn_bwd(const void* pre, const void* qs, const void* mask, const void* lse, const void* o,
                                  const void* dO, void* dpre, void* dq_part, int B, int L, int H, int K, int VD,
                                  int nsplit, hipStream_t stream) {
  if (K != PA_K || VD != PA_VD || B <= 0 || L <= 0 || H <= 0 || nsplit <= 0 || nsplit > L) return (int)hipErrorInvalidValue;
  const int chunk = (L + nsplit - 1) / nsplit;
  if ((nsplit - 1) * chunk >= L) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(paper_attn_bwd_kernel, dim3(nsplit, B * H), dim3(256), 0, stream,
                     (const unsigned short*)pre, (const float*)qs, (const unsigned char*)mask, (const float*)lse,
                     (const float*)o, (const float*)dO, (unsigned short*)dpre, (float*)dq_part, L, H, chunk, nsplit);
  return pbx_launch_status();
}
