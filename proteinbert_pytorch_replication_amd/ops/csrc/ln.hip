// Whole-sequence LayerNorm, local MLP, local->global attention pool and their backward passes
// (reference semantics).
//
// Reference: ProteinBERT/modules.py:148-164 (LayerNorm over (L, C) with an [L, C] affine, twice),
// :153-164,214-217 (Linear C->C + GELU + residual), :21-92,219 (global attention).  In reference
// semantics the attention softmax runs over an axis whose rows are identical, so every head
// reduces exactly to (1/K) * sum_l GELU(h Wv_j); the pool is one GEMM
// [rows, 128] x [128, 512] with a GELU + column-sum epilogue.  Statistics of the (L, C)
// LayerNorms span the whole sequence, so every producer writes per-tile partials ((mean, M2)
// forward, (sum dxhat, sum dxhat*xhat) backward) and every consumer combines them.
//
// Tiles are 128 positions of one sequence; a workgroup (4 waves, 32 positions each) is persistent
// over tiles so the weight matrix it needs is staged into LDS once.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int BML = 128;   // LN-kernel tile (positions)

__device__ __forceinline__ void load_f8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 c = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
}
__device__ __forceinline__ void load_f4(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}

// stage a [rows x 128] bf16 weight matrix into a swz256 LDS image (256 threads)
__device__ __forceinline__ void stage_weight(unsigned char* dst, const bf16_t* __restrict__ w, int rows) {
  for (int idx = threadIdx.x; idx < rows * 16; idx += 256) {
    const int row = idx >> 4, ch = idx & 15;
    *reinterpret_cast<uint4*>(dst + swz256(row, ch)) =
        *reinterpret_cast<const uint4*>(w + (size_t)row * CH + ch * 8);
  }
}

// ------------------------------------------------------------------------------------------------
// h1 = LN(s1) ; pre = h1 Wl^T + bl ; s2 = h1 + GELU(pre)  (+ s2 tile (mean, M2) partials)
__global__ void __launch_bounds__(256) ln_linear_fwd_kernel(
    const bf16_t* __restrict__ s1, const float* __restrict__ st1, int T1, int BM1, const float* __restrict__ g1,
    const float* __restrict__ be1, const bf16_t* __restrict__ wl, const float* __restrict__ bl,
    bf16_t* __restrict__ pre_l, bf16_t* __restrict__ s2, float* __restrict__ st2, int B, int L, float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;                                     // 32 KB
  float* scratch = reinterpret_cast<float*>(smem + 32768);      // 16 floats
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int T2 = (L + BML - 1) / BML;
  stage_weight(ws, wl, CH);
  __syncthreads();
  for (int tile = blockIdx.x; tile < B * T2; tile += gridDim.x) {
    const int b = tile / T2, t = tile - (tile / T2) * T2;
    const int pos0 = t * BML;
    float mean, rstd;
    ln_stats(st1 + (size_t)b * T1 * 2, T1, BM1, L, CH, eps, mean, rstd);
    const int p = w * 32 + r;
    const int pos = pos0 + p;
    const bool okb = pos < L;
    const size_t rowoff = ((size_t)b * L + pos) * CH;
    bf16x8 hf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int ci = kk * 16 + 8 * h;
      float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (okb) {
        float s[8], g[8], be[8];
        unpack8(*reinterpret_cast<const uint4*>(s1 + rowoff + ci), s);
        load_f8(g1 + (size_t)pos * CH + ci, g);
        load_f8(be1 + (size_t)pos * CH + ci, be);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (s[e] - mean) * rstd * g[e] + be[e];
      }
      hf[kk] = pack8(v);
    }
    f32x16_t acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = zero16();
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        acc[ct] = mfma32(lds_frag(ws, swz256(ct * 32 + r, kk * 2 + h)), hf[kk], acc[ct]);
    // D[co][pos]: lane -> position p, registers -> output channels
    float lsum = 0.f;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int co0 = ct * 32 + 8 * g + 4 * h;
        float s[4] = {0, 0, 0, 0}, gg[4] = {0, 0, 0, 0}, be[4] = {0, 0, 0, 0}, bb[4], pre[4], o[4];
        if (okb) {
          unpack4(*reinterpret_cast<const uint2*>(s1 + rowoff + co0), s);
          load_f4(g1 + (size_t)pos * CH + co0, gg);
          load_f4(be1 + (size_t)pos * CH + co0, be);
        }
        load_f4(bl + co0, bb);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float h1 = (s[e] - mean) * rstd * gg[e] + be[e];
          pre[e] = acc[ct][4 * g + e] + bb[e];
          o[e] = okb ? bfround(h1 + gelu_f(pre[e])) : 0.f;
          acc[ct][4 * g + e] = o[e];
          lsum += o[e];
        }
        if (okb) {
          *reinterpret_cast<uint2*>(pre_l + rowoff + co0) = packq4(pre);
          *reinterpret_cast<uint2*>(s2 + rowoff + co0) = packq4(o);
        }
      }
    const int vrows = min(BML, L - pos0);
    const float tmean = block_sum(lsum, scratch, 4) / (float)(vrows * CH);
    float m2 = 0.f;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float d = acc[ct][i] - tmean;
        m2 += okb ? d * d : 0.f;
      }
    m2 = block_sum(m2, scratch + 4, 4);
    if (tid == 0) {
      st2[((size_t)b * T2 + t) * 2] = tmean;
      st2[((size_t)b * T2 + t) * 2 + 1] = m2;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// h2 = LN(s2) (written: block output) ; vpart[b][t][j] = sum_{pos in tile} GELU(h2[pos] . Wv[j])
__global__ void __launch_bounds__(256) ln_attn_fwd_kernel(
    const bf16_t* __restrict__ s2, const float* __restrict__ st2, const float* __restrict__ g2,
    const float* __restrict__ be2, const bf16_t* __restrict__ wv, bf16_t* __restrict__ h2,
    float* __restrict__ vpart, int B, int L, int NJ, float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;                                          // NJ rows x 256 B
  float* red = reinterpret_cast<float*>(smem + NJ * 256);            // NJ floats
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int T2 = (L + BML - 1) / BML;
  stage_weight(ws, wv, NJ);
  __syncthreads();
  for (int tile = blockIdx.x; tile < B * T2; tile += gridDim.x) {
    const int b = tile / T2, t = tile - (tile / T2) * T2;
    const int pos0 = t * BML;
    float mean, rstd;
    ln_stats(st2 + (size_t)b * T2 * 2, T2, BML, L, CH, eps, mean, rstd);
    for (int j = tid; j < NJ; j += 256) red[j] = 0.f;
    const int pos = pos0 + w * 32 + r;
    const bool okb = pos < L;
    const size_t rowoff = ((size_t)b * L + pos) * CH;
    bf16x8 hf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int ci = kk * 16 + 8 * h;
      float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (okb) {
        float s[8], g[8], be[8];
        unpack8(*reinterpret_cast<const uint4*>(s2 + rowoff + ci), s);
        load_f8(g2 + (size_t)pos * CH + ci, g);
        load_f8(be2 + (size_t)pos * CH + ci, be);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (s[e] - mean) * rstd * g[e] + be[e];
        const uint4 q = packq8(v);
        *reinterpret_cast<uint4*>(h2 + rowoff + ci) = q;
        hf[kk] = __builtin_bit_cast(bf16x8, q);
      } else {
        hf[kk] = pack8(v);
      }
    }
    __syncthreads();   // red zeroed
    // D[pos][j]: lane -> column j, registers -> positions; GELU then sum over positions
    const int rowbase = pos0 + w * 32 + 4 * h;
    for (int jt = 0; jt < NJ / 32; ++jt) {
      f32x16_t acc = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) acc = mfma32(hf[kk], lds_frag(ws, swz256(jt * 32 + r, kk * 2 + h)), acc);
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int prow = rowbase + (i & 3) + 8 * (i >> 2);
        s += prow < L ? gelu_f(acc[i]) : 0.f;
      }
      s += __shfl_xor(s, 32, 64);
      if (h == 0) atomicAdd(&red[jt * 32 + r], s);
    }
    __syncthreads();
    for (int j = tid; j < NJ; j += 256) vpart[((size_t)b * T2 + t) * NJ + j] = red[j];
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// attention pool backward + LayerNorm-2 backward partials.
// dP[j][pos] = dv[b][t][j] * GELU'(Wv[j] . h2[pos]) ; dh2 = dh2_in + Wv^T dP  (dP never leaves
// registers: the 32x32 accumulator of the recompute is the B operand of the second MFMA)
__global__ void __launch_bounds__(256) attn_bwd_kernel(
    const bf16_t* __restrict__ h2, const bf16_t* __restrict__ s2, const float* __restrict__ st2,
    const float* __restrict__ g2, const bf16_t* __restrict__ dh2_in, const float* __restrict__ dvpart,
    const bf16_t* __restrict__ wv, bf16_t* __restrict__ dh2, float* __restrict__ sums2, int B, int L, int NJ,
    float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;
  float* scratch = reinterpret_cast<float*>(smem + NJ * 256);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int T2 = (L + BML - 1) / BML;
  stage_weight(ws, wv, NJ);
  __syncthreads();
  for (int tile = blockIdx.x; tile < B * T2; tile += gridDim.x) {
    const int b = tile / T2, t = tile - (tile / T2) * T2;
    const int pos0 = t * BML;
    const int pos = pos0 + w * 32 + r;
    const bool okb = pos < L;
    const size_t rowoff = ((size_t)b * L + pos) * CH;
    bf16x8 hf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (okb) v = *reinterpret_cast<const uint4*>(h2 + rowoff + kk * 16 + 8 * h);
      hf[kk] = __builtin_bit_cast(bf16x8, v);
    }
    f32x16_t y[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) y[ct] = zero16();
    const float* dv = dvpart + ((size_t)b * T2 + t) * NJ;
    for (int jt = 0; jt < NJ / 32; ++jt) {
      f32x16_t d1 = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) d1 = mfma32(lds_frag(ws, swz256(jt * 32 + r, kk * 2 + h)), hf[kk], d1);
      float dp[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float dvv[4];
        load_f4(dv + jt * 32 + 8 * g + 4 * h, dvv);
#pragma unroll
        for (int e = 0; e < 4; ++e) dp[4 * g + e] = okb ? dvv[e] * gelu_grad_f(d1[4 * g + e]) : 0.f;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 fb = pack8(dp + 8 * s);
        const int rlo = jt * 32 + 16 * s + 4 * h + q;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const int col = ct * 32 + tc;
          const bf16x8 fa = cat_tr(lds_tr(ws, swz256e(rlo, col)), lds_tr(ws, swz256e(rlo + 8, col)));
          y[ct] = mfma32(fa, fb, y[ct]);
        }
      }
    }
    // Y[ci][pos]; LN2 backward partials
    float mean, rstd;
    ln_stats(st2 + (size_t)b * T2 * 2, T2, BML, L, CH, eps, mean, rstd);
    float sa = 0.f, sc = 0.f;
    if (okb) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ci0 = ct * 32 + 8 * g + 4 * h;
          float din[4] = {0, 0, 0, 0}, s[4], gg[4], o[4];
          if (dh2_in != nullptr) unpack4(*reinterpret_cast<const uint2*>(dh2_in + rowoff + ci0), din);
          unpack4(*reinterpret_cast<const uint2*>(s2 + rowoff + ci0), s);
          load_f4(g2 + (size_t)pos * CH + ci0, gg);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = bfround(din[e] + y[ct][4 * g + e]);
            const float xh = (s[e] - mean) * rstd;
            const float dxh = o[e] * gg[e];
            sa += dxh;
            sc += dxh * xh;
          }
          *reinterpret_cast<uint2*>(dh2 + rowoff + ci0) = packq4(o);
        }
    }
    sa = block_sum(sa, scratch, 4);
    sc = block_sum(sc, scratch + 4, 4);
    if (tid == 0) {
      sums2[((size_t)b * T2 + t) * 2] = sa;
      sums2[((size_t)b * T2 + t) * 2 + 1] = sc;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// LayerNorm-2 backward finalize + local MLP backward + LayerNorm-1 backward partials.
// ds2 = rstd2 (dh2 g2 - m1 - xhat2 m2) ; dpre = ds2 GELU'(pre) ; dh1 = ds2 + Wl^T dpre
// writes dh1, dpre (and the recomputed h1) for the Linear weight gradient.
__global__ void __launch_bounds__(256) ln2_linear_bwd_kernel(
    const bf16_t* __restrict__ dh2, const bf16_t* __restrict__ s2, const float* __restrict__ st2,
    const float* __restrict__ sums2, const float* __restrict__ g2, const bf16_t* __restrict__ pre_l,
    const bf16_t* __restrict__ s1, const float* __restrict__ st1, int T1, int BM1, const float* __restrict__ g1,
    const float* __restrict__ be1, const bf16_t* __restrict__ wl, bf16_t* __restrict__ dh1,
    bf16_t* __restrict__ dpre_out, bf16_t* __restrict__ h1_out, float* __restrict__ sums1, int B, int L,
    float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;
  float* scratch = reinterpret_cast<float*>(smem + 32768);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int T2 = (L + BML - 1) / BML;
  const float inv_n = 1.0f / (float)(L * CH);
  stage_weight(ws, wl, CH);
  __syncthreads();
  for (int tile = blockIdx.x; tile < B * T2; tile += gridDim.x) {
    const int b = tile / T2, t = tile - (tile / T2) * T2;
    const int pos0 = t * BML;
    const int pos = pos0 + w * 32 + r;
    const bool okb = pos < L;
    const size_t rowoff = ((size_t)b * L + pos) * CH;
    float mean2, rstd2, m1, m2, mean1, rstd1;
    ln_stats(st2 + (size_t)b * T2 * 2, T2, BML, L, CH, eps, mean2, rstd2);
    ln_bwd_consts(sums2 + (size_t)b * T2 * 2, T2, inv_n, m1, m2);
    ln_stats(st1 + (size_t)b * T1 * 2, T1, BM1, L, CH, eps, mean1, rstd1);
    bf16x8 df[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int co = kk * 16 + 8 * h;
      float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (okb) {
        float dh[8], s[8], g[8], pr[8];
        unpack8(*reinterpret_cast<const uint4*>(dh2 + rowoff + co), dh);
        unpack8(*reinterpret_cast<const uint4*>(s2 + rowoff + co), s);
        unpack8(*reinterpret_cast<const uint4*>(pre_l + rowoff + co), pr);
        load_f8(g2 + (size_t)pos * CH + co, g);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (s[e] - mean2) * rstd2;
          const float ds = rstd2 * (dh[e] * g[e] - m1 - xh * m2);
          v[e] = ds * gelu_grad_f(pr[e]);
        }
        const uint4 qv = packq8(v);
        *reinterpret_cast<uint4*>(dpre_out + rowoff + co) = qv;
        df[kk] = __builtin_bit_cast(bf16x8, qv);
      } else {
        df[kk] = pack8(v);
      }
    }
    f32x16_t y[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) y[ct] = zero16();
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int rlo = kk * 16 + 8 * h + q;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int col = ct * 32 + tc;
        const bf16x8 fa = cat_tr(lds_tr(ws, swz256e(rlo, col)), lds_tr(ws, swz256e(rlo + 4, col)));
        y[ct] = mfma32(fa, df[kk], y[ct]);
      }
    }
    float sa = 0.f, sc = 0.f;
    if (okb) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ci0 = ct * 32 + 8 * g + 4 * h;
          float dh[4], s[4], gg[4], sv1[4], ga[4], bb[4], o[4], hv[4];
          unpack4(*reinterpret_cast<const uint2*>(dh2 + rowoff + ci0), dh);
          unpack4(*reinterpret_cast<const uint2*>(s2 + rowoff + ci0), s);
          load_f4(g2 + (size_t)pos * CH + ci0, gg);
          unpack4(*reinterpret_cast<const uint2*>(s1 + rowoff + ci0), sv1);
          load_f4(g1 + (size_t)pos * CH + ci0, ga);
          load_f4(be1 + (size_t)pos * CH + ci0, bb);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float xh2 = (s[e] - mean2) * rstd2;
            const float ds = rstd2 * (dh[e] * gg[e] - m1 - xh2 * m2);
            o[e] = bfround(ds + y[ct][4 * g + e]);
            const float xh1 = (sv1[e] - mean1) * rstd1;
            hv[e] = xh1 * ga[e] + bb[e];
            const float dxh = o[e] * ga[e];
            sa += dxh;
            sc += dxh * xh1;
          }
          *reinterpret_cast<uint2*>(dh1 + rowoff + ci0) = packq4(o);
          *reinterpret_cast<uint2*>(h1_out + rowoff + ci0) = packq4(hv);
        }
    }
    sa = block_sum(sa, scratch, 4);
    sc = block_sum(sc, scratch + 4, 4);
    if (tid == 0) {
      sums1[((size_t)b * T2 + t) * 2] = sa;
      sums1[((size_t)b * T2 + t) * 2 + 1] = sc;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// [L, C]-affine gradients of a whole-sequence LayerNorm (sum over the batch) and, optionally, the
// input gradient ds = rstd (dh g - m1 - xhat m2) plus its per-sample column sum (gradient of the
// broadcast global->local vector, reference modules.py:208-211).
// grid (ceil(L/16), nbg); thread = (position pl = tid>>4, channel chunk c8 = tid&15)
__global__ void __launch_bounds__(256) ln_affine_bwd_kernel(
    const bf16_t* __restrict__ dh, const bf16_t* __restrict__ s, const float* __restrict__ st, int Tst, int BMst,
    const float* __restrict__ sums, int Tsm, const float* __restrict__ gamma, float* __restrict__ dgamma,
    float* __restrict__ dbeta, bf16_t* __restrict__ ds, float* __restrict__ dgb, int B, int L, float eps) {
  __shared__ float consts[4 * 64];
  __shared__ float red[16 * CH];
  const int tid = threadIdx.x, pl = tid >> 4, c8 = tid & 15;
  const int l = blockIdx.x * 16 + pl;
  const int nbg = gridDim.y, bg = blockIdx.y;
  const int b0 = (int)((long)B * bg / nbg), b1 = (int)((long)B * (bg + 1) / nbg);
  const float inv_n = 1.0f / (float)(L * CH);
  const bool okl = l < L;
  float gam[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (okl) load_f8(gamma + (size_t)l * CH + c8 * 8, gam);
  float dg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, db[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int bc = b0; bc < b1; bc += 64) {
    const int nb = min(64, b1 - bc);
    __syncthreads();
    if (tid < nb) {
      const int bb = bc + tid;
      float mean, rstd, m1, m2;
      ln_stats(st + (size_t)bb * Tst * 2, Tst, BMst, L, CH, eps, mean, rstd);
      ln_bwd_consts(sums + (size_t)bb * Tsm * 2, Tsm, inv_n, m1, m2);
      consts[4 * tid] = mean; consts[4 * tid + 1] = rstd; consts[4 * tid + 2] = m1; consts[4 * tid + 3] = m2;
    }
    __syncthreads();
    for (int i = 0; i < nb; ++i) {
      const int bb = bc + i;
      const float mean = consts[4 * i], rstd = consts[4 * i + 1], m1 = consts[4 * i + 2], m2 = consts[4 * i + 3];
      float dsv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (okl) {
        const size_t off = ((size_t)bb * L + l) * CH + c8 * 8;
        float dv[8], sv[8];
        unpack8(*reinterpret_cast<const uint4*>(dh + off), dv);
        unpack8(*reinterpret_cast<const uint4*>(s + off), sv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (sv[e] - mean) * rstd;
          dg[e] += dv[e] * xh;
          db[e] += dv[e];
          dsv[e] = rstd * (dv[e] * gam[e] - m1 - xh * m2);
        }
        if (ds != nullptr) {
          const uint4 qv = packq8(dsv);
          *reinterpret_cast<uint4*>(ds + off) = qv;
          unpack8(qv, dsv);
        }
      }
      if (dgb != nullptr) {
#pragma unroll
        for (int e = 0; e < 8; ++e) red[pl * CH + c8 * 8 + e] = dsv[e];
        __syncthreads();
        if (tid < CH) {
          float a = 0.f;
#pragma unroll
          for (int k = 0; k < 16; ++k) a += red[k * CH + tid];
          atomicAdd(dgb + (size_t)bb * CH + tid, a);
        }
        __syncthreads();
      }
    }
  }
  if (okl) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      atomicAdd(dgamma + (size_t)l * CH + c8 * 8 + e, dg[e]);
      atomicAdd(dbeta + (size_t)l * CH + c8 * 8 + e, db[e]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// token embedding: forward gather to bf16, backward per-token segmented sum
__global__ void __launch_bounds__(256) embed_fwd_kernel(const long long* __restrict__ tok, const float* __restrict__ E,
                                                        bf16_t* __restrict__ out, long rows) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * 16) return;
  const long row = i >> 4;
  const int c8 = (int)(i & 15);
  const long long t = tok[row];
  float v[8];
  load_f8(E + (size_t)t * CH + c8 * 8, v);
  *reinterpret_cast<uint4*>(out + row * CH + c8 * 8) = packq8(v);
}

__global__ void __launch_bounds__(256) embed_bwd_kernel(const long long* __restrict__ tok,
                                                        const bf16_t* __restrict__ dout, float* __restrict__ dE,
                                                        long rows, int V) {
  __shared__ float acc[32 * CH];
  for (int i = threadIdx.x; i < V * CH; i += 256) acc[i] = 0.f;
  __syncthreads();
  const int c8 = threadIdx.x & 15;
  for (long row = (long)blockIdx.x * 16 + (threadIdx.x >> 4); row < rows; row += (long)gridDim.x * 16) {
    const int t = (int)tok[row];
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(dout + row * CH + c8 * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) atomicAdd(&acc[t * CH + c8 * 8 + e], v[e]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < V * CH; i += 256) atomicAdd(dE + i, acc[i]);
}

int grid_for(int tiles) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess) cus = p.multiProcessorCount;
  }
  return tiles < cus ? tiles : cus;
}
int g_cus = -1;
int persistent_grid(int tiles) {
  if (g_cus < 0) g_cus = grid_for(1 << 30);
  return tiles < g_cus ? (tiles > 0 ? tiles : 1) : g_cus;
}
}  // namespace

static bool ln_attrs_set = false;
static void set_ln_attrs() {
  if (ln_attrs_set) return;
  (void)hipFuncSetAttribute((const void*)ln_attn_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  ln_attrs_set = true;
}

PBX_EXPORT int pbx_ln_linear_fwd(const void* s1, const float* st1, int T1, int BM1, const float* g1,
                                 const float* be1, const void* wl, const float* bl, void* pre_l, void* s2,
                                 float* st2, int B, int L, float eps, hipStream_t st) {
  const int T2 = (L + BML - 1) / BML;
  hipLaunchKernelGGL(ln_linear_fwd_kernel, dim3(persistent_grid(B * T2)), dim3(256), 32768 + 64, st,
                     (const bf16_t*)s1, st1, T1, BM1, g1, be1, (const bf16_t*)wl, bl, (bf16_t*)pre_l, (bf16_t*)s2,
                     st2, B, L, eps);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_ln_attn_fwd(const void* s2, const float* st2, const float* g2, const float* be2, const void* wv,
                               void* h2, float* vpart, int B, int L, int NJ, float eps, hipStream_t st) {
  set_ln_attrs();
  if (NJ % 32 != 0 || NJ * 256 + NJ * 4 > 163840) return (int)hipErrorInvalidValue;
  const int T2 = (L + BML - 1) / BML;
  hipLaunchKernelGGL(ln_attn_fwd_kernel, dim3(persistent_grid(B * T2)), dim3(256), NJ * 256 + NJ * 4, st,
                     (const bf16_t*)s2, st2, g2, be2, (const bf16_t*)wv, (bf16_t*)h2, vpart, B, L, NJ, eps);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_attn_bwd(const void* h2, const void* s2, const float* st2, const float* g2, const void* dh2_in,
                            const float* dvpart, const void* wv, void* dh2, float* sums2, int B, int L, int NJ,
                            float eps, hipStream_t st) {
  set_ln_attrs();
  if (NJ % 32 != 0 || NJ * 256 + 64 > 163840) return (int)hipErrorInvalidValue;
  const int T2 = (L + BML - 1) / BML;
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(persistent_grid(B * T2)), dim3(256), NJ * 256 + 64, st,
                     (const bf16_t*)h2, (const bf16_t*)s2, st2, g2, (const bf16_t*)dh2_in, dvpart,
                     (const bf16_t*)wv, (bf16_t*)dh2, sums2, B, L, NJ, eps);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_ln2_linear_bwd(const void* dh2, const void* s2, const float* st2, const float* sums2,
                                  const float* g2, const void* pre_l, const void* s1, const float* st1, int T1,
                                  int BM1, const float* g1, const float* be1, const void* wl, void* dh1,
                                  void* dpre, void* h1, float* sums1, int B, int L, float eps, hipStream_t st) {
  const int T2 = (L + BML - 1) / BML;
  hipLaunchKernelGGL(ln2_linear_bwd_kernel, dim3(persistent_grid(B * T2)), dim3(256), 32768 + 64, st,
                     (const bf16_t*)dh2, (const bf16_t*)s2, st2, sums2, g2, (const bf16_t*)pre_l,
                     (const bf16_t*)s1, st1, T1, BM1, g1, be1, (const bf16_t*)wl, (bf16_t*)dh1, (bf16_t*)dpre,
                     (bf16_t*)h1, sums1, B, L, eps);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_ln_affine_bwd(const void* dh, const void* s, const float* stp, int Tst, int BMst,
                                 const float* sums, int Tsm, const float* gamma, float* dgamma, float* dbeta,
                                 void* ds, float* dgb, int B, int L, int nbg, float eps, hipStream_t st) {
  dim3 grid((L + 15) / 16, nbg);
  hipLaunchKernelGGL(ln_affine_bwd_kernel, grid, dim3(256), 0, st, (const bf16_t*)dh, (const bf16_t*)s, stp, Tst,
                     BMst, sums, Tsm, gamma, dgamma, dbeta, (bf16_t*)ds, dgb, B, L, eps);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_embed_fwd(const void* tok, const float* E, void* out, long rows, hipStream_t st) {
  const long n = rows * 16;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const long long*)tok, E,
                     (bf16_t*)out, rows);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_embed_bwd(const void* tok, const void* dout, float* dE, long rows, int V, hipStream_t st) {
  if (V > 32) return (int)hipErrorInvalidValue;
  long g = (rows + 15) / 16;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)g), dim3(256), 0, st, (const long long*)tok,
                     (const bf16_t*)dout, dE, rows, V);
  return pbx_launch_status();
}
