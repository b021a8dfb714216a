// Whole-sequence LayerNorm and local MLP forward / backward passes (reference semantics;
// the attention pool and the LayerNorm-2 apply are csrc/pool.hip).
//
// Reference: ProteinBERT/modules.py:148-164 (LayerNorm over (L, C) with an [L, C] affine, twice),
// :153-164,214-217 (Linear C->C + GELU + residual), :21-92,219 (global attention).  In reference
// semantics the attention softmax runs over an axis whose rows are identical, so every head
// reduces exactly to (1/K) * sum_l GELU(h Wv_j).  Statistics of the (L, C)
// LayerNorms span the whole sequence, so every producer writes per-tile partials ((mean, M2)
// forward, (sum dxhat, sum dxhat*xhat) backward) and every consumer combines them.
//
// Tiles are 128 positions of one sequence; a workgroup (4 waves, 32 positions each) is persistent
// over tiles so the weight matrix it needs is staged into LDS once.
#include "mfma.h"
#include <stdlib.h>

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int BML = 32;    // tile of the s2 (mean, M2) partials written by ln_linear_fwd

__device__ __forceinline__ void load_f8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 c = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
}

// stage a [rows x 128] bf16 weight matrix into a swz256 LDS image (whole workgroup)
__device__ __forceinline__ void stage_weight(unsigned char* dst, const bf16_t* __restrict__ w, int rows) {
  stage_chunks(
      rows * 16, [&](int idx) { return *reinterpret_cast<const uint4*>(w + (size_t)idx * 8); },
      [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(dst + swz256(idx >> 4, idx & 15)) = v; });
}

// ------------------------------------------------------------------------------------------------
// Position-major LayerNorm kernels.  A workgroup owns PB = 32 positions of the [L, C] LayerNorm
// affine and walks a group of samples, so every thread keeps the affine parameters (and, in the
// backward, the affine-gradient accumulators) of its fixed (position, 8-channel chunk) in registers
// and the next sample's rows are prefetched while the current one is in the MFMA.
// Thread t (of 512) owns row j = t >> 4 (position l0 + j) and channel chunk ch = t & 15.
constexpr int PB = 32;
constexpr int YS = CH + 4;   // padded row stride of the fp32 D^T tile (lanes write 32 different rows)

__device__ __forceinline__ uint4 ldq(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u);
}

// per-sample statistics through LDS (computed by one wave, broadcast)
__device__ __forceinline__ void sample_stats(float* sh, const float* __restrict__ st, int T, int BM, int L, float eps,
                                             const float* __restrict__ sums, int Ts, float inv_n) {
  if (threadIdx.x == 0) {
    float mean, rstd;
    ln_stats(st, T, BM, L, CH, eps, mean, rstd);
    sh[0] = mean;
    sh[1] = rstd;
    if (sums != nullptr) {
      float m1, m2;
      ln_bwd_consts(sums, Ts, inv_n, m1, m2);
      sh[2] = m1;
      sh[3] = m2;
    }
  }
}

// h1 = LN(s1) ; pre = h1 Wl^T + bl ; s2 = h1 + GELU(pre)  (+ s2 (mean, M2) partial per 32 positions)
// grid (ceil(L/PB), nbg), 512 threads; waves 0-3 run the 32x32 MFMA tiles of D[co][pos].
// Per-sample LN1 statistics are computed for all of the workgroup's samples up front (one wave per
// sample, parallel partial loads) and the s2 tile partials are merged per wave into an LDS table
// that is reduced once at the end, so a sample costs two barriers.
__global__ void __launch_bounds__(512) ln_linear_fwd_kernel(
    const bf16_t* __restrict__ s1, const float* __restrict__ st1, int T1, int BM1, const float* __restrict__ g1,
    const float* __restrict__ be1, const bf16_t* __restrict__ wl, const float* __restrict__ bl,
    bf16_t* __restrict__ pre_l, bf16_t* __restrict__ s2, float* __restrict__ st2, int B, int L, float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;                                          // Wl, 32 KB
  unsigned char* ht = smem + 32768;                                  // h1 tile bf16, PB x 256 B
  float* yt = reinterpret_cast<float*>(smem + 32768 + PB * 256);     // D^T tile fp32 [PB][YS]
  float* tab = yt + PB * YS;                                         // [nb][2] stats, [nb][8][2] partials
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int j = tid >> 4, ch = tid & 15;
  const int l0 = blockIdx.x * PB, l = l0 + j;
  const bool okl = l < L;
  const int TP = (L + PB - 1) / PB;
  const int nbg = gridDim.y;
  const int b0 = (int)((long)B * blockIdx.y / nbg), b1 = (int)((long)B * (blockIdx.y + 1) / nbg);
  const int nb = b1 - b0;
  float* part = tab + 2 * nb;
  stage_weight(ws, wl, CH);
  for (int i = w; i < nb; i += 8) {
    float mean, rstd;
    wave_ln_stats(st1 + (size_t)(b0 + i) * T1 * 2, T1, BM1, L, CH, eps, mean, rstd);
    if (lane == 0) {
      tab[2 * i] = mean;
      tab[2 * i + 1] = rstd;
    }
  }
  float gam[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bet[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bb[8];
  if (okl) {
    load_f8(g1 + (size_t)l * CH + ch * 8, gam);
    load_f8(be1 + (size_t)l * CH + ch * 8, bet);
  }
  load_f8(bl + ch * 8, bb);
  uint4 nxt = ldq(s1 + ((size_t)b0 * L + l) * CH + ch * 8, okl && nb > 0);
  __syncthreads();
  for (int b = b0; b < b1; ++b) {
    const int i = b - b0;
    const float mean = tab[2 * i], rstd = tab[2 * i + 1];
    float sv[8], h1[8];
    unpack8(nxt, sv);
#pragma unroll
    for (int e = 0; e < 8; ++e) h1[e] = okl ? (sv[e] - mean) * rstd * gam[e] + bet[e] : 0.f;
    *reinterpret_cast<uint4*>(ht + swz256(j, ch)) = packq8(h1);
    __syncthreads();
    nxt = ldq(s1 + ((size_t)(b + 1) * L + l) * CH + ch * 8, okl && b + 1 < b1);
    if (w < 4) {
      f32x16_t acc = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
        acc = mfma32(lds_frag(ws, swz256(w * 32 + r, kk * 2 + h)), lds_frag(ht, swz256(r, kk * 2 + h)), acc);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(yt + r * YS + w * 32 + 8 * g + 4 * h) =
            make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
    }
    __syncthreads();
    float pre[8], o[8];
    const float4 ya = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8);
    const float4 yb = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8 + 4);
    const float yv[8] = {ya.x, ya.y, ya.z, ya.w, yb.x, yb.y, yb.z, yb.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) pre[e] = yv[e] + bb[e];
    f32x2 gg[4];
    {
      const f32x2 xi[4] = {(f32x2){pre[0], pre[1]}, (f32x2){pre[2], pre[3]}, (f32x2){pre[4], pre[5]},
                           (f32x2){pre[6], pre[7]}};
      gelu2_fast_n<4, false>(xi, gg);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = h1[e] + ((e & 1) ? gg[e >> 1].y : gg[e >> 1].x);
    const uint4 oq = packq8(o);
    if (okl) {
      const size_t off = ((size_t)b * L + l) * CH + ch * 8;
      if (pre_l != nullptr) *reinterpret_cast<uint4*>(pre_l + off) = packq8(pre);   // null: no backward
      *reinterpret_cast<uint4*>(s2 + off) = oq;
    }
    // (sum, sum of squares) of the stored values, reduced over the wave into the LDS partial table
    // (a per-lane Chan merge costs a division per butterfly step)
    float orr[8];
    unpack8(oq, orr);
    float sa = 0.f, sq = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sa += orr[e];
      sq += orr[e] * orr[e];
    }
    sa = wave_reduce_sum(okl ? sa : 0.f);
    sq = wave_reduce_sum(okl ? sq : 0.f);
    if (lane == 0) { part[(i * 8 + w) * 2] = sa; part[(i * 8 + w) * 2 + 1] = sq; }
  }
  __syncthreads();
  const int vrows = min(PB, L - l0);
  for (int i = tid; i < nb; i += 512) {
    float sa = 0.f, sq = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) {
      sa += part[(i * 8 + ww) * 2];
      sq += part[(i * 8 + ww) * 2 + 1];
    }
    const float m = sa / (float)(vrows * CH);
    st2[((size_t)(b0 + i) * TP + blockIdx.x) * 2] = m;
    st2[((size_t)(b0 + i) * TP + blockIdx.x) * 2 + 1] = fmaxf(sq - sa * m, 0.f);
  }
}

// ------------------------------------------------------------------------------------------------
// Per-sample constants for the LayerNorm-2 / local-MLP backward: one wave per sample combines the
// tile partials once (instead of every consumer workgroup doing it):
//   c[b] = (mean2, rstd2, m1_2, m2_2, mean1, rstd1, 0, 0)
__global__ void __launch_bounds__(256) ln2_consts_kernel(const float* __restrict__ st2, int T2, int BM2,
                                                         const float* __restrict__ sums2, int TS2,
                                                         const float* __restrict__ st1, int T1, int BM1,
                                                         float* __restrict__ consts, float* __restrict__ zero128,
                                                         int B, int L, float eps) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  // zero row b of the [B, 128] accumulator the LN1 finalize adds into (saves a fill launch per block)
  if (zero128 != nullptr)
    *reinterpret_cast<float2*>(zero128 + (size_t)b * CH + 2 * (threadIdx.x & 63)) = make_float2(0.f, 0.f);
  float mean2, rstd2, m1, m2, mean1, rstd1;
  wave_ln_stats(st2 + (size_t)b * T2 * 2, T2, BM2, L, CH, eps, mean2, rstd2);
  wave_bwd_consts(sums2 + (size_t)b * TS2 * 2, TS2, 1.0f / (float)(L * CH), m1, m2);
  wave_ln_stats(st1 + (size_t)b * T1 * 2, T1, BM1, L, CH, eps, mean1, rstd1);
  if ((threadIdx.x & 63) == 0) {
    float4* c = reinterpret_cast<float4*>(consts + (size_t)b * 8);
    c[0] = make_float4(mean2, rstd2, m1, m2);
    c[1] = make_float4(mean1, rstd1, 0.f, 0.f);
  }
}

// LayerNorm-2 backward + local MLP backward (input AND weight gradient) + LayerNorm-1 backward
// partials + both [L, C] affine gradients:
//   ds2 = rstd2 (dh2 g2 - m1 - xhat2 m2) ; dpre = ds2 GELU'(pre) ; dh1 = ds2 + Wl^T dpre
//   dWl += dpre^T h1 ; dbl += sum dpre ; dg2 += dh2 xhat2 ; db2 += dh2 ; dg1 += dh1 xhat1 ; db1 += dh1
// A workgroup owns a PAIR of positions (l0, l0 + 1) for a range of samples (grid (ceil(L/2), nsplit));
// an MFMA tile row is (sample, position) = (bc + j/2, l0 + j%2), 16 samples per tile.  The [L, C]
// affine gradients therefore accumulate in registers over every sample the workgroup sees and are
// written once (no cross-workgroup reduction when nsplit == 1); dWl sums 32 x nsamples rows per
// workgroup before its one atomic flush.  LN1 partials: sums1[b][pair][2].
// (Recomputing the MLP pre-activation here instead of reading the forward's pre_l measured slower.)
__global__ void __launch_bounds__(512) ln2_linear_bwd_kernel(
    const bf16_t* __restrict__ dh2, const bf16_t* __restrict__ s2, const float* __restrict__ g2,
    const bf16_t* __restrict__ pre_l, const bf16_t* __restrict__ s1,
    const float* __restrict__ g1, const float* __restrict__ be1, const bf16_t* __restrict__ wl,
    const float* __restrict__ consts,
    bf16_t* __restrict__ dh1, float* __restrict__ sums1, float* __restrict__ dg2, float* __restrict__ db2,
    float* __restrict__ dg1, float* __restrict__ db1, float* __restrict__ dwl, float* __restrict__ dbl,
    float* __restrict__ dwl_slab, float* __restrict__ dbl_slab, int B, int L) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;                                          // Wl, 32 KB
  unsigned char* dt = smem + 32768;                                  // dpre tile bf16 [32][128]
  unsigned char* ht = dt + 32 * 256;                                 // h1 tile bf16
  float* yt = reinterpret_cast<float*>(ht + 32 * 256);               // [32][YS] fp32
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int j = tid >> 4, ch = tid & 15;
  const int TS1 = (L + 1) / 2;                      // position pairs (LN1 partials per sample)
  const int nsplit = gridDim.y;
  const int b0 = (int)((long)B * blockIdx.y / nsplit), b1 = (int)((long)B * (blockIdx.y + 1) / nsplit);
  stage_weight(ws, wl, CH);
  float adbl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // dWl accumulators: wave w owns co tile (w >> 1) and ci tiles 2 (w & 1) + {0, 1}; they sum over every
  // pair the workgroup walks (long sequences: fewer workgroups than pairs, so fewer dWl flushes)
  f32x16_t aw0 = zero16(), aw1 = zero16();
  const int wco = (w >> 1) * 32, wci = (w & 1) * 64;
  for (int pair = blockIdx.x; pair < TS1; pair += gridDim.x) {
    const int l = pair * 2 + (j & 1);
    const bool okl = l < L;
    float ga2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ga1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bt1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (okl) {
      load_f8(g2 + (size_t)l * CH + ch * 8, ga2);
      load_f8(g1 + (size_t)l * CH + ch * 8, ga1);
      load_f8(be1 + (size_t)l * CH + ch * 8, bt1);
    }
    float adg2[8] = {0, 0, 0, 0, 0, 0, 0, 0}, adb2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float adg1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, adb1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const size_t coff = (size_t)l * CH + ch * 8;
    // prefetch the first chunk
    int bs = b0 + (j >> 1);
    bool ok = okl && bs < b1;
    size_t off = (size_t)bs * L * CH + coff;
    uint4 n_dh = ldq(dh2 + off, ok), n_s2 = ldq(s2 + off, ok), n_s1 = ldq(s1 + off, ok);
    uint4 n_pr = ldq(pre_l + off, ok);
    float4 n_c0 = make_float4(0.f, 1.f, 0.f, 0.f), n_c1 = make_float4(0.f, 1.f, 0.f, 0.f);
    if (bs < b1) {
      n_c0 = *reinterpret_cast<const float4*>(consts + (size_t)bs * 8);
      n_c1 = *reinterpret_cast<const float4*>(consts + (size_t)bs * 8 + 4);
    }
    for (int bc = b0; bc < b1; bc += 16) {
      const int bcur = bs;
      const bool okc = ok;
      const size_t offc = off;
      const float mean2 = n_c0.x, rstd2 = n_c0.y, m1 = n_c0.z, m2 = n_c0.w, mean1 = n_c1.x, rstd1 = n_c1.y;
      float dh[8], sv2[8], pr[8], sv1[8], ds2[8], dp[8], xh1[8], hv[8];
      unpack8(n_dh, dh);
      unpack8(n_s2, sv2);
      unpack8(n_s1, sv1);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh2 = (sv2[e] - mean2) * rstd2;
        adg2[e] += okc ? dh[e] * xh2 : 0.f;
        adb2[e] += okc ? dh[e] : 0.f;
        ds2[e] = okc ? rstd2 * (dh[e] * ga2[e] - m1 - xh2 * m2) : 0.f;
        xh1[e] = (sv1[e] - mean1) * rstd1;
        hv[e] = okc ? xh1[e] * ga1[e] + bt1[e] : 0.f;
      }
      *reinterpret_cast<uint4*>(ht + swz256(j, ch)) = packq8(hv);
      auto prefetch = [&]() {
        bs = bc + 16 + (j >> 1);
        ok = okl && bs < b1;
        off = (size_t)bs * L * CH + coff;
        n_dh = ldq(dh2 + off, ok);
        n_s2 = ldq(s2 + off, ok);
        n_pr = ldq(pre_l + off, ok);
        n_s1 = ldq(s1 + off, ok);
        if (bs < b1) {
          n_c0 = *reinterpret_cast<const float4*>(consts + (size_t)bs * 8);
          n_c1 = *reinterpret_cast<const float4*>(consts + (size_t)bs * 8 + 4);
        }
      };
      unpack8(n_pr, pr);
      float gp[8];
      {
        const f32x2 xi[4] = {(f32x2){pr[0], pr[1]}, (f32x2){pr[2], pr[3]}, (f32x2){pr[4], pr[5]},
                             (f32x2){pr[6], pr[7]}};
        f32x2 go[4];
        gelu2_fast_n<4, true>(xi, go);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gp[2 * e] = go[e].x;
          gp[2 * e + 1] = go[e].y;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) dp[e] = ds2[e] * gp[e];
      const uint4 dq = packq8(dp);
      *reinterpret_cast<uint4*>(dt + swz256(j, ch)) = dq;
      {
        float dpr[8];
        unpack8(dq, dpr);
#pragma unroll
        for (int e = 0; e < 8; ++e) adbl[e] += dpr[e];
      }
      __syncthreads();
      // prefetch the next chunk while the MFMAs run
      prefetch();
      if (w < 4) {
        // D[ci][row] = sum_co Wl[co][ci] dpre[row][co]: A = Wl^T (transposed LDS read), B = dpre rows
        f32x16_t acc = zero16();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const int rlo = kk * 16 + 8 * h + q;
          const int col = w * 32 + tc;
          const bf16x8 fa = cat_tr(lds_tr(ws, swz256e(rlo, col)), lds_tr(ws, swz256e(rlo + 4, col)));
          acc = mfma32(fa, lds_frag(dt, swz256(r, kk * 2 + h)), acc);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(yt + r * YS + w * 32 + 8 * g + 4 * h) =
              make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
      }
      // dWl[co][ci] += sum_row dpre[row][co] h1[row][ci]   (both operands transposed LDS reads)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int rlo = ks * 16 + 8 * h + q;
        const bf16x8 fa = cat_tr(lds_tr(dt, swz256e(rlo, wco + tc)), lds_tr(dt, swz256e(rlo + 4, wco + tc)));
        const bf16x8 fb0 = cat_tr(lds_tr(ht, swz256e(rlo, wci + tc)), lds_tr(ht, swz256e(rlo + 4, wci + tc)));
        const bf16x8 fb1 =
            cat_tr(lds_tr(ht, swz256e(rlo, wci + 32 + tc)), lds_tr(ht, swz256e(rlo + 4, wci + 32 + tc)));
        aw0 = mfma32(fa, fb0, aw0);
        aw1 = mfma32(fa, fb1, aw1);
      }
      __syncthreads();
      const float4 ya = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8);
      const float4 yb = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8 + 4);
      const float yv[8] = {ya.x, ya.y, ya.z, ya.w, yb.x, yb.y, yb.z, yb.w};
      float o[8], sa = 0.f, sc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = okc ? bfround(ds2[e] + yv[e]) : 0.f;
        const float dxh = o[e] * ga1[e];
        sa += dxh;
        sc += dxh * xh1[e];
        adg1[e] += o[e] * xh1[e];
        adb1[e] += o[e];
      }
      if (okc) *reinterpret_cast<uint4*>(dh1 + offc) = packq8(o);
      // LN1 partial of (sample, position pair): 16 lanes per row, rows j and j+1 share the sample
#pragma unroll
      for (int m = 1; m <= 16; m <<= 1) {
        sa += __shfl_xor(sa, m, 64);
        sc += __shfl_xor(sc, m, 64);
      }
      if ((lane & 31) == 0 && bcur < b1) {
        sums1[((size_t)bcur * TS1 + pair) * 2] = sa;
        sums1[((size_t)bcur * TS1 + pair) * 2 + 1] = sc;
      }
    }
    // [L, C] affine gradients: sum the 16 rows of each position through LDS, one add per element
    const int l0 = pair * 2;
    float* accs[4] = {adg2, adb2, adg1, adb1};
    float* dsts[4] = {dg2, db2, dg1, db1};
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) yt[j * CH + ch * 8 + e] = accs[a][e];
      __syncthreads();
      if (tid < 2 * CH) {
        const int par = tid >> 7, c = tid & (CH - 1);
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) v += yt[(2 * k + par) * CH + c];
        if (l0 + par < L) atomicAdd(dsts[a] + (size_t)(l0 + par) * CH + c, v);
      }
    }
    __syncthreads();                                // yt reads done before the next pair's MFMA writes
  }
  // local-MLP bias: column sums over all rows
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 8; ++e) yt[j * CH + ch * 8 + e] = adbl[e];
  __syncthreads();
  if (tid < CH) {
    float a = 0.f;
#pragma unroll 8
    for (int k = 0; k < 32; ++k) a += yt[k * CH + tid];
    // one slab row per workgroup (folded in a fixed order with dWl's slab) or one atomic
    if (dbl_slab != nullptr) dbl_slab[(size_t)(blockIdx.y * gridDim.x + blockIdx.x) * CH + tid] = a;
    else atomicAdd(dbl + tid, a);
  }
  // local-MLP weight: D[co][ci], lane -> ci (128 contiguous bytes per half-wave).  dwl_slab: this
  // workgroup's partial goes to its own slab row (folded by one column-sum pass) instead of 16 K float
  // atomics on the same 16 K addresses from every workgroup
  float* dw = dwl_slab != nullptr ? dwl_slab + (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * CH * CH : dwl;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int co = wco + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (dwl_slab != nullptr) {
      dw[(size_t)co * CH + wci + r] = aw0[i];
      dw[(size_t)co * CH + wci + 32 + r] = aw1[i];
    } else {
      atomicAdd(dw + (size_t)co * CH + wci + r, aw0[i]);
      atomicAdd(dw + (size_t)co * CH + wci + 32 + r, aw1[i]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// LayerNorm-1 backward finalize: ds1 = rstd1 (dh1 g1 - m1 - xhat1 m2) and dgb[b][c] = sum_l ds1
// (gradient of the broadcast global->local vector, reference modules.py:208-211).
// grid (ceil(L/PB), nbg), 512 threads, same (position, chunk) ownership.
__global__ void __launch_bounds__(512) ln1_finalize_kernel(
    const bf16_t* __restrict__ dh1, const bf16_t* __restrict__ s1, const float* __restrict__ st1, int T1, int BM1,
    const float* __restrict__ sums1, int TS1, const float* __restrict__ g1, bf16_t* __restrict__ ds1,
    float* __restrict__ dgb, int B, int L, float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* red = reinterpret_cast<float*>(smem);            // 2 x [PB][CH] (double-buffered)
  float* tab = red + 2 * PB * CH;                          // [nb][4]: mean rstd m1 m2
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j = tid >> 4, ch = tid & 15;
  const int nbg = gridDim.y;
  const int b0 = (int)((long)B * blockIdx.y / nbg), b1 = (int)((long)B * (blockIdx.y + 1) / nbg);
  const int nb = b1 - b0;
  float* dacc = tab + 4 * nb;                              // [nb][CH] dgb partial over the walked tiles
  const float inv_n = 1.0f / (float)(L * CH);
  for (int i = w; i < nb; i += 8) {
    float mean, rstd, m1, m2;
    wave_ln_stats(st1 + (size_t)(b0 + i) * T1 * 2, T1, BM1, L, CH, eps, mean, rstd);
    wave_bwd_consts(sums1 + (size_t)(b0 + i) * TS1 * 2, TS1, inv_n, m1, m2);
    if (lane == 0) { tab[4 * i] = mean; tab[4 * i + 1] = rstd; tab[4 * i + 2] = m1; tab[4 * i + 3] = m2; }
  }
  for (int i = tid; i < nb * CH; i += 512) dacc[i] = 0.f;
  // a workgroup walks position tiles blockIdx.x, + gridDim.x, ... (long sequences): its dgb partial
  // sums them in LDS and is flushed once (one atomic per (sample, channel) and workgroup)
  const int TP = (L + PB - 1) / PB;
  int it = 0;                                              // red double-buffer parity across tiles
  for (int px = blockIdx.x; px < TP; px += gridDim.x) {
    const int l = px * PB + j;
    const bool okl = l < L;
    float ga[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (okl) load_f8(g1 + (size_t)l * CH + ch * 8, ga);
    // loads from a clamped valid row (masked at use): a select on the load becomes a branch around
    // it, and the wait for it a vmcnt(0)
    const size_t coff = (size_t)min(l, L - 1) * CH + ch * 8;
    uint4 n_dh = *reinterpret_cast<const uint4*>(dh1 + (size_t)min(b0, B - 1) * L * CH + coff);
    uint4 n_s = *reinterpret_cast<const uint4*>(s1 + (size_t)min(b0, B - 1) * L * CH + coff);
    __syncthreads();
    for (int b = b0; b < b1; ++b, ++it) {
      const float* tb = tab + 4 * (b - b0);
      const float mean = tb[0], rstd = tb[1], m1 = tb[2], m2 = tb[3];
      float* rb = red + (it & 1) * PB * CH;
      float dv[8], sv[8], o[8];
      unpack8(n_dh, dv);
      unpack8(n_s, sv);
      const size_t noff = (size_t)min(b + 1, B - 1) * L * CH + coff;
      n_dh = *reinterpret_cast<const uint4*>(dh1 + noff);
      n_s = *reinterpret_cast<const uint4*>(s1 + noff);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = okl ? rstd * (dv[e] * ga[e] - m1 - (sv[e] - mean) * rstd * m2) : 0.f;
      const uint4 qv = packq8(o);
      if (okl) *reinterpret_cast<uint4*>(ds1 + (size_t)b * L * CH + (size_t)l * CH + ch * 8) = qv;
      // dgb column sums: the wave's 4 rows by shuffles, one [128] partial per wave, 8 adds per channel
      unpack8(qv, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] += __shfl_xor(o[e], 16, 64);
        o[e] += __shfl_xor(o[e], 32, 64);
      }
      if (lane < 16) {
        *reinterpret_cast<float4*>(rb + w * CH + ch * 8) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(rb + w * CH + ch * 8 + 4) = make_float4(o[4], o[5], o[6], o[7]);
      }
      __syncthreads();   // (double buffer: the next sample writes the other half)
      if (tid < CH) {
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) a += rb[k * CH + tid];
        dacc[(b - b0) * CH + tid] += a;
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < nb * CH; i += 512) atomicAdd(dgb + (size_t)(b0 + i / CH) * CH + i % CH, dacc[i]);
}

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

// Embedding backward as a one-hot GEMM on MFMA: dE[v][c] = sum_rows [tok[row] == v] dout[row][c].
// A workgroup (4 waves) reduces a contiguous run of rows in 256-row tiles: the dout tile is staged
// in LDS (swz256) and read transposed as the B operand, the one-hot A operand is built in registers
// from the staged tokens, wave w owns channels 32w..32w+31; one atomic flush of [V][128] per
// workgroup.  (The previous LDS-atomic scatter serialised on the 26 hot token rows.)
// dE: accumulated with one atomic per (token, channel) and workgroup, or (slab != nullptr, the
// deterministic mode) this workgroup's [V][128] partial goes to slab row blockIdx.x (folded in a fixed
// order by the caller)
// DPRE (the first block's fold, pbx_embed_dpre): dout is that block's dS1 (the residual part of the
// embedding gradient) and the staging pass also writes the conv pre-activation gradients
// dpre_c = dS1 * GELU'(pre_c) of both convolutions (the products conv_dgrad4 would stage, bitwise)
template <bool DPRE>
__global__ void __launch_bounds__(256) embed_bwd_kernel(const long long* __restrict__ tok,
                                                        const bf16_t* __restrict__ dout, float* __restrict__ dE,
                                                        long rows, int V, float* __restrict__ slab,
                                                        const bf16_t* __restrict__ gdn, const bf16_t* __restrict__ gdw,
                                                        bf16_t* __restrict__ dpn, bf16_t* __restrict__ dpw) {
  __shared__ __attribute__((aligned(16))) unsigned char ds[256 * 256];
  __shared__ int ts[256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const long per = (rows + gridDim.x - 1) / gridDim.x;
  const long r0 = (long)blockIdx.x * per, r1 = min(rows, r0 + per);
  f32x16_t acc = zero16();
  for (long t0 = r0; t0 < r1; t0 += 256) {
    const int n = (int)min((long)256, r1 - t0);
    __syncthreads();
    if constexpr (DPRE) {
      // 4 chunks x (dS1, GELU'_n, GELU'_w) in flight per thread
      for (int base = tid; base < 256 * 16; base += 4 * 256) {
        uint4 gq[4], nq[4], wq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int idx = base + i * 256, row = idx >> 4;
          const size_t off = (size_t)(t0 + min(row, n - 1)) * CH + (idx & 15) * 8;
          gq[i] = *reinterpret_cast<const uint4*>(dout + off);
          nq[i] = *reinterpret_cast<const uint4*>(gdn + off);
          wq[i] = *reinterpret_cast<const uint4*>(gdw + off);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int idx = base + i * 256, row = idx >> 4;
          const bool ok = row < n;
          *reinterpret_cast<uint4*>(ds + swz256(row, idx & 15)) = ok ? gq[i] : make_uint4(0u, 0u, 0u, 0u);
          if (ok) {
            float g[8], pn[8], pw[8], on[8], ow[8];
            unpack8(gq[i], g);
            unpack8(nq[i], pn);
            unpack8(wq[i], pw);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              on[e] = pn[e] * g[e];
              ow[e] = pw[e] * g[e];
            }
            const size_t off = (size_t)(t0 + row) * CH + (idx & 15) * 8;
            *reinterpret_cast<uint4*>(dpn + off) = packq8(on);
            *reinterpret_cast<uint4*>(dpw + off) = packq8(ow);
          }
        }
      }
    } else {
      stage_chunks(
          256 * 16,
          [&](int idx) {
            const int row = idx >> 4;
            return row < n ? *reinterpret_cast<const uint4*>(dout + (t0 + row) * CH + (idx & 15) * 8)
                           : make_uint4(0u, 0u, 0u, 0u);
          },
          [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(ds + swz256(idx >> 4, idx & 15)) = v; });
    }
    ts[tid] = tid < n ? (int)tok[t0 + tid] : -1;
    __syncthreads();
    const int colb = w * 32 + tc;
#pragma unroll 4
    for (int kb = 0; kb < 16; ++kb) {
      // A[i = v][k = row]: lane's v = r, rows kb*16 + 8h + j
      typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
      u16x8 oh;
#pragma unroll
      for (int j = 0; j < 8; ++j) oh[j] = ts[kb * 16 + 8 * h + j] == r ? (unsigned short)0x3F80 : (unsigned short)0;
      const int rb = kb * 16 + 8 * h + q;
      const bf16x8 fb = cat_tr(lds_tr(ds, swz256e(rb, colb)), lds_tr(ds, swz256e(rb + 4, colb)));
      acc = mfma32(__builtin_bit_cast(bf16x8, oh), fb, acc);
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int v = (i & 3) + 8 * (i >> 2) + 4 * h;
    if (slab != nullptr) {
      if (v < V) slab[((size_t)blockIdx.x * V + v) * CH + w * 32 + r] = acc[i];
    } else if (v < V && acc[i] != 0.f) {
      atomicAdd(dE + v * CH + w * 32 + r, acc[i]);
    }
  }
}

int g_cus = -1;
int num_cus() {
  if (g_cus < 0) {
    int dev = 0;
    g_cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, dev) == hipSuccess) g_cus = p.multiProcessorCount;
    }
  }
  return g_cus;
}
// persistent grid: at most `per_cu` workgroups per CU, never more than the tile count
int persistent_grid(int tiles, int per_cu) {
  const int cap = num_cus() * per_cu;
  return tiles < cap ? (tiles > 0 ? tiles : 1) : cap;
}
}  // namespace

extern "C" int pbx_colsum_add(const float* src, int rows, int cols, float* dst, const float* scale, hipStream_t st);

static bool ln_attrs_set = false;
static void set_ln_attrs() {
  if (ln_attrs_set) return;
  (void)hipFuncSetAttribute((const void*)ln_linear_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)ln2_linear_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)ln1_finalize_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  ln_attrs_set = true;
}

static int ln_groups(int B, int L) {
  const int tp = (L + PB - 1) / PB;
  int g = (2 * num_cus() + tp - 1) / tp;          // ~2 workgroups of 8 waves per CU
  return g < 1 ? 1 : (g > B ? B : g);
}

// pre_l (nullable): the MLP pre-activation for the backward (inference forwards skip it)
PBX_EXPORT int pbx_ln_linear_fwd(const void* s1, const float* st1, int T1, int BM1, const float* g1,
                                 const float* be1, const void* wl, const float* bl, void* pre_l, void* s2,
                                 float* st2, int B, int L, float eps, hipStream_t st) {
  dim3 grid((L + PB - 1) / PB, ln_groups(B, L));
  const int nbmax = (B + (int)grid.y - 1) / (int)grid.y;
  const int lds = 32768 + PB * 256 + PB * YS * 4 + nbmax * 18 * 4;
  if (lds > 163840) return (int)hipErrorInvalidValue;
  set_ln_attrs();
  hipLaunchKernelGGL(ln_linear_fwd_kernel, grid, dim3(512), lds, st, (const bf16_t*)s1, st1, T1, BM1, g1, be1,
                     (const bf16_t*)wl, bl, (bf16_t*)pre_l, (bf16_t*)s2, st2, B, L, eps);
  return pbx_launch_status();
}

// dg2/db2/dg1/db1 ([L, C]), dwl ([128, 128]) and dbl ([128]) fp32 are accumulated into.
// consts: [B][8] fp32 workspace; sums1: [B][ceil(L/2)][2] LN1 partials (TS1 = ceil(L/2)).
// dwl_slab (nullable): [slab_rows][128 * 128 + 128] scratch for per-workgroup dWl / dbl partials (else
// atomics).  det: one workgroup per position pair for every sample (the [L, C] affine gradients then
// have a single writer each) -- with the slab the whole kernel is run-to-run deterministic.
// grid of ln2_linear_bwd_kernel: (position-pair groups, sample splits)
static void ln2_bwd_grid(int B, int L, int det, int& gx, int& nsplit) {
  const int pairs = (L + 1) / 2;
  const int target = num_cus();
  nsplit = (target + pairs - 1) / pairs;            // at least one workgroup per CU
  if (nsplit > (B + 15) / 16) nsplit = (B + 15) / 16;
  if (nsplit < 1 || det) nsplit = 1;
  // long sequences: one workgroup walks several position pairs (its dWl partial is flushed once; at
  // L = 4096 one workgroup per pair made 33 M float atomics on the 16 K dWl elements)
  gx = pairs < target ? pairs : target;
}

// slab rows (workgroups) the dWl / dbl partials of pbx_ln2_linear_bwd occupy
PBX_EXPORT int pbx_ln2_bwd_slab_rows(int B, int L, int det) {
  int gx, nsplit;
  ln2_bwd_grid(B, L, det, gx, nsplit);
  return gx * nsplit;
}

// fold: 1 = the dWl / dbl slab partials are summed into dwl / dbl here (same stream); 0 = the caller
// folds them later (pbx_colsum_add over pbx_ln2_bwd_slab_rows rows, e.g. on the weight-gradient stream)
PBX_EXPORT int pbx_ln2_linear_bwd(const void* dh2, const void* s2, const float* st2, const float* sums2, int TS2,
                                  const float* g2, const void* pre_l, const void* s1, const float* st1, int T1,
                                  int BM1, const float* g1, const float* be1, const void* wl, float* consts,
                                  void* dh1, float* sums1, float* dg2, float* db2, float* dg1, float* db1, float* dwl,
                                  float* dbl, float* dgb_zero, int B, int L, float eps, float* dwl_slab, int slab_rows,
                                  int det, int fold, int consts_ready, hipStream_t st) {
  set_ln_attrs();
  const int T2 = (L + PB - 1) / PB;
  // consts_ready: the caller already wrote consts and zeroed dgb_zero
  if (!consts_ready)
    hipLaunchKernelGGL(ln2_consts_kernel, dim3((B + 3) / 4), dim3(256), 0, st, st2, T2, PB, sums2, TS2, st1, T1, BM1,
                       consts, dgb_zero, B, L, eps);
  int gx, nsplit;
  ln2_bwd_grid(B, L, det, gx, nsplit);
  const int lds = 32768 + 2 * 32 * 256 + 32 * YS * 4;
  // dWl partials: one slab row per workgroup when the caller's slab is large enough, else atomics
  const int nwg = gx * nsplit;
  float* slab = dwl_slab != nullptr && nwg <= slab_rows ? dwl_slab : nullptr;
  float* bslab = slab != nullptr ? slab + (size_t)slab_rows * CH * CH : nullptr;    // [slab_rows][128] after dWl's
  if ((det || !fold) && slab == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ln2_linear_bwd_kernel, dim3(gx, nsplit), dim3(512), lds, st, (const bf16_t*)dh2,
                     (const bf16_t*)s2, g2, (const bf16_t*)pre_l, (const bf16_t*)s1, g1, be1, (const bf16_t*)wl,
                     consts, (bf16_t*)dh1, sums1, dg2, db2, dg1, db1, dwl, dbl, slab, bslab, B, L);
  if (slab != nullptr && fold) {
    int rc = pbx_launch_status();
    if (rc != 0) return rc;
    rc = pbx_colsum_add(slab, nwg, CH * CH, dwl, nullptr, st);
    if (rc != 0) return rc;
    return pbx_colsum_add(bslab, nwg, CH, dbl, nullptr, st);
  }
  return pbx_launch_status();
}

// dgb ([B, 128] fp32) is accumulated into
// det: one workgroup walks every position tile of its samples (dgb then has a single writer per row)
PBX_EXPORT int pbx_ln1_finalize(const void* dh1, const void* s1, const float* st1, int T1, int BM1,
                                const float* sums1, int TS1, const float* g1, void* ds1, float* dgb, int B, int L,
                                float eps, int det, hipStream_t st) {
  // at most 16 position tiles across x (a workgroup walks the rest), ~2 workgroups per CU overall
  const int tp = (L + PB - 1) / PB;
  const int gx = det ? 1 : (tp < 16 ? tp : 16);
  int gy = (2 * num_cus() + gx - 1) / gx;
  gy = gy < 1 ? 1 : (gy > B ? B : gy);
  dim3 grid(gx, gy);
  const int nbmax = (B + (int)grid.y - 1) / (int)grid.y;
  const int lds = 2 * PB * CH * 4 + nbmax * 16 + nbmax * CH * 4;
  if (lds > 163840) return (int)hipErrorInvalidValue;
  set_ln_attrs();
  hipLaunchKernelGGL(ln1_finalize_kernel, grid, dim3(512), lds, st, (const bf16_t*)dh1, (const bf16_t*)s1, st1, T1,
                     BM1, sums1, TS1, g1, (bf16_t*)ds1, dgb, B, L, eps);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_embed_fwd(const void* tok, const float* E, void* out, long rows, hipStream_t st) {
  const long n = rows * 16;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const long long*)tok, E,
                     (bf16_t*)out, rows);
  return pbx_launch_status();
}

// number of workgroups (= slab rows of the deterministic form) pbx_embed_bwd uses
PBX_EXPORT int pbx_embed_bwd_groups(long rows) {
  long g = (rows + 511) / 512;
  if (g > 2 * num_cus()) g = 2 * num_cus();
  return g < 1 ? 1 : (int)g;
}

// slab (nullable): [pbx_embed_bwd_groups(rows)][V][128] fp32 -> deterministic fixed-order fold into dE
PBX_EXPORT int pbx_embed_bwd(const void* tok, const void* dout, float* dE, long rows, int V, float* slab,
                             hipStream_t st) {
  if (V > 32) return (int)hipErrorInvalidValue;
  const int g = pbx_embed_bwd_groups(rows);
  hipLaunchKernelGGL(embed_bwd_kernel<false>, dim3((unsigned)g), dim3(256), 0, st, (const long long*)tok,
                     (const bf16_t*)dout, dE, rows, V, slab, nullptr, nullptr, nullptr, nullptr);
  if (slab != nullptr) {
    const int rc = pbx_launch_status();
    if (rc != 0) return rc;
    return pbx_colsum_add(slab, g, V * CH, dE, nullptr, st);
  }
  return pbx_launch_status();
}

// The first block's backward without its conv data gradient (reference modules.py:249-253,300: the
// block input is the embedding, so dE = sum_{tok} dx, dx = dS1 + conv^T(dpre); the conv^T part is
// E-space and added by pbx_wgrad_tok from its one-hot sums): dE += sum_{rows : tok = v} dS1[row] and
// dpre_n / dpre_w = dS1 * GELU'(pre) for the weight gradient, one pass over dS1.  Same slab contract
// as pbx_embed_bwd.
PBX_EXPORT int pbx_embed_dpre(const void* tok, const void* ds1, const void* gdn, const void* gdw, void* dpn, void* dpw,
                              float* dE, long rows, int V, float* slab, hipStream_t st) {
  if (V > 32 || rows < 1) return (int)hipErrorInvalidValue;
  const int g = pbx_embed_bwd_groups(rows);
  hipLaunchKernelGGL(embed_bwd_kernel<true>, dim3((unsigned)g), dim3(256), 0, st, (const long long*)tok,
                     (const bf16_t*)ds1, dE, rows, V, slab, (const bf16_t*)gdn, (const bf16_t*)gdw, (bf16_t*)dpn,
                     (bf16_t*)dpw);
  if (slab != nullptr) {
    const int rc = pbx_launch_status();
    if (rc != 0) return rc;
    return pbx_colsum_add(slab, g, V * CH, dE, nullptr, st);
  }
  return pbx_launch_status();
}
