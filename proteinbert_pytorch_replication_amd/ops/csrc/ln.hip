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
__device__ __forceinline__ void load_f4(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}

// One 1-KiB global->LDS DMA wave instruction (lane i's 16 source bytes land at lds_base + 16 i), as
// inline asm so hipcc does not make later ds_reads wait for it (see wgrad.hip); it retires in vmcnt
// order with the wave's other vector-memory operations.
__device__ __forceinline__ void glds16_ln(const void* src, unsigned char* lds_base) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}

// stage a [rows x 128] bf16 weight matrix into a swz256 LDS image (whole workgroup)
__device__ __forceinline__ void stage_weight(unsigned char* dst, const bf16_t* __restrict__ w, int rows) {
  stage_chunks(
      rows * 16, [&](int idx) { return *reinterpret_cast<const uint4*>(w + (size_t)idx * 8); },
      [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(dst + swz256(idx >> 4, idx & 15)) = v; });
}

// LN-normalised B/A fragment of one position row: 8 x (8 channels kk*16 + 8h .. +8)
// The caller passes in-bounds pointers (rows clamped); `ok` only masks the values, so every load is
// unconditional and all 24 of them are in flight together (a load under a divergent branch costs
// one exposed memory round trip per branch).
// KB: channel chunks whose loads are in flight together (8: one round trip, ~160 VGPRs of operands;
// 4: two round trips at half the registers, for the high-occupancy pool variant)
template <int KB = 8>
__device__ __forceinline__ void ln_row_frags(bf16x8* f, const bf16_t* __restrict__ src, const float* __restrict__ gam,
                                             const float* __restrict__ bet, float mean, float rstd, bool ok,
                                             int h, bf16_t* __restrict__ out) {
#pragma unroll
  for (int k0 = 0; k0 < 8; k0 += KB) {
  uint4 sq[KB];
  float4 ga[KB][2], ba[KB][2];
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int ci = (k0 + k) * 16 + 8 * h;
    sq[k] = *reinterpret_cast<const uint4*>(src + ci);
#ifdef PBX_ABL_NOAFFINE   // ablation builds only: the cost of the [L, C] affine loads
    ga[k][0] = ga[k][1] = ba[k][0] = ba[k][1] = make_float4(mean, rstd, mean, rstd);
#else
    ga[k][0] = *reinterpret_cast<const float4*>(gam + ci);
    ga[k][1] = *reinterpret_cast<const float4*>(gam + ci + 4);
    ba[k][0] = *reinterpret_cast<const float4*>(bet + ci);
    ba[k][1] = *reinterpret_cast<const float4*>(bet + ci + 4);
#endif
  }
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int kk = k0 + k;
    const int ci = kk * 16 + 8 * h;
    float sv[8], v[8];
    unpack8(sq[k], sv);
    const float g[8] = {ga[k][0].x, ga[k][0].y, ga[k][0].z, ga[k][0].w,
                        ga[k][1].x, ga[k][1].y, ga[k][1].z, ga[k][1].w};
    const float be[8] = {ba[k][0].x, ba[k][0].y, ba[k][0].z, ba[k][0].w,
                         ba[k][1].x, ba[k][1].y, ba[k][1].z, ba[k][1].w};
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = ok ? (sv[e] - mean) * rstd * g[e] + be[e] : 0.f;
    const uint4 q = packq8(v);
#ifdef PBX_ABL_NOH2   // ablation builds only: the cost of the h2 stores
    if (ok && out != nullptr && mean > 1e30f) *reinterpret_cast<uint4*>(out + ci) = q;
#else
    if (ok && out != nullptr) *reinterpret_cast<uint4*>(out + ci) = q;
#endif
    f[kk] = __builtin_bit_cast(bf16x8, q);
  }
  }
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
// h2 = LN(s2) (written: block output) ; vpart[b][t][j] = sum_{pos in 64-row tile t} GELU(h2[pos] . Wv[j])
// Work item = 64 positions of one sample, owned by one wave (waves are independent: no barrier after
// the Wv staging).  Each Wv fragment read from LDS feeds two MFMAs (the wave's two 32-row position
// tiles), the two accumulator chains are interleaved, and the 8 Wv fragments of column block jt+1
// are loaded while block jt runs, so neither LDS latency nor MFMA dependency stalls the wave; the
// packed-fp32 GELU / column sums of block jt-1 fill the MFMA shadow.
__global__ void __launch_bounds__(512) ln_attn_fwd_kernel(
    const bf16_t* __restrict__ s2, const float* __restrict__ st2, const float* __restrict__ g2,
    const float* __restrict__ be2, const bf16_t* __restrict__ wv, bf16_t* __restrict__ h2,
    float* __restrict__ vpart, int B, int L, int NJ, float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;                                          // NJ rows x 256 B
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int NW = blockDim.x >> 6;
  const int T2 = (L + BML - 1) / BML;
  const int TW = (L + 63) / 64;
  const int NJT = NJ / 32;
  const long items = (long)B * TW;
  stage_weight(ws, wv, NJ);
  __syncthreads();
  for (long item = (long)blockIdx.x * NW + w; item < items; item += (long)gridDim.x * NW) {
    const int b = (int)(item / TW), tw = (int)(item - (item / TW) * TW);
    const int pos0 = tw * 64;
    float mean, rstd;
    wave_ln_stats(st2 + (size_t)b * T2 * 2, T2, BML, L, CH, eps, mean, rstd);
    bf16x8 hf0[8], hf1[8];
    {
      const int pa = pos0 + r, pb = pos0 + 32 + r;
      const int ca = min(pa, L - 1), cb = min(pb, L - 1);          // clamped: loads stay in bounds
      const size_t ra = ((size_t)b * L + ca) * CH, rb = ((size_t)b * L + cb) * CH;
      ln_row_frags(hf0, s2 + ra, g2 + (size_t)ca * CH, be2 + (size_t)ca * CH, mean, rstd, pa < L, h, h2 + ra);
      ln_row_frags(hf1, s2 + rb, g2 + (size_t)cb * CH, be2 + (size_t)cb * CH, mean, rstd, pb < L, h, h2 + rb);
    }
    float* vrow = vpart + ((size_t)b * TW + tw) * NJ;
    // rows beyond L are zero fragments (ln_row_frags) and GELU(0) = 0: no masking needed
    auto colsum = [&](const f32x16_t& c0, const f32x16_t& c1, int jt) {
      f32x2 sv = {0.f, 0.f};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x2 xv[4] = {(f32x2){c0[4 * g], c0[4 * g + 1]}, (f32x2){c0[4 * g + 2], c0[4 * g + 3]},
                             (f32x2){c1[4 * g], c1[4 * g + 1]}, (f32x2){c1[4 * g + 2], c1[4 * g + 3]}};
        f32x2 gv[4];
        gelu2_fast_n<4, false>(xv, gv);
        sv += (gv[0] + gv[1]) + (gv[2] + gv[3]);
      }
      float sacc = sv.x + sv.y;
      sacc += __shfl_xor(sacc, 32, 64);
      if (h == 0) vrow[jt * 32 + r] = sacc;
    };
    bf16x8 wf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) wf[kk] = lds_frag(ws, swz256(r, kk * 2 + h));
    f32x16_t p0 = zero16(), p1 = zero16();
    for (int jt = 0; jt < NJT; ++jt) {
      f32x16_t c0 = zero16(), c1 = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        c0 = mfma32(hf0[kk], wf[kk], c0);
        c1 = mfma32(hf1[kk], wf[kk], c1);
      }
      if (jt + 1 < NJT) {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) wf[kk] = lds_frag(ws, swz256((jt + 1) * 32 + r, kk * 2 + h));
      }
      if (jt > 0) colsum(p0, p1, jt - 1);
      p0 = c0;
      p1 = c1;
    }
    colsum(p0, p1, NJT - 1);
  }
}

// ------------------------------------------------------------------------------------------------
// h2 = LN_(L,C)(s2) as a streaming position-major pass (the pattern of ln_linear_fwd): a workgroup
// owns PB = 32 positions, keeps their fp32 affine in registers (thread: position j, 8 channels) and
// walks its sample group with AP samples' rows in flight per thread.  The pool forward then reads the
// normalised rows directly.
constexpr int AP = 4;
__global__ void __launch_bounds__(512) ln2_apply_kernel(const bf16_t* __restrict__ s2, const float* __restrict__ st2,
                                                        const float* __restrict__ g2, const float* __restrict__ be2,
                                                        bf16_t* __restrict__ h2, int B, int L, float eps) {
  __shared__ float tab[2 * 256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j = tid >> 4, ch = tid & 15;
  const int l = blockIdx.x * PB + j;
  const bool okl = l < L;
  const int T2 = (L + BML - 1) / BML;
  const int nbg = gridDim.y;
  const int b0 = (int)((long)B * blockIdx.y / nbg), b1 = (int)((long)B * (blockIdx.y + 1) / nbg);
  const int nb = b1 - b0;                          // <= 256 (host: nbg >= ceil(B / 256))
  for (int i = w; i < nb; i += 8) {
    float mean, rstd;
    wave_ln_stats(st2 + (size_t)(b0 + i) * T2 * 2, T2, BML, L, CH, eps, mean, rstd);
    if (lane == 0) {
      tab[2 * i] = mean;
      tab[2 * i + 1] = rstd;
    }
  }
  float gam[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bet[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (okl) {
    load_f8(g2 + (size_t)l * CH + ch * 8, gam);
    load_f8(be2 + (size_t)l * CH + ch * 8, bet);
  }
  __syncthreads();
  if (!okl) return;
  const size_t col = (size_t)l * CH + ch * 8;
  for (int bb = b0; bb < b1; bb += AP) {
    uint4 q[AP];
#pragma unroll
    for (int k = 0; k < AP; ++k) q[k] = ldq(s2 + (size_t)min(bb + k, b1 - 1) * L * CH + col, true);
#pragma unroll
    for (int k = 0; k < AP; ++k) {
      if (bb + k >= b1) break;
      const float mean = tab[2 * (bb + k - b0)], rstd = tab[2 * (bb + k - b0) + 1];
      float sv[8], o[8];
      unpack8(q[k], sv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (sv[e] - mean) * rstd * gam[e] + bet[e];
      *reinterpret_cast<uint4*>(h2 + (size_t)(bb + k) * L * CH + col) = packq8(o);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Attention pool with the GELU derivative stored by the forward (v2).
//
// The backward of the pool needs GELU'(h2 Wv) at every (position, value column): recomputing it costs
// the [32 x 512] projection per tile (128 MFMAs) plus GELU' (2 transcendentals per element), all to
// multiply it by dv (the round-1 form; 1.6 % slower on the step).  Here the forward evaluates GELU and GELU' from ONE shared
// erf/exp core, column-sums GELU as before and writes GELU' as bf16 in the exact per-lane order of
// the backward's MFMA B operand (`gfrag`: [B][2 ceil(L/64)][NJ/32][2][64 lanes][8], one coalesced
// 1-KB store / load per wave-instruction); the backward is then 128 MFMAs per 32-position tile fed
// by a streamed, prefetched load, with no recompute and no transcendental.
//
// Fragment order (backward MFMA k-step (jt, s), lane (r = position, h), element jj):
//   j = jt*32 + 16 s + 8 (jj >> 2) + 4 h + (jj & 3)        (= the A-operand rows of the Wv^T reads)
// The forward holds D[pos][j] (lane = column j, 16 positions in registers, so the column sums stay
// in-lane); each 32x32 block of GELU' goes through a per-wave LDS tile Gt[j][pos] (ds_write_b64 of
// 4 contiguous positions) and comes back transposed (ds_read_b64_tr_b16) as two fragments.
constexpr int GT_STRIDE = 72;       // bytes per Gt row (32 positions + 8 B pad: spreads the banks)
constexpr int GT_BYTES = 32 * GT_STRIDE;

#ifdef PBX_STAMPS   // instrumented builds only (tools/ubench/build_flags.sh st -DPBX_STAMPS): per-phase clocks
__device__ long long* pbx_stamp_buf;
#define PBX_STAMP(k)                                                                       \
  do {                                                                                     \
    if (blockIdx.x < 4 && lane == 0 && (k) < 64)                                           \
      pbx_stamp_buf[(blockIdx.x * 8 + w) * 64 + (k)] = (long long)clock64();               \
  } while (0)
#else
#define PBX_STAMP(k) do {} while (0)
#endif

// Work item: 64 positions (two 32-position MFMA tiles; each Wv fragment read from LDS feeds two MFMAs;
// ~248 VGPRs, two waves per SIMD).  NI: GELU pairs interleaved per core call.
// PRENORM: s2 already holds the normalised rows (h2 from ln2_apply_kernel); no statistics, no affine
// loads and no h2 stores (the [L, C] fp32 affine re-read per 64-position item cost ~35 us of ~175)
template <int NWAVE, int NI, bool PRENORM, bool STOREG = true>   // STOREG: GELU' fragments for attn_bwd2
__global__ void __launch_bounds__(64 * NWAVE) ln_attn_fwd2_kernel(
    const bf16_t* __restrict__ s2, const float* __restrict__ st2, const float* __restrict__ g2,
    const float* __restrict__ be2, const bf16_t* __restrict__ wv, bf16_t* __restrict__ h2,
    float* __restrict__ vpart, bf16x8* __restrict__ gfrag, int B, int L, int NJ, float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;                                          // NJ rows x 256 B
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  unsigned char* gt = smem + NJ * 256 + w * GT_BYTES;               // this wave's transpose tile
  const int NW = blockDim.x >> 6;
  const int T2 = (L + BML - 1) / BML;
  const int TW64 = (L + 63) / 64;
  const int TW = TW64;                              // work items per sample
  constexpr int NP = 2;                             // 32-position MFMA tiles per work item
  const int NJT = NJ / 32;
  const long items = (long)B * TW;
  PBX_STAMP(0);
  stage_weight(ws, wv, NJ);
  __syncthreads();
#ifdef PBX_DESYNC   // experiment builds: the second wave of each SIMD starts PBX_DESYNC x 8k cycles late
  if (w >= 4)
    for (int i = 0; i < PBX_DESYNC; ++i) __builtin_amdgcn_s_sleep(127);
#endif
  PBX_STAMP(1);
  int sb = 2;
  for (long item = (long)blockIdx.x * NW + w; item < items; item += (long)gridDim.x * NW, sb += 20) {
    const int b = (int)(item / TW), tw = (int)(item - (item / TW) * TW);
    const int pos0 = tw * 32 * NP;
    PBX_STAMP(sb);
    bf16x8 hf0[8], hf1[8];
    if constexpr (PRENORM) {
      const int pa = pos0 + r, pb = pos0 + 32 + r;
      const bf16_t* ra = s2 + ((size_t)b * L + min(pa, L - 1)) * CH + 8 * h;
      const bf16_t* rb = s2 + ((size_t)b * L + min(pb, L - 1)) * CH + 8 * h;
      uint4 qa[8], qb[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        qa[kk] = *reinterpret_cast<const uint4*>(ra + kk * 16);
        qb[kk] = *reinterpret_cast<const uint4*>(rb + kk * 16);
      }
      const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        hf0[kk] = __builtin_bit_cast(bf16x8, pa < L ? qa[kk] : z);
        hf1[kk] = __builtin_bit_cast(bf16x8, pb < L ? qb[kk] : z);
      }
      PBX_STAMP(sb + 1);
    } else {
      float mean, rstd;
      wave_ln_stats(st2 + (size_t)b * T2 * 2, T2, BML, L, CH, eps, mean, rstd);
      PBX_STAMP(sb + 1);
      const int pa = pos0 + r;
      const int ca = min(pa, L - 1);
      const size_t ra = ((size_t)b * L + ca) * CH;
      ln_row_frags(hf0, s2 + ra, g2 + (size_t)ca * CH, be2 + (size_t)ca * CH, mean, rstd, pa < L, h, h2 + ra);
      const int pb = pos0 + 32 + r;
      const int cb = min(pb, L - 1);
      const size_t rb = ((size_t)b * L + cb) * CH;
      ln_row_frags(hf1, s2 + rb, g2 + (size_t)cb * CH, be2 + (size_t)cb * CH, mean, rstd, pb < L, h, h2 + rb);
    }
    PBX_STAMP(sb + 2);
    float* vrow = vpart + ((size_t)b * TW + tw) * NJ;
    // fragment base of this item's 32-position tiles: [b][2 ceil(L/64)][jt][s][lane]
    bf16x8* gdst = gfrag + ((size_t)b * 2 * TW64 + NP * tw) * NJT * 2 * 64 + lane;
    auto epi = [&](const f32x16_t& c0, const f32x16_t& c1, int jt) {
      f32x2 sv = {0.f, 0.f};
      if constexpr (!STOREG) {
        // GELU only (the backward recomputes GELU', attn_bwd3)
        constexpr int NPAIR = 8 * NP;
#pragma unroll
        for (int c8 = 0; c8 < NPAIR; c8 += NI) {
          f32x2 xv[NI], gv[NI];
#pragma unroll
          for (int k = 0; k < NI; ++k) {
            const int pi = c8 + k;
            const f32x16_t& c = (pi >> 3) ? c1 : c0;
            xv[k] = (f32x2){c[2 * (pi & 7)], c[2 * (pi & 7) + 1]};
          }
          gelu2_fast_n<NI, false>(xv, gv);
#pragma unroll
          for (int k = 0; k < NI; ++k) sv += gv[k];
        }
        float sacc = sv.x + sv.y;
        sacc += __shfl_xor(sacc, 32, 64);
        if (h == 0) vrow[jt * 32 + r] = sacc;
        return;
      }
      // GELU / GELU' of the item's 32x32 tiles: NI pairs per interleaved core call
      constexpr int NPAIR = 8 * NP;
      f32x2 gdall[NPAIR];
#pragma unroll
      for (int c8 = 0; c8 < NPAIR; c8 += NI) {
        f32x2 xv[NI], gv[NI], gd[NI];
#pragma unroll
        for (int k = 0; k < NI; ++k) {
          const int pi = c8 + k;                  // pair index 0..15: tile pi >> 3, values 2 (pi & 7) ..
          const f32x16_t& c = (pi >> 3) ? c1 : c0;
          xv[k] = (f32x2){c[2 * (pi & 7)], c[2 * (pi & 7) + 1]};
        }
        gelu2_both_n<NI>(xv, gv, gd);
#pragma unroll
        for (int k = 0; k < NI; ++k) {
          sv += gv[k];
          gdall[c8 + k] = gd[k];
        }
      }
#pragma unroll
      for (int pt = 0; pt < NP; ++pt) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          // positions 8g + 4h .. +3 of column j = r -> Gt[r][8g + 4h]
          const f32x2 a = gdall[pt * 8 + 2 * g], bq = gdall[pt * 8 + 2 * g + 1];
          uint2 pk;
          pk.x = (unsigned)f2bf(a.x) | ((unsigned)f2bf(a.y) << 16);
          pk.y = (unsigned)f2bf(bq.x) | ((unsigned)f2bf(bq.y) << 16);
          *reinterpret_cast<uint2*>(gt + r * GT_STRIDE + (8 * g + 4 * h) * 2) = pk;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int rlo = 16 * s + 4 * h + q;
          const bf16x8 f = cat_tr(lds_tr(gt, rlo * GT_STRIDE + tc * 2), lds_tr(gt, (rlo + 8) * GT_STRIDE + tc * 2));
#ifdef PBX_ABL_NOGSTORE   // ablation builds only: the cost of the GELU' fragment stores (B > 0 always)
          if (B < 0)
#endif
          gdst[((size_t)pt * NJT * 2 + jt * 2 + s) * 64] = f;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      float sacc = sv.x + sv.y;
      sacc += __shfl_xor(sacc, 32, 64);
      if (h == 0) vrow[jt * 32 + r] = sacc;
    };
    bf16x8 wf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) wf[kk] = lds_frag(ws, swz256(r, kk * 2 + h));
    f32x16_t p0 = zero16(), p1 = zero16();
    for (int jt = 0; jt < NJT; ++jt) {
      f32x16_t c0 = zero16(), c1 = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        c0 = mfma32(hf0[kk], wf[kk], c0);
        c1 = mfma32(hf1[kk], wf[kk], c1);
      }
      if (jt + 1 < NJT) {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) wf[kk] = lds_frag(ws, swz256((jt + 1) * 32 + r, kk * 2 + h));
      }
      if (jt > 0) epi(p0, p1, jt - 1);
      p0 = c0;
      p1 = c1;
      PBX_STAMP(sb + 3 + jt);
    }
    epi(p0, p1, NJT - 1);
    PBX_STAMP(sb + 19);
  }
}

// attention pool backward from the stored GELU' fragments + LayerNorm-2 backward partials:
//   dh2[pos][ci] = dh2_in + sum_j Wv[j][ci] dv[b][j] GELU'[pos][j]
// Work item = one 32-position tile, one wave per SIMD (4 waves, <= 512 registers).  Every load of an
// item is issued at its start, in the order the wave consumes them (vmcnt retires in issue order):
// the dv row, all 2 NJT GELU' fragments of the tile (one coalesced 1-KiB load each, ~32 KiB in
// flight per wave), then the epilogue operands; no load is outstanding across the item loop's back
// edge, so the compiler's waits stay exact.
// FIXTW: the grid stride is a multiple of the tiles per sample, so every item of a wave has the same
// 32 positions and their [L, C] affine gamma is loaded once per wave, not per item (~16 of ~72 KB per
// item; the compiler's vmcnt tracking wants the item loads branch-free, hence a template flag)
template <int NJT, bool FIXTW>
__global__ void __launch_bounds__(256) attn_bwd2_kernel(
    const bf16x8* __restrict__ gfrag, const bf16_t* __restrict__ s2, const float* __restrict__ st2,
    const float* __restrict__ g2, const bf16_t* __restrict__ dh2_in, const float* __restrict__ dvpart, int BMV,
    const bf16_t* __restrict__ wv, bf16_t* __restrict__ dh2, float* __restrict__ sums2, int B, int L, float eps) {
  constexpr int NJ = NJT * 32;
  constexpr int NF = 2 * NJT;                       // fragments (k-steps) per 32-position tile
  constexpr int NDV = NJ / 256;                     // 1-KiB DMA instructions per dv row
  constexpr int NW = 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int T2 = (L + BML - 1) / BML;
  const int TW = (L + 31) / 32;
  const int TWG = 2 * ((L + 63) / 64);              // 32-position tiles per sample in gfrag
  const int TV = (L + BMV - 1) / BMV;
  const long items = (long)B * TW;
  const long stride = (long)gridDim.x * NW;
  stage_weight(ws, wv, NJ);
  // per-wave dv rows, double-buffered: item k reads slot k & 1; the DMA of item k+1's row into the
  // other slot is issued with item k's epilogue operands (whose waits retire it)
  unsigned char* dvslot = ws + NJ * 256 + w * 2 * NJ * 4;
  int woff[4], woff8[4];   // Wv^T fragment offsets at step 0; step i adds 16 i rows = 4096 i bytes
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    woff[ct] = swz256e(4 * h + q, ct * 32 + tc);
    woff8[ct] = swz256e(4 * h + q + 8, ct * 32 + tc);
  }
  auto dv_src = [&](long it) {
    const int b = (int)(it / TW), tw = (int)(it - (it / TW) * TW);
    return dvpart + ((size_t)b * TV + (tw * 32) / BMV) * NJ;
  };
  long item = (long)blockIdx.x * NW + w;
  float4 gq4[4][4];
  if constexpr (FIXTW) {
    const int pc = min((int)(item % TW) * 32 + r, L - 1);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) gq4[ct][i] = *reinterpret_cast<const float4*>(g2 + (size_t)pc * CH + ct * 32 + 8 * i + 4 * h);
  }
  if (item < items) {
    const float* dvg = dv_src(item);
#pragma unroll
    for (int k = 0; k < NDV; ++k) glds16_ln(dvg + lane * 4 + 256 * k, dvslot + 1024 * k);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  int slot = 0;
  for (; item < items; item += stride, slot ^= 1) {
    const int b = (int)(item / TW), tw = (int)(item - (item / TW) * TW);
    const int pos = tw * 32 + r;
    const bool okb = pos < L;
    const bf16x8* gsrc = gfrag + ((size_t)b * TWG + tw) * NF * 64 + lane;
    const float* dv = reinterpret_cast<const float*>(dvslot + slot * NJ * 4);
    const bool has_next = item + stride < items;
    const float* dvn = dv_src(has_next ? item + stride : item);
    bf16x8 ring[NF];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      ring[i] = gsrc[i * 64];
      __builtin_amdgcn_sched_barrier(0);      // keep the issue order = the consumption order
    }
    const int pc = min(pos, L - 1);
    const size_t roff = ((size_t)b * L + pc) * CH;
    // branch-free loads (a load under a branch makes the compiler's vmcnt tracking fall back to
    // vmcnt(0) at the merge): a missing dh2_in reads s2 and is masked
    const bf16_t* dsrc = dh2_in != nullptr ? dh2_in : s2;
    const float dmask = dh2_in != nullptr ? 1.f : 0.f;
    const float* stb = st2 + (size_t)b * T2 * 2;
    uint2 dq[4][4], sq[4][4];
    float2 pm0, pm1;
    // the epilogue operands are issued EPI steps before the end of the tile: vmcnt counts at most 63
    // outstanding operations per wave (2 + 2 NJT ring + 50 would overflow it if issued up front)
    auto epi_loads = [&]() {
      if (has_next) {
#pragma unroll
        for (int k = 0; k < NDV; ++k) glds16_ln(dvn + lane * 4 + 256 * k, dvslot + (slot ^ 1) * NJ * 4 + 1024 * k);
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ci0 = ct * 32 + 8 * i + 4 * h;
          dq[ct][i] = *reinterpret_cast<const uint2*>(dsrc + roff + ci0);
          sq[ct][i] = *reinterpret_cast<const uint2*>(s2 + roff + ci0);
          if constexpr (!FIXTW) gq4[ct][i] = *reinterpret_cast<const float4*>(g2 + (size_t)pc * CH + ci0);
        }
      pm0 = *reinterpret_cast<const float2*>(stb + 2 * min(lane, T2 - 1));
      pm1 = *reinterpret_cast<const float2*>(stb + 2 * min(lane + 64, T2 - 1));
    };
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    f32x16_t y[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) y[ct] = zero16();
    constexpr int EPI = NF < 8 ? NF : 8;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      if (i == NF - EPI) {
        __builtin_amdgcn_sched_barrier(0);
        epi_loads();
        __builtin_amdgcn_sched_barrier(0);
      }
      float dvv[8], gv[8];
      load_f4(dv + 16 * i + 4 * h, dvv);            // j = jt*32 + 16 s (= 16 i) + 4 h + ...
      load_f4(dv + 16 * i + 8 + 4 * h, dvv + 4);
      unpack8(__builtin_bit_cast(uint4, ring[i]), gv);
#pragma unroll
      for (int e = 0; e < 8; ++e) gv[e] *= dvv[e];
      const bf16x8 fb = pack8(gv);
      const unsigned char* wsi = ws + 4096 * i;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const bf16x8 fw = cat_tr(lds_tr(wsi, woff[ct]), lds_tr(wsi, woff8[ct]));
        y[ct] = mfma32(fw, fb, y[ct]);
      }
    }
    // LN2 statistics of sample b (Chan merge of the tile partials; T2 <= 128 from the early loads)
    float mean, rstd;
    if (T2 <= 128) {
      float n = 0.f, m = 0.f, M2 = 0.f;
      if (lane < T2) chan_merge(n, m, M2, (float)(min(BML, L - lane * BML) * CH), pm0.x, pm0.y);
      if (lane + 64 < T2) chan_merge(n, m, M2, (float)(min(BML, L - (lane + 64) * BML) * CH), pm1.x, pm1.y);
      wave_chan(n, m, M2);
      mean = m;
      rstd = rsqrtf(M2 / n + eps);
    } else {
      wave_ln_stats(stb, T2, BML, L, CH, eps, mean, rstd);
    }
    float sa = 0.f, sc = 0.f;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ci0 = ct * 32 + 8 * g + 4 * h;
        float din[4], sv[4], o[4];
        unpack4(dq[ct][g], din);
        unpack4(sq[ct][g], sv);
        const float gg[4] = {gq4[ct][g].x, gq4[ct][g].y, gq4[ct][g].z, gq4[ct][g].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = bfround(fmaf(din[e], dmask, y[ct][4 * g + e]));
          const float xh = (sv[e] - mean) * rstd;
          const float dxh = o[e] * gg[e];
          sa += okb ? dxh : 0.f;
          sc += okb ? dxh * xh : 0.f;
        }
        if (okb) *reinterpret_cast<uint2*>(dh2 + roff + ci0) = packq4(o);
      }
    }
    sa = wave_reduce_sum(sa);
    sc = wave_reduce_sum(sc);
    if (lane == 0) {
      sums2[((size_t)b * TW + tw) * 2] = sa;
      sums2[((size_t)b * TW + tw) * 2 + 1] = sc;
    }
  }
}

// attention pool backward that RECOMPUTES GELU'(h2 Wv) instead of streaming the stored fragments
// (268 MB per block at B = L = 512, the dominant traffic of attn_bwd2):
//   zT[j][pos]  = sum_c Wv[j][c] h2[pos][c]      MFMA, A = Wv rows (LDS), B = the tile's h2 rows (registers)
//   uT[j][pos]  = dv[b][j] GELU'(zT[j][pos])     VALU on the 16 accumulator values of each lane
//   dh^T[c][pos] += sum_j Wv[j][c] uT[j][pos]    MFMA, A = Wv^T read transposed from LDS
// The D layout of zT (lane = position, rows 4h + {0..3, 8..11} + 16 s of a 32-row chunk) is the B
// operand of the second product with its K order permuted to {4h + 0..3, 8 + 4h + 0..3} per 16-step,
// which is exactly the order the transposed Wv reads of attn_bwd2 deliver: no data movement between
// the two MFMAs.  The GELU' of chunk jt runs while the MFMAs of chunk jt + 1's zT are in flight.
// Epilogue (dh2 = bf16(dh2_in + dh), LN2 partials) as attn_bwd2.  One wave per SIMD.
template <int NJT, bool FIXTW, int NW>
__global__ void __launch_bounds__(64 * NW) attn_bwd3_kernel(
    const bf16_t* __restrict__ h2, const bf16_t* __restrict__ s2, const float* __restrict__ st2,
    const float* __restrict__ g2, const bf16_t* __restrict__ dh2_in, const float* __restrict__ dvpart, int BMV,
    const bf16_t* __restrict__ wv, bf16_t* __restrict__ dh2, float* __restrict__ sums2, int B, int L, float eps) {
  constexpr int NJ = NJT * 32;
  constexpr int NDV = NJ / 256;                     // 1-KiB DMA instructions per dv row
  // NW = 4: one wave per SIMD, every load of an item issued up front; NW = 8: two waves per SIMD sharing
  // one Wv image (LDS 128 + 32 KB), the epilogue operands loaded after the MFMA / GELU' body (<= 256
  // registers a wave) -- the other wave's VALU / MFMA work covers that latency
  constexpr bool EARLY = NW == 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int T2 = (L + BML - 1) / BML;
  const int TW = (L + 31) / 32;
  const int TV = (L + BMV - 1) / BMV;
  const long items = (long)B * TW;
  const long stride = (long)gridDim.x * NW;
  stage_weight(ws, wv, NJ);
  unsigned char* dvslot = ws + NJ * 256 + w * 2 * NJ * 4;
  int woff[4], woff8[4];   // Wv^T fragment offsets at 16-step 0; step i adds 16 i rows = 4096 i bytes
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    woff[ct] = swz256e(4 * h + q, ct * 32 + tc);
    woff8[ct] = swz256e(4 * h + q + 8, ct * 32 + tc);
  }
  auto dv_src = [&](long it) {
    const int b = (int)(it / TW), tw = (int)(it - (it / TW) * TW);
    return dvpart + ((size_t)b * TV + (tw * 32) / BMV) * NJ;
  };
  long item = (long)blockIdx.x * NW + w;
  float4 gq4[4][4];
  if constexpr (FIXTW) {
    const int pc = min((int)(item % TW) * 32 + r, L - 1);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) gq4[ct][i] = *reinterpret_cast<const float4*>(g2 + (size_t)pc * CH + ct * 32 + 8 * i + 4 * h);
  }
  if (item < items) {
    const float* dvg = dv_src(item);
#pragma unroll
    for (int k = 0; k < NDV; ++k) glds16_ln(dvg + lane * 4 + 256 * k, dvslot + 1024 * k);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  int slot = 0;
  for (; item < items; item += stride, slot ^= 1) {
    const int b = (int)(item / TW), tw = (int)(item - (item / TW) * TW);
    const int pos = tw * 32 + r;
    const bool okb = pos < L;
    const float* dv = reinterpret_cast<const float*>(dvslot + slot * NJ * 4);
    const bool has_next = item + stride < items;
    const float* dvn = dv_src(has_next ? item + stride : item);
    const int pc = min(pos, L - 1);
    const size_t roff = ((size_t)b * L + pc) * CH;
    // the tile's h2 rows as B fragments (lane: position r, channels 16 kk + 8 h ..), issued first
    uint4 hq[8];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) hq[kk] = *reinterpret_cast<const uint4*>(h2 + roff + kk * 16 + 8 * h);
    __builtin_amdgcn_sched_barrier(0);
    const bf16_t* dsrc = dh2_in != nullptr ? dh2_in : s2;
    const float dmask = dh2_in != nullptr ? 1.f : 0.f;
    const float* stb = st2 + (size_t)b * T2 * 2;
    uint2 dq[4][4], sq[4][4];
    float2 pm0, pm1;
    // epilogue operands and the next item's dv row
    auto epi_loads = [&]() {
      if (has_next) {
#pragma unroll
        for (int k = 0; k < NDV; ++k) glds16_ln(dvn + lane * 4 + 256 * k, dvslot + (slot ^ 1) * NJ * 4 + 1024 * k);
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ci0 = ct * 32 + 8 * i + 4 * h;
          dq[ct][i] = *reinterpret_cast<const uint2*>(dsrc + roff + ci0);
          sq[ct][i] = *reinterpret_cast<const uint2*>(s2 + roff + ci0);
          if constexpr (!FIXTW) gq4[ct][i] = *reinterpret_cast<const float4*>(g2 + (size_t)pc * CH + ci0);
        }
      pm0 = *reinterpret_cast<const float2*>(stb + 2 * min(lane, T2 - 1));
      pm1 = *reinterpret_cast<const float2*>(stb + 2 * min(lane + 64, T2 - 1));
    };
    if constexpr (EARLY) epi_loads();   // in flight during the whole MFMA / GELU' body
    bf16x8 hf[8];
    const uint4 zq = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) hf[kk] = __builtin_bit_cast(bf16x8, okb ? hq[kk] : zq);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    f32x16_t y[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) y[ct] = zero16();
    auto zchunk = [&](int jt) {
      f32x16_t z = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) z = mfma32(lds_frag(ws, swz256(jt * 32 + r, kk * 2 + h)), hf[kk], z);
      return z;
    };
    f32x16_t zc = zchunk(0);
#pragma unroll EARLY ? 2 : 1
    for (int jt = 0; jt < NJT; ++jt) {
      f32x16_t zn = zc;
      if (jt + 1 < NJT) zn = zchunk(jt + 1);          // in flight during this chunk's GELU'
      f32x2 xv[8], gd[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = (f32x2){zc[2 * i], zc[2 * i + 1]};
      gelu2_fast_n<8, true>(xv, gd);
      // reg 4g + e <-> j = 32 jt + 8 g + 4 h + e
      float u[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 d4 = *reinterpret_cast<const float4*>(dv + jt * 32 + 8 * g + 4 * h);
        u[4 * g] = gd[2 * g].x * d4.x;
        u[4 * g + 1] = gd[2 * g].y * d4.y;
        u[4 * g + 2] = gd[2 * g + 1].x * d4.z;
        u[4 * g + 3] = gd[2 * g + 1].y * d4.w;
      }
      const bf16x8 b0 = pack8(u), b1 = pack8(u + 8);
#pragma unroll
      for (int sidx = 0; sidx < 2; ++sidx) {
        const unsigned char* wsi = ws + 4096 * (2 * jt + sidx);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const bf16x8 fw = cat_tr(lds_tr(wsi, woff[ct]), lds_tr(wsi, woff8[ct]));
          y[ct] = mfma32(fw, sidx ? b1 : b0, y[ct]);
        }
      }
      zc = zn;
    }
    if constexpr (!EARLY) epi_loads();
    // LN2 statistics of sample b (Chan merge of the tile partials; T2 <= 128 from the early loads)
    float mean, rstd;
    if (T2 <= 128) {
      float n = 0.f, m = 0.f, M2 = 0.f;
      if (lane < T2) chan_merge(n, m, M2, (float)(min(BML, L - lane * BML) * CH), pm0.x, pm0.y);
      if (lane + 64 < T2) chan_merge(n, m, M2, (float)(min(BML, L - (lane + 64) * BML) * CH), pm1.x, pm1.y);
      wave_chan(n, m, M2);
      mean = m;
      rstd = rsqrtf(M2 / n + eps);
    } else {
      wave_ln_stats(stb, T2, BML, L, CH, eps, mean, rstd);
    }
    float sa = 0.f, sc = 0.f;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ci0 = ct * 32 + 8 * g + 4 * h;
        float din[4], sv[4], o[4];
        unpack4(dq[ct][g], din);
        unpack4(sq[ct][g], sv);
        const float gg[4] = {gq4[ct][g].x, gq4[ct][g].y, gq4[ct][g].z, gq4[ct][g].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = bfround(fmaf(din[e], dmask, y[ct][4 * g + e]));
          const float xh = (sv[e] - mean) * rstd;
          const float dxh = o[e] * gg[e];
          sa += okb ? dxh : 0.f;
          sc += okb ? dxh * xh : 0.f;
        }
        if (okb) *reinterpret_cast<uint2*>(dh2 + roff + ci0) = packq4(o);
      }
    }
    sa = wave_reduce_sum(sa);
    sc = wave_reduce_sum(sc);
    if (lane == 0) {
      sums2[((size_t)b * TW + tw) * 2] = sa;
      sums2[((size_t)b * TW + tw) * 2 + 1] = sc;
    }
    // the next item's dv row (DMA issued above) must be in LDS before its first read
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
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
  (void)hipFuncSetAttribute((const void*)ln_attn_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)ln_linear_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)ln_attn_fwd2_kernel<8, 4, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)ln_attn_fwd2_kernel<8, 4, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd2_kernel<16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd2_kernel<16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd2_kernel<8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd2_kernel<8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<16, true, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<16, false, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<8, true, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<8, false, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<16, false, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<8, false, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)ln_attn_fwd2_kernel<8, 4, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
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

// nw: waves per workgroup; vpart is [B][ceil(L / 64)][NJ] (one row per 64-position wave tile)
PBX_EXPORT int pbx_ln_attn_fwd(const void* s2, const float* st2, const float* g2, const float* be2, const void* wv,
                               void* h2, float* vpart, int B, int L, int NJ, int nw, float eps, hipStream_t st) {
  set_ln_attrs();
  if (NJ % 64 != 0 || NJ * 256 > 163840 || nw < 1 || nw > 8) return (int)hipErrorInvalidValue;
  const long items = (long)B * ((L + 63) / 64);
  long wgl = (items + nw - 1) / nw;
  if (wgl > num_cus()) wgl = num_cus();
  hipLaunchKernelGGL(ln_attn_fwd_kernel, dim3((int)wgl), dim3(64 * nw), NJ * 256, st, (const bf16_t*)s2, st2, g2, be2,
                     (const bf16_t*)wv, (bf16_t*)h2, vpart, B, L, NJ, eps);
  return pbx_launch_status();
}

// dvpart rows follow the forward tiling (bmv positions, a multiple of 32); sums2 is [B][ceil(L / 32)][2]
// v2 pool: also writes gfrag (bf16 GELU' fragments, B * 2 ceil(L/64) * NJ * 32 elements).  8 waves per
// workgroup (two per SIMD), 4 GELU pairs per interleaved core call; measured against 4 waves x 8 / 16
// pairs and 12 waves of 32-position items (profiles/r2_v8_pool_32pos_ab.txt): equal or slower.
#ifdef PBX_STAMPS
PBX_EXPORT int pbx_set_stamps(long long* buf) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(pbx_stamp_buf), &buf, sizeof(buf));
}
#endif

PBX_EXPORT int pbx_ln_attn_fwd2(const void* s2, const float* st2, const float* g2, const float* be2, const void* wv,
                                void* h2, float* vpart, void* gfrag, int B, int L, int NJ, float eps, int prenorm,
                                hipStream_t st) {
  set_ln_attrs();
  constexpr int nw = 8;
  if (NJ % 64 != 0 || NJ * 256 + nw * GT_BYTES > 163840) return (int)hipErrorInvalidValue;
  if (!prenorm && gfrag == nullptr) return (int)hipErrorInvalidValue;   // the GELU-only form reads h2 rows
  const long items2 = (long)B * ((L + 63) / 64);
  long wg2 = (items2 + nw - 1) / nw;
  if (wg2 > num_cus()) wg2 = num_cus();
  if (prenorm) {
    // h2 = LN(s2) first (streaming pass), then the pool on the normalised rows
    const int tp = (L + PB - 1) / PB;
    int nbg = (2 * num_cus() + tp - 1) / tp;
    nbg = max(nbg, (B + 255) / 256);
    nbg = min(nbg, B);
    hipLaunchKernelGGL(ln2_apply_kernel, dim3(tp, nbg), dim3(512), 0, st, (const bf16_t*)s2, st2, g2, be2,
                       (bf16_t*)h2, B, L, eps);
    if (gfrag != nullptr)
      hipLaunchKernelGGL((ln_attn_fwd2_kernel<nw, 4, true>), dim3((int)wg2), dim3(64 * nw), NJ * 256 + nw * GT_BYTES,
                         st, (const bf16_t*)h2, st2, g2, be2, (const bf16_t*)wv, (bf16_t*)h2, vpart, (bf16x8*)gfrag,
                         B, L, NJ, eps);
    else   // the backward recomputes GELU' (attn_bwd3): GELU column sums only
      hipLaunchKernelGGL((ln_attn_fwd2_kernel<nw, 4, true, false>), dim3((int)wg2), dim3(64 * nw),
                         NJ * 256 + nw * GT_BYTES, st, (const bf16_t*)h2, st2, g2, be2, (const bf16_t*)wv,
                         (bf16_t*)h2, vpart, (bf16x8*)nullptr, B, L, NJ, eps);
  } else {
    hipLaunchKernelGGL((ln_attn_fwd2_kernel<nw, 4, false>), dim3((int)wg2), dim3(64 * nw), NJ * 256 + nw * GT_BYTES,
                       st, (const bf16_t*)s2, st2, g2, be2, (const bf16_t*)wv, (bf16_t*)h2, vpart, (bf16x8*)gfrag,
                       B, L, NJ, eps);
  }
  return pbx_launch_status();
}

// v2 pool backward (NJ = 256 or 512): reads gfrag instead of recomputing h2 Wv
PBX_EXPORT int pbx_attn_bwd2(const void* gfrag, const void* s2, const float* st2, const float* g2,
                             const void* dh2_in, const float* dvpart, int bmv, const void* wv, void* dh2,
                             float* sums2, int B, int L, int NJ, float eps, hipStream_t st) {
  set_ln_attrs();
  const int nw = 4;
  if ((NJ != 256 && NJ != 512) || bmv % 32 != 0) return (int)hipErrorInvalidValue;
  const long items = (long)B * ((L + 31) / 32);
  long wgl = (items + nw - 1) / nw;
  if (wgl > num_cus()) wgl = num_cus();
  const int lds = NJ * 256 + nw * 2 * NJ * 4;
  const bool fix = ((wgl * nw) % ((L + 31) / 32)) == 0;
  const auto kern = NJ == 512 ? (fix ? attn_bwd2_kernel<16, true> : attn_bwd2_kernel<16, false>)
                              : (fix ? attn_bwd2_kernel<8, true> : attn_bwd2_kernel<8, false>);
  hipLaunchKernelGGL(kern, dim3((int)wgl), dim3(64 * nw), lds, st,
                     (const bf16x8*)gfrag, (const bf16_t*)s2, st2, g2, (const bf16_t*)dh2_in, dvpart, bmv,
                     (const bf16_t*)wv, (bf16_t*)dh2, sums2, B, L, eps);
  return pbx_launch_status();
}

// recomputing pool backward (NJ = 256 or 512): h2 = the block output rows the forward pool read
PBX_EXPORT int pbx_attn_bwd3(const void* h2, const void* s2, const float* st2, const float* g2, const void* dh2_in,
                             const float* dvpart, int bmv, const void* wv, void* dh2, float* sums2, int B, int L,
                             int NJ, float eps, int wide, hipStream_t st) {
  set_ln_attrs();
  const int nw = wide ? 8 : 4;
  if ((NJ != 256 && NJ != 512) || bmv % 32 != 0) return (int)hipErrorInvalidValue;
  const long items = (long)B * ((L + 31) / 32);
  long wgl = (items + nw - 1) / nw;
  if (wgl > num_cus()) wgl = num_cus();
  const int lds = NJ * 256 + nw * 2 * NJ * 4;
  const bool fix = ((wgl * nw) % ((L + 31) / 32)) == 0;
  decltype(&attn_bwd3_kernel<16, true, 4>) kern;
  if (wide)   // two waves per SIMD: the gamma rows are loaded per item (no FIXTW registers)
    kern = NJ == 512 ? attn_bwd3_kernel<16, false, 8> : attn_bwd3_kernel<8, false, 8>;
  else
    kern = NJ == 512 ? (fix ? attn_bwd3_kernel<16, true, 4> : attn_bwd3_kernel<16, false, 4>)
                     : (fix ? attn_bwd3_kernel<8, true, 4> : attn_bwd3_kernel<8, false, 4>);
  hipLaunchKernelGGL(kern, dim3((int)wgl), dim3(64 * nw), lds, st, (const bf16_t*)h2, (const bf16_t*)s2, st2, g2,
                     (const bf16_t*)dh2_in, dvpart, bmv, (const bf16_t*)wv, (bf16_t*)dh2, sums2, B, L, eps);
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
  // consts_ready: the pool backward (pbx_attn_bwd4c) already wrote consts and zeroed dgb_zero
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
