// MFMA / LDS building blocks shared by the pbx CDNA4 kernels (gfx950, wave64).
//
// Every GEMM-shaped piece of ProteinBERT uses v_mfma_f32_32x32x16_bf16 with
// bf16 operands and fp32 accumulation.  Operand fragments (per lane: 8 bf16
// along K) come from LDS tiles whose rows are 256 B (128 bf16 channels) and are
// XOR-swizzled on 16-B chunks so that BOTH access kinds are conflict-free:
//   * row reads  (ds_read_b128: lane = row, 16 B of K)            -> GEMM with K along channels
//   * transposed reads (ds_read_b64_tr_b16: lane = column, 4 rows) -> GEMM with K along positions
// (chunk' = chunk ^ ((row&3)<<2 | (row>>2)&3): rows 0..15 map to 16 distinct chunks, and any 4
// consecutive rows land on 4 distinct 64-B groups).
//
// Fragment maps for mfma_f32_32x32x16_bf16 (lane l, r = l&31, h = l>>5):
//   A[i=r][k = 8h + j], B[k = 8h + j][col = r], j = 0..7
//   D[row = (reg&3) + 8*(reg>>2) + 4h][col = r], reg = 0..15
#pragma once
#include "common.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;

namespace pbx {

__device__ __forceinline__ f32x16_t mfma32(const bf16x8& a, const bf16x8& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16_t zero16() {
  f32x16_t z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// byte offset of 16-B chunk `chunk` (0..15) of row `row` in a 256-B-row swizzled tile
__device__ __forceinline__ int swz256(int row, int chunk) {
  return (row << 8) + ((chunk ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}
// byte offset of bf16 element `col` (0..127) of row `row`
__device__ __forceinline__ int swz256e(int row, int col) {
  return swz256(row, col >> 3) + ((col & 7) << 1);
}
// 128-B rows (64 bf16), row reads only: rows 0..15 of a 16-lane group hit 16 distinct bank slots
__device__ __forceinline__ int swz128(int row, int chunk) {
  return (row << 7) + ((chunk ^ ((row >> 1) & 7)) << 4);
}

__device__ __forceinline__ bf16x8 lds_frag(const unsigned char* base, int byte_off) {
  return *reinterpret_cast<const bf16x8*>(base + byte_off);
}

// Transposed fragment: element q (q=0..3) of the result = tile[rowA + q][col] where col is this
// lane's column; elements 4..7 come from rows rowB + q.  The caller passes, per lane, the rows and
// column its 16-lane group needs (see tr_rows/tr_col below).
__device__ __forceinline__ s16x4 lds_tr(const unsigned char* base, int byte_off) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + byte_off));
}

__device__ __forceinline__ bf16x8 cat_tr(const s16x4& lo, const s16x4& hi) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// For ds_read_b64_tr_b16 in a 32x32x16 operand: lane l of 16-lane group g = l>>4 supplies
// row (q = (l>>2)&3) and column block 4*(l&3) + 16*(g&1); it receives column (l&31) of those rows.
__device__ __forceinline__ int tr_q(int lane) { return (lane >> 2) & 3; }
__device__ __forceinline__ int tr_c(int lane) { return ((lane & 3) << 2) + (((lane >> 4) & 1) << 4); }

// 8 fp32 -> bf16x8 (RNE)
__device__ __forceinline__ bf16x8 pack8(const float* v) {
  typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
  u16x8 u;
#pragma unroll
  for (int i = 0; i < 8; ++i) u[i] = f2bf(v[i]);
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ void unpack8(const uint4& q, float* v) {
  v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
  v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  v[4] = __uint_as_float(q.z << 16); v[5] = __uint_as_float(q.z & 0xffff0000u);
  v[6] = __uint_as_float(q.w << 16); v[7] = __uint_as_float(q.w & 0xffff0000u);
}
__device__ __forceinline__ void unpack4(const uint2& q, float* v) {
  v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
  v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
}
__device__ __forceinline__ uint4 packq8(const float* v) {
  uint4 q;
  q.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
  q.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
  q.z = (unsigned)f2bf(v[4]) | ((unsigned)f2bf(v[5]) << 16);
  q.w = (unsigned)f2bf(v[6]) | ((unsigned)f2bf(v[7]) << 16);
  return q;
}
__device__ __forceinline__ uint2 packq4(const float* v) {
  uint2 q;
  q.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
  q.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
  return q;
}
__device__ __forceinline__ float bfround(float f) { return bf2f(f2bf(f)); }

// Block-wide sum over `nw` waves through an LDS scratch of >= nw floats. All threads get the sum.
__device__ __forceinline__ float block_sum(float v, float* scratch, int nw) {
  v = wave_reduce_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += scratch[i];
  return s;
}

// Whole-sequence LayerNorm statistics from per-tile (mean, M2) partials (Chan et al. combine).
// Tile t of a sample covers min(BM, L - t*BM) rows x C channels.
__device__ __forceinline__ void ln_stats(const float* __restrict__ part, int T, int BM, int L, int C, float eps,
                                         float& mean, float& rstd) {
  float n = 0.f, m = 0.f, M2 = 0.f;
  for (int t = 0; t < T; ++t) {
    const float nt = (float)(min(BM, L - t * BM) * C);
    const float mt = part[2 * t], M2t = part[2 * t + 1];
    const float nn = n + nt;
    const float d = mt - m;
    m += d * (nt / nn);
    M2 += M2t + d * d * (n * nt / nn);
    n = nn;
  }
  mean = m;
  rstd = rsqrtf(M2 / n + eps);
}

// LayerNorm-backward per-sample constants from per-tile (sum dxhat, sum dxhat*xhat) partials.
__device__ __forceinline__ void ln_bwd_consts(const float* __restrict__ part, int T, float inv_n, float& m1,
                                              float& m2) {
  float a = 0.f, c = 0.f;
  for (int t = 0; t < T; ++t) { a += part[2 * t]; c += part[2 * t + 1]; }
  m1 = a * inv_n;
  m2 = c * inv_n;
}

// Global -> LDS staging of n 16-byte chunks with up to 8 loads in flight per thread (a plain
// load -> store loop waits one memory round trip per iteration).  src(idx) -> uint4 (may apply
// bounds / zero-fill), dst(idx, v) stores into LDS.
template <typename SrcF, typename DstF>
__device__ __forceinline__ void stage_chunks(int n, SrcF src, DstF dst) {
  const int bs = blockDim.x;
  for (int base = threadIdx.x; base < n; base += 8 * bs) {
    uint4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = base + i * bs;
      v[i] = idx < n ? src(idx) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = base + i * bs;
      if (idx < n) dst(idx, v[i]);
    }
  }
}

// Chan et al. merge of (count, mean, M2) partials: (n, m, M2) <- (n, m, M2) + (nb, mb, M2b)
__device__ __forceinline__ void chan_merge(float& n, float& m, float& M2, float nb, float mb, float M2b) {
  const float nn = n + nb;
  if (nn > 0.f) {
    const float d = mb - m;
    const float f = nb / nn;
    m += d * f;
    M2 += M2b + d * d * n * f;
  }
  n = nn;
}

// ln_stats computed by a whole wave: lane t loads tile t (t, t+64, ...), then a butterfly merge, so
// the latency is one load round trip instead of T dependent ones.  Every lane gets the result.
__device__ __forceinline__ void wave_ln_stats(const float* __restrict__ part, int T, int BM, int L, int C, float eps,
                                              float& mean, float& rstd) {
  const int lane = threadIdx.x & 63;
  float n = 0.f, m = 0.f, M2 = 0.f;
  for (int t = lane; t < T; t += 64) {
    const float2 pm = *reinterpret_cast<const float2*>(part + 2 * t);
    chan_merge(n, m, M2, (float)(min(BM, L - t * BM) * C), pm.x, pm.y);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float nb = __shfl_xor(n, o, 64), mb = __shfl_xor(m, o, 64), M2b = __shfl_xor(M2, o, 64);
    chan_merge(n, m, M2, nb, mb, M2b);
  }
  mean = m;
  rstd = rsqrtf(M2 / n + eps);
}

// ln_bwd_consts computed by a whole wave (parallel loads + butterfly sums)
__device__ __forceinline__ void wave_bwd_consts(const float* __restrict__ part, int T, float inv_n, float& m1,
                                                float& m2) {
  const int lane = threadIdx.x & 63;
  float a = 0.f, c = 0.f;
  for (int t = lane; t < T; t += 64) {
    const float2 pm = *reinterpret_cast<const float2*>(part + 2 * t);
    a += pm.x;
    c += pm.y;
  }
  m1 = wave_reduce_sum(a) * inv_n;
  m2 = wave_reduce_sum(c) * inv_n;
}

// (count, mean, M2) of one wave's values: each lane contributes cnt values with sum s and sum of
// squared deviations from its own mean q; merged across the wave.  Returned on every lane.
__device__ __forceinline__ void wave_chan(float& n, float& m, float& M2) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float nb = __shfl_xor(n, o, 64), mb = __shfl_xor(m, o, 64), M2b = __shfl_xor(M2, o, 64);
    chan_merge(n, m, M2, nb, mb, M2b);
  }
}

}  // namespace pbx
