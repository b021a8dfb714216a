// Global track of one ProteinBERT block, column-split: three launches forward and three backward,
// each over ceil(B / 16) x (G / 64) workgroups (256 at B = G = 512) instead of B / 16.
//
// Reference: ProteinBERT/modules.py:175-199,219-229 (g + GELU(Linear G->G) + attention -> LayerNorm(G),
// twice) and :166-173,208-209 (the next block's global->local vector GELU(Linear G->C)), reference
// semantics (attention = (sum W / K) * sum_l GELU(h Wv)).
//
// Why split (glob2.hip, the one-launch form): a workgroup there owns 16 rows for the whole block and
// streams all three weight matrices (1.15 MB) through its CU, so 32 workgroups at B = 512 ran the
// block in 36 us (forward) / 46 us (backward) on 32 of the 256 CUs.  Here a workgroup owns a 16-row x
// 64-column output tile of one layer: it streams 64 KB of weights, the row LayerNorm is carried
// between launches as per-(row, column tile) partials ((mean, M2) forward, plain sums backward) that
// the next launch folds in its prologue while it normalises the full rows of its A tile, and the
// kernel boundary (~2 us) is the only synchronisation.  Column sums of the bias / affine / attention
// weight gradients go to a per-row-tile slab (every workgroup writes its own columns; deterministic)
// folded by one launch on the weight-gradient stream.
//
// MFMA v_mfma_f32_16x16x32_bf16: A = 16 activation rows (bf16, XOR-swizzled LDS tile), B = weight
// fragments in the packed layout of pbx_pack_glob_frags (one coalesced 1-KB load per fragment and
// wave), D: lane l holds column (l & 15) of rows 4 (l >> 4) .. +3; wave w owns 16-column tile w of the
// workgroup's 64 columns.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
typedef __attribute__((ext_vector_type(4))) float f4_t;
constexpr int RB = 16;       // rows per workgroup
constexpr int CT = 64;       // output columns per workgroup (4 waves x 16)
constexpr int PF = 4;        // B-fragment prefetch depth
constexpr int GMAX = 512;

__device__ __forceinline__ f4_t mfma16(const bf16x8& a, const bf16x8& b, const f4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int atile(int row, int chunk, int W) { return row * W * 2 + ((chunk ^ row) << 4); }
__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// acc += A(16 x KK, LDS tile of width KK) x B(KK x 16, packed tile `tile`): KK / 32 k-steps, a multiple
// of PF; the loads of step s + PF - 1 are in flight while step s runs
__device__ __forceinline__ f4_t gemm16(const unsigned char* at, int KK, const bf16x8* __restrict__ frag, int tile,
                                       int lane) {
  const int S = KK / 32;
  const int c16 = lane & 15, q = lane >> 4;
  const bf16x8* base = frag + (size_t)tile * S * 64 + lane;
  f4_t acc = {0.f, 0.f, 0.f, 0.f};
  bf16x8 ring[PF];
#pragma unroll
  for (int p = 0; p < PF - 1; ++p) ring[p] = base[(size_t)p * 64];
  for (int s0 = 0; s0 < S; s0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int s = s0 + u;
      ring[(u + PF - 1) % PF] = base[(size_t)min(s + PF - 1, S - 1) * 64];
      __builtin_amdgcn_sched_barrier(0);
      acc = mfma16(lds_frag(at, atile(c16, s * 4 + q, KK)), ring[u], acc);
    }
  }
  return acc;
}

// sums over the 16 lanes of a q group (the 16 columns of a wave tile), then over the 4 waves: per-row
// totals over the workgroup's 64 columns for this lane's rows 4q + i
__device__ __forceinline__ void tile_row_sums(const float* v, float* red, float* out, int lane, int w) {
  float s[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float a = v[i];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) a += __shfl_xor(a, o, 64);
    s[i] = a;
  }
  const int q = lane >> 4;
  __syncthreads();
  if ((lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w * RB + 4 * q + i] = s[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = red[4 * q + i] + red[RB + 4 * q + i] + red[2 * RB + 4 * q + i] + red[3 * RB + 4 * q + i];
}

// sum over the 16 rows (valid ones) of this lane's column: result on lanes 0..15 (column c16)
__device__ __forceinline__ float col_sum16(const float* v, const bool* rok) {
  float a = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) a += rok[i] ? v[i] : 0.f;
  a += __shfl_xor(a, 16, 64);
  a += __shfl_xor(a, 32, 64);
  return a;
}

__device__ __forceinline__ float mean_of(const float* __restrict__ wp, int K, int lane) {
  float a = 0.f;
  for (int i = lane; i < K; i += 64) a += wp[i];
  return wave_reduce_sum(a) / (float)K;
}

// per-row statistics of a row LayerNorm from NCT (mean, M2) partials of 64 columns each (Chan merge)
__device__ __forceinline__ void fold_ln_stats(const float2* __restrict__ part, int NCT, int G, float eps, int row0,
                                              int B, float* st) {
  const int t = threadIdx.x;
  if (t < RB) {
    const int row = min(row0 + t, B - 1);
    float m = 0.f;
    for (int c = 0; c < NCT; ++c) m += part[(size_t)row * NCT + c].x;
    m /= (float)NCT;
    float M2 = 0.f;
    for (int c = 0; c < NCT; ++c) {
      const float2 p = part[(size_t)row * NCT + c];
      M2 += p.y + (float)CT * (p.x - m) * (p.x - m);
    }
    st[2 * t] = m;
    st[2 * t + 1] = rsqrtf(M2 / (float)G + eps);
  }
}

// per-row (m1, m2) = (sum dxh, sum dxh xh) / G of the LayerNorm backward from NCT column-tile sums
__device__ __forceinline__ void fold_bwd_stats(const float2* __restrict__ part, int NCT, int G, int row0, int B,
                                               float* st) {
  const int t = threadIdx.x;
  if (t < RB) {
    const int row = min(row0 + t, B - 1);
    float a = 0.f, c = 0.f;
    for (int k = 0; k < NCT; ++k) {
      const float2 p = part[(size_t)row * NCT + k];
      a += p.x;
      c += p.y;
    }
    st[2 * t] = a / (float)G;
    st[2 * t + 1] = c / (float)G;
  }
}

// ---- layer 1: z1 = g + GELU(g W1^T + b1) + scale * sum_t vpart; (mean, M2) partials of z1 --------------
__global__ void __launch_bounds__(256) glob3_fwd1_kernel(
    const float* __restrict__ g, const bf16_t* __restrict__ g_bf, const float* __restrict__ vpart, int TV,
    const float* __restrict__ wp, int K, const bf16x8* __restrict__ f1, const float* __restrict__ b1,
    float* __restrict__ pre1, float* __restrict__ vsum, float* __restrict__ z1, float2* __restrict__ part, int B,
    int G) {
  __shared__ __attribute__((aligned(16))) unsigned char at[RB * GMAX * 2];
  __shared__ float red[4 * RB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * RB, ct = blockIdx.y * 4 + w, col = ct * 16 + c16;
  const int NCT = G / CT;
  int grow[4];
  bool rok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rok[i] = row0 + 4 * q + i < B;
    grow[i] = min(row0 + 4 * q + i, B - 1);
  }
  for (int idx = tid; idx < RB * G / 8; idx += 256) {
    const int row = idx / (G / 8), ch = idx % (G / 8);
    *reinterpret_cast<uint4*>(at + atile(row, ch, G)) =
        *reinterpret_cast<const uint4*>(g_bf + (size_t)min(row0 + row, B - 1) * G + ch * 8);
  }
  const float scale = mean_of(wp, K, lane);
  float res[4], vs[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    res[i] = g[(size_t)grow[i] * G + col];
    vs[i] = 0.f;
  }
  for (int tv0 = 0; tv0 < TV; tv0 += 4) {         // 4 tile rows in flight (clamped, surplus weighted 0)
    float v[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) v[u][i] = vpart[((size_t)grow[i] * TV + min(tv0 + u, TV - 1)) * G + col];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) vs[i] = fmaf(tv0 + u < TV ? 1.f : 0.f, v[u][i], vs[i]);
  }
  __syncthreads();
  const f4_t acc = gemm16(at, G, f1, ct, lane);
  const float bc = b1[col];
  float z[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float p = acc[i] + bc;
    z[i] = res[i] + gelu_f(p) + scale * vs[i];
    if (rok[i]) {
      const size_t e = (size_t)grow[i] * G + col;
      pre1[e] = p;
      vsum[e] = vs[i];
      z1[e] = z[i];
    }
  }
  float mean[4], d2[4], m2[4];
  tile_row_sums(z, red, mean, lane, w);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    mean[i] *= 1.f / (float)CT;
    d2[i] = (z[i] - mean[i]) * (z[i] - mean[i]);
  }
  tile_row_sums(d2, red, m2, lane, w);
  if (w == 0 && c16 == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (rok[i]) part[(size_t)grow[i] * NCT + blockIdx.y] = make_float2(mean[i], m2[i]);
  }
}

// Prologue of the layers that consume a row LayerNorm: fold the partials, normalise the 16 full rows
// into the bf16 A tile, write this workgroup's 64 columns of xh / out (bf16, optional fp32) and r.
// Returns (via st[]) the per-row (mean, rstd).
__device__ __forceinline__ void ln_prologue(const float* __restrict__ z, const float2* __restrict__ part,
                                            const float* __restrict__ nw, const float* __restrict__ nb, float eps,
                                            float* __restrict__ xh_o, float* __restrict__ r_o,
                                            bf16_t* __restrict__ out_bf, float* __restrict__ out_f32,
                                            unsigned char* at, float* st, int row0, int B, int G) {
  const int tid = threadIdx.x;
  fold_ln_stats(part, G / CT, G, eps, row0, B, st);
  __syncthreads();
  if (blockIdx.y == 0 && tid < RB && row0 + tid < B) r_o[row0 + tid] = st[2 * tid + 1];
  const int c0 = blockIdx.y * CT;
  for (int idx = tid; idx < RB * G / 8; idx += 256) {
    const int row = idx / (G / 8), ch = idx % (G / 8);
    const int gr = min(row0 + row, B - 1);
    const float m = st[2 * row], rs = st[2 * row + 1];
    float zv[8], gw[8], gb[8], xh[8], o[8];
    load8(z + (size_t)gr * G + ch * 8, zv);
    load8(nw + ch * 8, gw);
    load8(nb + ch * 8, gb);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xh[e] = (zv[e] - m) * rs;
      o[e] = xh[e] * gw[e] + gb[e];
    }
    const uint4 ob = packq8(o);
    *reinterpret_cast<uint4*>(at + atile(row, ch, G)) = ob;
    if (ch * 8 >= c0 && ch * 8 < c0 + CT && row0 + row < B) {
      const size_t e = (size_t)gr * G + ch * 8;
      store8(xh_o + e, xh);
      *reinterpret_cast<uint4*>(out_bf + e) = ob;
      if (out_f32 != nullptr) store8(out_f32 + e, o);
    }
  }
  __syncthreads();
}

// ---- layer 2: g1 = LN1(z1) (prologue); z2 = g1 + GELU(g1 W2^T + b2); (mean, M2) partials of z2 ------
__global__ void __launch_bounds__(256) glob3_fwd2_kernel(
    const float* __restrict__ z1, const float2* __restrict__ part1, const float* __restrict__ n1w,
    const float* __restrict__ n1b, float eps, float* __restrict__ xh1, float* __restrict__ r1,
    bf16_t* __restrict__ g1_bf, const bf16x8* __restrict__ f2, const float* __restrict__ b2,
    float* __restrict__ pre2, float* __restrict__ z2, float2* __restrict__ part2, int B, int G) {
  __shared__ __attribute__((aligned(16))) unsigned char at[RB * GMAX * 2];
  __shared__ float red[4 * RB];
  __shared__ float st[2 * RB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * RB, ct = blockIdx.y * 4 + w, col = ct * 16 + c16;
  ln_prologue(z1, part1, n1w, n1b, eps, xh1, r1, g1_bf, nullptr, at, st, row0, B, G);
  int grow[4];
  bool rok[4];
  float res[4];
  const float gw = n1w[col], gbv = n1b[col];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rok[i] = row0 + 4 * q + i < B;
    grow[i] = min(row0 + 4 * q + i, B - 1);
    res[i] = (z1[(size_t)grow[i] * G + col] - st[2 * (4 * q + i)]) * st[2 * (4 * q + i) + 1] * gw + gbv;
  }
  const f4_t acc = gemm16(at, G, f2, ct, lane);
  const float bc = b2[col];
  float z[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float p = acc[i] + bc;
    z[i] = res[i] + gelu_f(p);
    if (rok[i]) {
      const size_t e = (size_t)grow[i] * G + col;
      pre2[e] = p;
      z2[e] = z[i];
    }
  }
  float mean[4], d2[4], m2[4];
  tile_row_sums(z, red, mean, lane, w);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    mean[i] *= 1.f / (float)CT;
    d2[i] = (z[i] - mean[i]) * (z[i] - mean[i]);
  }
  tile_row_sums(d2, red, m2, lane, w);
  if (w == 0 && c16 == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (rok[i]) part2[(size_t)grow[i] * (G / CT) + blockIdx.y] = make_float2(mean[i], m2[i]);
  }
}

// ---- layer 3: g2 = LN2(z2) (prologue: xh2, r2, g2 fp32 + bf16); gb = GELU(g2 Wgl^T + bgl) on the
// workgroups with blockIdx.y < NGL / 64 ---------------------------------------------------------------
__global__ void __launch_bounds__(256) glob3_fwd3_kernel(
    const float* __restrict__ z2, const float2* __restrict__ part2, const float* __restrict__ n2w,
    const float* __restrict__ n2b, float eps, float* __restrict__ xh2, float* __restrict__ r2,
    float* __restrict__ g2, bf16_t* __restrict__ g2_bf, const bf16x8* __restrict__ fgl,
    const float* __restrict__ bgl, float* __restrict__ pregl, float* __restrict__ gb, int B, int G, int NGL) {
  __shared__ __attribute__((aligned(16))) unsigned char at[RB * GMAX * 2];
  __shared__ float st[2 * RB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * RB;
  ln_prologue(z2, part2, n2w, n2b, eps, xh2, r2, g2_bf, g2, at, st, row0, B, G);
  if ((int)blockIdx.y * CT >= NGL) return;
  const int ct = blockIdx.y * 4 + w, col = ct * 16 + c16;
  const f4_t acc = gemm16(at, G, fgl, ct, lane);
  const float bc = bgl[col];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = row0 + 4 * q + i;
    if (row < B) {
      const float p = acc[i] + bc;
      pregl[(size_t)row * NGL + col] = p;
      gb[(size_t)row * NGL + col] = gelu_f(p);
    }
  }
}

// slab row layout (one row per 16-row tile): [db1 | dn1w | dn1b | db2 | dn2w | dn2b] (G each) | dbgl
// (NGL) | dwp partials (G / 64)
enum { S_DB1 = 0, S_DN1W, S_DN1B, S_DB2, S_DN2W, S_DN2B };

// ---- backward 1: dugl = dgb * GELU'(pregl) (A tile, K = NGL), dg2 += dugl Wgl; LayerNorm-2 backward
// partials (sum dxh, sum dxh xh2) per (row, column tile); dn2w / dn2b column sums ------------------
__global__ void __launch_bounds__(256) glob3_bwd1_kernel(
    const float* __restrict__ dg2_in, const float* __restrict__ dgb, const float* __restrict__ pregl,
    const bf16x8* __restrict__ fglT, const float* __restrict__ xh2, const float* __restrict__ n2w,
    float* __restrict__ dg2_out, bf16_t* __restrict__ dugl, float2* __restrict__ part, float* __restrict__ slab,
    int ld, int B, int G, int NGL) {
  __shared__ __attribute__((aligned(16))) unsigned char at[RB * 128 * 2];
  __shared__ float red[4 * RB];
  __shared__ float dsl[RB * 128];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * RB, ct = blockIdx.y * 4 + w, col = ct * 16 + c16;
  float* srow = slab + (size_t)blockIdx.x * ld;
  int grow[4];
  bool rok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rok[i] = row0 + 4 * q + i < B;
    grow[i] = min(row0 + 4 * q + i, B - 1);
  }
  float dg[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dg[i] = dg2_in[(size_t)grow[i] * G + col];
  if (NGL > 0) {
    for (int idx = tid; idx < RB * NGL / 8; idx += 256) {
      const int row = idx / (NGL / 8), ch = idx % (NGL / 8);
      const int gr = min(row0 + row, B - 1);
      float dv[8], pv[8], o[8];
      load8(dgb + (size_t)gr * NGL + ch * 8, dv);
      load8(pregl + (size_t)gr * NGL + ch * 8, pv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = row0 + row < B ? dv[e] * gelu_grad_f(pv[e]) : 0.f;
      const uint4 ob = packq8(o);
      *reinterpret_cast<uint4*>(at + atile(row, ch, NGL)) = ob;
#pragma unroll
      for (int e = 0; e < 8; ++e) dsl[row * 128 + ch * 8 + e] = o[e];
      if (blockIdx.y == 0 && row0 + row < B) *reinterpret_cast<uint4*>(dugl + (size_t)gr * NGL + ch * 8) = ob;
    }
    __syncthreads();
    if (blockIdx.y == 0 && tid < NGL) {            // dbgl column sums (fp32 values) of the 16 rows
      float a = 0.f;
#pragma unroll
      for (int r = 0; r < RB; ++r) a += dsl[r * 128 + tid];
      srow[6 * G + tid] = a;
    }
    const f4_t acc = gemm16(at, NGL, fglT, ct, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) dg[i] += acc[i];
  }
  const float gw = n2w[col];
  float dxh[4], dxx[4], xv[4], sa[4], sc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xv[i] = xh2[(size_t)grow[i] * G + col];
    dxh[i] = dg[i] * gw;
    dxx[i] = dxh[i] * xv[i];
    if (rok[i]) dg2_out[(size_t)grow[i] * G + col] = dg[i];
  }
  tile_row_sums(dxh, red, sa, lane, w);
  tile_row_sums(dxx, red, sc, lane, w);
  if (w == 0 && c16 == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (rok[i]) part[(size_t)grow[i] * (G / CT) + blockIdx.y] = make_float2(sa[i], sc[i]);
  }
  float t1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) t1[i] = dg[i] * xv[i];
  const float cw = col_sum16(t1, rok), cb = col_sum16(dg, rok);
  if (lane < 16) {
    srow[S_DN2W * G + col] = cw;
    srow[S_DN2B * G + col] = cb;
  }
}

// LayerNorm backward of one element: dz = r (dxh - m1 - xh m2), dxh = dg * gamma
__device__ __forceinline__ float ln_bwd(float dg, float gam, float xh, float r, float m1, float m2) {
  return r * (dg * gam - m1 - xh * m2);
}

// Prologue of backward 2 / 3: fold the partials; A tile = bf16 dpre = dz * GELU'(pre) of the 16 full
// rows; this workgroup's columns of du (bf16) are written.
__device__ __forceinline__ void bwd_prologue(const float* __restrict__ dgin, const float2* __restrict__ part,
                                             const float* __restrict__ xh, const float* __restrict__ r,
                                             const float* __restrict__ gam, const float* __restrict__ pre,
                                             bf16_t* __restrict__ du, unsigned char* at, float* st, int row0, int B,
                                             int G) {
  const int tid = threadIdx.x;
  fold_bwd_stats(part, G / CT, G, row0, B, st);
  __syncthreads();
  const int c0 = blockIdx.y * CT;
  for (int idx = tid; idx < RB * G / 8; idx += 256) {
    const int row = idx / (G / 8), ch = idx % (G / 8);
    const int gr = min(row0 + row, B - 1);
    const float m1 = st[2 * row], m2 = st[2 * row + 1], rr = r[gr];
    float dv[8], xv[8], gw[8], pv[8], o[8];
    load8(dgin + (size_t)gr * G + ch * 8, dv);
    load8(xh + (size_t)gr * G + ch * 8, xv);
    load8(gam + ch * 8, gw);
    load8(pre + (size_t)gr * G + ch * 8, pv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = row0 + row < B ? ln_bwd(dv[e], gw[e], xv[e], rr, m1, m2) * gelu_grad_f(pv[e]) : 0.f;
    const uint4 ob = packq8(o);
    *reinterpret_cast<uint4*>(at + atile(row, ch, G)) = ob;
    if (ch * 8 >= c0 && ch * 8 < c0 + CT && row0 + row < B) *reinterpret_cast<uint4*>(du + (size_t)gr * G + ch * 8) = ob;
  }
  __syncthreads();
}

// ---- backward 2: dz2 (LayerNorm-2 backward), du2 = dz2 GELU'(pre2) (A tile), dg1 = dz2 + du2 W2;
// LayerNorm-1 backward partials of dg1; db2 / dn1w / dn1b column sums ------------------------------
__global__ void __launch_bounds__(256) glob3_bwd2_kernel(
    const float* __restrict__ dg2, const float2* __restrict__ part2, const float* __restrict__ xh2,
    const float* __restrict__ r2, const float* __restrict__ n2w, const float* __restrict__ pre2,
    const bf16x8* __restrict__ f2T, const float* __restrict__ xh1, const float* __restrict__ n1w,
    bf16_t* __restrict__ du2, float* __restrict__ dg1_out, float2* __restrict__ part1, float* __restrict__ slab,
    int ld, int B, int G) {
  __shared__ __attribute__((aligned(16))) unsigned char at[RB * GMAX * 2];
  __shared__ float red[4 * RB];
  __shared__ float st[2 * RB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * RB, ct = blockIdx.y * 4 + w, col = ct * 16 + c16;
  float* srow = slab + (size_t)blockIdx.x * ld;
  bwd_prologue(dg2, part2, xh2, r2, n2w, pre2, du2, at, st, row0, B, G);
  int grow[4];
  bool rok[4];
  float dz[4], dpre[4];
  const float gw2 = n2w[col];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rok[i] = row0 + 4 * q + i < B;
    grow[i] = min(row0 + 4 * q + i, B - 1);
    const size_t e = (size_t)grow[i] * G + col;
    const int rl = 4 * q + i;
    dz[i] = ln_bwd(dg2[e], gw2, xh2[e], r2[grow[i]], st[2 * rl], st[2 * rl + 1]);
    dpre[i] = dz[i] * gelu_grad_f(pre2[e]);
  }
  const f4_t acc = gemm16(at, G, f2T, ct, lane);
  const float gw1 = n1w[col];
  float dg1[4], dxh[4], dxx[4], xv[4], sa[4], sc[4], t1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dg1[i] = dz[i] + acc[i];
    xv[i] = xh1[(size_t)grow[i] * G + col];
    dxh[i] = dg1[i] * gw1;
    dxx[i] = dxh[i] * xv[i];
    t1[i] = dg1[i] * xv[i];
    if (rok[i]) dg1_out[(size_t)grow[i] * G + col] = dg1[i];
  }
  tile_row_sums(dxh, red, sa, lane, w);
  tile_row_sums(dxx, red, sc, lane, w);
  if (w == 0 && c16 == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (rok[i]) part1[(size_t)grow[i] * (G / CT) + blockIdx.y] = make_float2(sa[i], sc[i]);
  }
  const float cdb2 = col_sum16(dpre, rok), cw = col_sum16(t1, rok), cb = col_sum16(dg1, rok);
  if (lane < 16) {
    srow[S_DB2 * G + col] = cdb2;
    srow[S_DN1W * G + col] = cw;
    srow[S_DN1B * G + col] = cb;
  }
}

// ---- backward 3: dz1 (LayerNorm-1 backward), du1 = dz1 GELU'(pre1) (A tile), dg = dz1 + du1 W1,
// dvs = scale dz1 (the attention partial-sum gradient); db1 column sums, dwp partials --------------
__global__ void __launch_bounds__(256) glob3_bwd3_kernel(
    const float* __restrict__ dg1, const float2* __restrict__ part1, const float* __restrict__ xh1,
    const float* __restrict__ r1, const float* __restrict__ n1w, const float* __restrict__ pre1,
    const float* __restrict__ vsum, const float* __restrict__ wp, int K, const bf16x8* __restrict__ f1T,
    bf16_t* __restrict__ du1, float* __restrict__ dg, float* __restrict__ dvs, float* __restrict__ slab, int ld,
    int B, int G, int NGL) {
  __shared__ __attribute__((aligned(16))) unsigned char at[RB * GMAX * 2];
  __shared__ float red[4 * RB];
  __shared__ float st[2 * RB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * RB, ct = blockIdx.y * 4 + w, col = ct * 16 + c16;
  float* srow = slab + (size_t)blockIdx.x * ld;
  bwd_prologue(dg1, part1, xh1, r1, n1w, pre1, du1, at, st, row0, B, G);
  const float scale = mean_of(wp, K, lane);
  int grow[4];
  bool rok[4];
  float dz[4], dpre[4], av[4];
  const float gw1 = n1w[col];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rok[i] = row0 + 4 * q + i < B;
    grow[i] = min(row0 + 4 * q + i, B - 1);
    const size_t e = (size_t)grow[i] * G + col;
    const int rl = 4 * q + i;
    dz[i] = ln_bwd(dg1[e], gw1, xh1[e], r1[grow[i]], st[2 * rl], st[2 * rl + 1]);
    dpre[i] = dz[i] * gelu_grad_f(pre1[e]);
    av[i] = rok[i] ? dz[i] * vsum[e] : 0.f;
    if (rok[i]) dvs[e] = scale * dz[i];
  }
  const f4_t acc = gemm16(at, G, f1T, ct, lane);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (rok[i]) dg[(size_t)grow[i] * G + col] = dz[i] + acc[i];
  const float cdb1 = col_sum16(dpre, rok);
  if (lane < 16) srow[S_DB1 * G + col] = cdb1;
  // dwp partial: sum over the tile of dz1 * vsum (d scale / d wp_k = 1 / K for every k)
  float tot[4];
  tile_row_sums(av, red, tot, lane, w);
  if (tid == 0) {
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < RB; ++r) a += red[r] + red[RB + r] + red[2 * RB + r] + red[3 * RB + r];
    srow[6 * G + NGL + blockIdx.y] = a;
  }
  (void)tot;
}

// fold of the slab rows into the gradients (fixed row order): segment j of [6 G + NGL] columns -> dst,
// and dwp[k] += (sum of the dwp partials) / K
struct GlobDst {
  float* d[7];
};
__global__ void __launch_bounds__(256) glob3_fold_kernel(const float* __restrict__ slab, int rows, int ld, GlobDst dst,
                                                         float* __restrict__ dwp, int K, int G, int NGL) {
  __shared__ float red[256];
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int ncol = 6 * G + NGL;
  if (blockIdx.x < gridDim.x - 1) {
    if (j >= ncol) return;
    float a = 0.f;
    for (int r = 0; r < rows; ++r) a += slab[(size_t)r * ld + j];
    const int seg = j / G < 6 ? j / G : 6;
    const int off = seg < 6 ? j - seg * G : j - 6 * G;
    if (dst.d[seg] != nullptr) dst.d[seg][off] += a;
    return;
  }
  // last block: the dwp total
  const int nct = G / CT;
  float a = 0.f;
  for (int i = threadIdx.x; i < rows * nct; i += 256) a += slab[(size_t)(i / nct) * ld + ncol + (i % nct)];
  red[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < 256; ++i) s += red[i];
    red[0] = s / (float)K;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += 256) dwp[k] += red[0];
}
}  // namespace

PBX_EXPORT int pbx_glob3_slab_cols(int G, int NGL) { return 6 * G + NGL + G / CT; }

// p: g, g_bf, vpart, wp, f1, b1, n1w, n1b, f2, b2, n2w, n2b, fgl, bgl, pre1, xh1, r1, vsum, g1_bf, pre2, xh2,
//    r2, g2, g2_bf, pregl, gb, z1, z2, part1, part2   (30 pointers; fgl / bgl / pregl / gb null when NGL == 0;
//    z1 / z2 [B][G] fp32 and part1 / part2 [B][G / 64] float2 scratch)
PBX_EXPORT int pbx_glob3_fwd(const void* const* p, int B, int G, int NGL, int TV, int K, float eps, hipStream_t st) {
  if ((G != 256 && G != 512) || (NGL != 0 && NGL != 128) || B < 1 || K < 1 || TV < 1) return (int)hipErrorInvalidValue;
  const dim3 grid((B + RB - 1) / RB, G / CT);
  auto F = [&](int i) { return (const float*)p[i]; };
  auto W = [&](int i) { return (float*)p[i]; };
  hipLaunchKernelGGL(glob3_fwd1_kernel, grid, dim3(256), 0, st, F(0), (const bf16_t*)p[1], F(2), TV, F(3), K,
                     (const bf16x8*)p[4], F(5), W(14), W(17), W(26), (float2*)p[28], B, G);
  hipLaunchKernelGGL(glob3_fwd2_kernel, grid, dim3(256), 0, st, F(26), (const float2*)p[28], F(6), F(7), eps, W(15),
                     W(16), (bf16_t*)p[18], (const bf16x8*)p[8], F(9), W(19), W(27), (float2*)p[29], B, G);
  hipLaunchKernelGGL(glob3_fwd3_kernel, grid, dim3(256), 0, st, F(27), (const float2*)p[29], F(10), F(11), eps, W(20),
                     W(21), W(22), (bf16_t*)p[23], (const bf16x8*)p[12], F(13), W(24), W(25), B, G, NGL);
  return pbx_launch_status();
}

// p: dg2, dgb, pregl, fglT, xh2, r2, n2w, pre2, f2T, xh1, r1, n1w, pre1, vsum, wp, f1T, dg, dvs, du1, du2, dugl,
//    dg2s, dg1s, part2, part1   (25 pointers; dgb / pregl / fglT / dugl null when NGL == 0; dg2s / dg1s
//    [B][G] fp32 and part2 / part1 [B][G / 64] float2 scratch).  slab: [ceil(B / 16)][pbx_glob3_slab_cols]
//    per-row-tile column sums (fully written here), folded by pbx_glob3_fold.
PBX_EXPORT int pbx_glob3_bwd(const void* const* p, int B, int G, int NGL, int K, float* slab, hipStream_t st) {
  if ((G != 256 && G != 512) || (NGL != 0 && NGL != 128) || B < 1 || K < 1) return (int)hipErrorInvalidValue;
  const dim3 grid((B + RB - 1) / RB, G / CT);
  const int ld = pbx_glob3_slab_cols(G, NGL);
  auto F = [&](int i) { return (const float*)p[i]; };
  auto W = [&](int i) { return (float*)p[i]; };
  hipLaunchKernelGGL(glob3_bwd1_kernel, grid, dim3(256), 0, st, F(0), F(1), F(2), (const bf16x8*)p[3], F(4), F(6),
                     W(21), (bf16_t*)p[20], (float2*)p[23], slab, ld, B, G, NGL);
  hipLaunchKernelGGL(glob3_bwd2_kernel, grid, dim3(256), 0, st, F(21), (const float2*)p[23], F(4), F(5), F(6), F(7),
                     (const bf16x8*)p[8], F(9), F(11), (bf16_t*)p[19], W(22), (float2*)p[24], slab, ld, B, G);
  hipLaunchKernelGGL(glob3_bwd3_kernel, grid, dim3(256), 0, st, F(22), (const float2*)p[24], F(9), F(10), F(11),
                     F(12), F(13), F(14), K, (const bf16x8*)p[15], (bf16_t*)p[18], W(16), W(17), slab, ld, B, G, NGL);
  return pbx_launch_status();
}

// d: db1, dn1w, dn1b, db2, dn2w, dn2b, dbgl (nullable when NGL == 0), dwp
PBX_EXPORT int pbx_glob3_fold(const float* slab, int B, int G, int NGL, int K, const void* const* d, hipStream_t st) {
  const int rows = (B + RB - 1) / RB, ld = pbx_glob3_slab_cols(G, NGL);
  GlobDst dst;
  for (int i = 0; i < 7; ++i) dst.d[i] = (float*)d[i];
  const int nb = (6 * G + NGL + 255) / 256 + 1;
  hipLaunchKernelGGL(glob3_fold_kernel, dim3(nb), dim3(256), 0, st, slab, rows, ld, dst, (float*)d[7], K, G, NGL);
  return pbx_launch_status();
}
