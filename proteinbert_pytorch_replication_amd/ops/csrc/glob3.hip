// Global track of one ProteinBERT block, forward, column-split: three launches, each over ceil(B / 16) x
// (G / 64) workgroups (256 at B = G = 512) instead of B / 16.  The backward is the one-launch
// glob2.hip glob_bwd (a column-split backward measured slower beside the weight-gradient stream).
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
// kernel boundary (~2 us) is the only synchronisation.
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

}  // namespace

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
