// Fused global track of one ProteinBERT block, backward: ONE launch per block ("persistent
// global-track kernel"); the forward is the column-split glob3.hip.
//
// Reference: ProteinBERT/modules.py:175-199,219-229 (g + GELU(Linear G->G) + attention -> LayerNorm(G),
// twice) and :166-173,208-209 (the next block's global->local vector GELU(Linear G->C)), reference
// semantics (attention = (sum W / K) * sum_l GELU(h Wv)).
//
// Every row (protein) of the global track is independent except for the weight gradients, so a
// workgroup owns 16 rows for the WHOLE block: GEMM -> bias/GELU/residual/attention -> LayerNorm ->
// GEMM -> ... -> GEMM -> GELU, with the activations of its rows in LDS / registers and no
// inter-workgroup traffic.  This replaces 3 hipBLASLt GEMMs + 3 elementwise/row-LN launches per
// block forward and 6 GEMMs + 3 launches per block backward (~9-16 us each, latency bound at
// [256 x 512] x [512 x 512]).
//
// MFMA: v_mfma_f32_16x16x32_bf16 (wave64).  A = 16 activation rows (bf16, XOR-swizzled LDS tile),
// B = weight fragments streamed from L2 in a fragment-native packed layout (pbx_pack_glob_frags:
// one coalesced 1-KB load per fragment and wave), D: lane l holds column (l & 15) of rows
// 4(l >> 4) .. +3.  Wave w owns output column tiles w*NT .. w*NT+NT-1 (16 columns each).
//
// Backward data path in the same structure; the weight gradients dW = dU^T X (K = B rows) are
// left to three library GEMMs the caller issues off the critical path.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
typedef __attribute__((ext_vector_type(4))) float f4_t;
constexpr int RB = 16;       // rows per workgroup
constexpr int pbx_glob_pf = 4;   // B-fragment prefetch depth (k-steps in flight)

__device__ __forceinline__ f4_t mfma16(const bf16x8& a, const bf16x8& b, const f4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// [16][W] bf16 activation tile: row stride 2W bytes, 16-B chunks XOR-swizzled by row so the A-fragment
// reads (16 rows x 4 consecutive chunks) hit 16 distinct 16-B bank groups.
__device__ __forceinline__ int atile(int row, int chunk, int W) { return row * W * 2 + ((chunk ^ row) << 4); }
__device__ __forceinline__ int atile_e(int row, int col, int W) { return atile(row, col >> 3, W) + ((col & 7) << 1); }

// acc[t] += A(16 x KK, LDS tile of width KK) x B(KK x 16 tile (tile0 + t)), B fragments packed as
// [tile][kstep][lane] of bf16x8 (KK / 32 k-steps per tile, a multiple of PF).  Step s uses ring slot
// s % PF while the loads of step s + PF - 1 are in flight: the loop is unrolled by the ring size so
// no register rotates (which would make the compiler wait for the newest load every step).
template <int NT, int PF = (NT > 4 ? 2 : pbx_glob_pf)>   // 8 tiles a wave (4-wave backward): a 2-deep ring
__device__ __forceinline__ void gemm_rows(f4_t* acc, const unsigned char* at, int KK, const bf16x8* __restrict__ frag,
                                          int tile0, int lane) {
  const int S = KK / 32;
  const int c16 = lane & 15, q = lane >> 4;
  const bf16x8* base = frag + (size_t)tile0 * S * 64 + lane;
  bf16x8 ring[PF][NT];
#pragma unroll
  for (int p = 0; p < PF - 1; ++p)
#pragma unroll
    for (int t = 0; t < NT; ++t) ring[p][t] = base[((size_t)t * S + p) * 64];
  for (int s0 = 0; s0 < S; s0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int s = s0 + u;
      const int sn = min(s + PF - 1, S - 1);
#pragma unroll
      for (int t = 0; t < NT; ++t) ring[(u + PF - 1) % PF][t] = base[((size_t)t * S + sn) * 64];
      __builtin_amdgcn_sched_barrier(0);          // keep the prefetch ahead of this step's MFMAs
      const bf16x8 a = lds_frag(at, atile(c16, s * 4 + q, KK));
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma16(a, ring[u][t], acc[t]);
    }
  }
}

// per-row sums of v[t][i] (row 4q + i) over the workgroup's columns: lanes of one q share rows;
// red: [NW][RB] floats.  Returns the 4 row totals of this lane's rows.
template <int NT, int NW>
__device__ __forceinline__ void row_sums(const float (*v)[4], float* red, float* out, int lane, int w) {
  float s[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float a = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) a += v[t][i];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) a += __shfl_xor(a, o, 64);
    s[i] = a;
  }
  const int q = lane >> 4;
  __syncthreads();                              // red free (previous use done)
  if ((lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w * RB + 4 * q + i] = s[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float a = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) a += red[ww * RB + 4 * q + i];
    out[i] = a;
  }
}

// column sums over the workgroup's valid rows of v[t][i] -> one atomic per column, or (sl != nullptr,
// deterministic mode) one store into this workgroup's slab row, folded in a fixed order by the caller
template <int NT>
__device__ __forceinline__ void col_atomic(const float (*v)[4], const bool* rok, float* __restrict__ dst, int col0,
                                           int lane, float* __restrict__ sl) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) a += rok[i] ? v[t][i] : 0.f;
    a += __shfl_xor(a, 16, 64);
    a += __shfl_xor(a, 32, 64);
    if (lane < 16) {
      if (sl != nullptr) sl[col0 + t * 16 + lane] = a;
      else atomicAdd(dst + col0 + t * 16 + lane, a);
    }
  }
}

// mean of wp[0..K) on every lane: one load round trip per 64 values (a per-thread scalar loop waits
// one scalar-cache round trip per element)
__device__ __forceinline__ float wave_mean(const float* __restrict__ wp, int K, int lane) {
  float a = 0.f;
  for (int i = lane; i < K; i += 64) a += wp[i];
  return wave_reduce_sum(a) / (float)K;
}

// ------------------------------------------------------------------------------------------------
// backward data path.  dg2: [B, G] gradient of g2 (from the next block / heads); dgb: [B, NGL]
// gradient of gb (NT3 > 0).  Outputs: dg [B, G] (gradient of the block input g), dvs [B, G] (the
// attention partial-sum gradient, identical for every tile), du1/du2/dugl (bf16, the weight
// gradient GEMM operands), and column-sum gradients accumulated with one atomic per column and
// workgroup: db1, dn1w, dn1b, db2, dn2w, dn2b, dbgl, dwp.
template <int NT, int NW, int NGL>
__global__ void __launch_bounds__(NW * 64) glob_bwd_kernel(
    const float* __restrict__ dg2_in, const float* __restrict__ dgb, const float* __restrict__ pregl,
    const bf16x8* __restrict__ fglT, const float* __restrict__ xh2, const float* __restrict__ r2,
    const float* __restrict__ n2w, const float* __restrict__ pre2, const bf16x8* __restrict__ f2T,
    const float* __restrict__ xh1, const float* __restrict__ r1, const float* __restrict__ n1w,
    const float* __restrict__ pre1, const float* __restrict__ vsum, const float* __restrict__ wp, int K,
    const bf16x8* __restrict__ f1T, float* __restrict__ dg, float* __restrict__ dvs, bf16_t* __restrict__ du1,
    bf16_t* __restrict__ du2, bf16_t* __restrict__ dugl, float* __restrict__ db1, float* __restrict__ dn1w,
    float* __restrict__ dn1b, float* __restrict__ db2, float* __restrict__ dn2w, float* __restrict__ dn2b,
    float* __restrict__ dbgl, float* __restrict__ dwp, int B, float* __restrict__ slab, int K_) {
  constexpr int G = NT * 16 * NW, NT3 = NGL > 0 ? 1 : 0;
  // deterministic mode: this workgroup's column sums go to slab row blockIdx.x:
  //   [db1 | dn1w | dn1b | db2 | dn2w | dn2b] (G each) | dbgl (NGL) | dwp (K)
  float* srow = slab != nullptr ? slab + (size_t)blockIdx.x * (6 * G + NGL + K_) : nullptr;
  auto sub = [&](int k) { return srow != nullptr ? srow + k * G : nullptr; };
  __shared__ __attribute__((aligned(16))) unsigned char at[RB * G * 2];
  __shared__ float red[NW * RB];
  __shared__ float dsum[NT3 > 0 ? RB * NGL : 1];   // fp32 dugl for the bias-gradient column sums
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c16 = lane & 15, q = lane >> 4;
  const int row0 = blockIdx.x * RB;
  int grow[4];
  bool rok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rok[i] = row0 + 4 * q + i < B;
    grow[i] = min(row0 + 4 * q + i, B - 1);
  }
  const int col0 = w * NT * 16;
  f4_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[t][i] = dg2_in[(size_t)grow[i] * G + col0 + t * 16 + c16];

  // ---- gb = GELU(pregl): dugl = dgb * GELU'(pregl) ; dg2 += dugl Wgl ----
  if constexpr (NT3 > 0) {
    for (int idx = tid; idx < RB * NGL; idx += NW * 64) {
      const int row = idx / NGL, c = idx % NGL;
      const int gr = min(row0 + row, B - 1);
      const bool ok = row0 + row < B;
      const float d = ok ? dgb[(size_t)gr * NGL + c] * gelu_grad_f(pregl[(size_t)gr * NGL + c]) : 0.f;
      const bf16_t db = f2bf(d);
      *reinterpret_cast<bf16_t*>(at + atile_e(row, c, NGL)) = db;
      dsum[idx] = d;
      if (ok) dugl[(size_t)gr * NGL + c] = db;
    }
    __syncthreads();
    for (int c = tid; c < NGL; c += NW * 64) {    // dbgl: column sums over the rows
      float a = 0.f;
      for (int row = 0; row < RB; ++row) a += dsum[row * NGL + c];
      if (srow != nullptr) srow[6 * G + c] = a;
      else atomicAdd(dbgl + c, a);
    }
    gemm_rows<NT>(acc, at, NGL, fglT, w * NT, lane);
    __syncthreads();                              // A tile is rewritten below
  }

  const float scale = wave_mean(wp, K, lane);

  // LayerNorm + GELU backward of one stage: dy (acc) -> ds = rstd (dy g - m1 - xh m2) ;
  // du = ds GELU'(pre) (A tile + global) ; column sums dgam += dy xh, dbet += dy, dbias += du.
  auto ln_bwd = [&](const f4_t* dyv, const float* __restrict__ xh_in, const float* __restrict__ r_in,
                    const float* __restrict__ gam, const float* __restrict__ pre, bf16_t* __restrict__ du_o,
                    float* __restrict__ dbias, float* __restrict__ dgam, float* __restrict__ dbet,
                    float (*ds)[4], int sbase) {
    float xh[NT][4], dxh[NT][4], dxx[NT][4], tmp[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = col0 + t * 16 + c16;
      const float ga = gam[c];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xh[t][i] = xh_in[(size_t)grow[i] * G + c];
        dxh[t][i] = dyv[t][i] * ga;
        dxx[t][i] = dxh[t][i] * xh[t][i];
        tmp[t][i] = dyv[t][i] * xh[t][i];
      }
    }
    col_atomic<NT>(tmp, rok, dgam, col0, lane, sub(sbase + 1));
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) tmp[t][i] = dyv[t][i];
    col_atomic<NT>(tmp, rok, dbet, col0, lane, sub(sbase + 2));
    float m1[4], m2[4], rs[4];
    row_sums<NT, NW>(dxh, red, m1, lane, w);
    row_sums<NT, NW>(dxx, red, m2, lane, w);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      m1[i] *= 1.f / (float)G;
      m2[i] *= 1.f / (float)G;
      rs[i] = r_in[grow[i]];
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = col0 + t * 16 + c16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ds[t][i] = rs[i] * (dxh[t][i] - m1[i] - xh[t][i] * m2[i]);
        const float d = ds[t][i] * gelu_grad_f(pre[(size_t)grow[i] * G + c]);
        const bf16_t db = f2bf(d);
        tmp[t][i] = d;
        *reinterpret_cast<bf16_t*>(at + atile_e(4 * q + i, c, G)) = db;
        if (rok[i]) du_o[(size_t)grow[i] * G + c] = db;
      }
    }
    col_atomic<NT>(tmp, rok, dbias, col0, lane, sub(sbase));
    __syncthreads();                              // du tile complete
  };

  // ---- LN2 / MLP2: dg1 = ds2 + du2 W2 ----
  {
    float ds[NT][4];
    ln_bwd(acc, xh2, r2, n2w, pre2, du2, db2, dn2w, dn2b, ds, 3);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][i] = ds[t][i];
    gemm_rows<NT>(acc, at, G, f2T, w * NT, lane);
    __syncthreads();
  }
  // ---- LN1 / MLP1 / attention: dg = ds1 + du1 W1 ; dvs = scale ds1 ; dwp += sum(ds1 vsum) / K ----
  {
    float ds[NT][4];
    ln_bwd(acc, xh1, r1, n1w, pre1, du1, db1, dn1w, dn1b, ds, 0);
    float sv = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = col0 + t * 16 + c16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[t][i] = ds[t][i];
        if (rok[i]) {
          dvs[(size_t)grow[i] * G + c] = scale * ds[t][i];
          sv += ds[t][i] * vsum[(size_t)grow[i] * G + c];
        }
      }
    }
    sv = wave_reduce_sum(sv);
    __syncthreads();
    if (lane == 0) red[w] = sv;
    __syncthreads();
    if (tid < K) {
      float a = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) a += red[ww];
      if (srow != nullptr) srow[6 * G + NGL + tid] = a / (float)K;
      else atomicAdd(dwp + tid, a / (float)K);
    }
    gemm_rows<NT>(acc, at, G, f1T, w * NT, lane);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (rok[i]) dg[(size_t)grow[i] * G + col0 + t * 16 + c16] = acc[t][i];
  }
}

// fp32 weight W [N][Kd] -> bf16 B-fragment images for the two products of the global track:
//   fwd (D = X W^T):  tile n16 = n/16, k-step s = k/32: lane l = W[16 n16 + (l&15)][32 s + 8(l>>4) + j]
//   bwd (D = dU W):   tile k16 = k/16, n-step s = n/32: lane l = W[32 s + 8(l>>4) + j][16 k16 + (l&15)]
__global__ void __launch_bounds__(256) pack_glob_frags_kernel(const float* __restrict__ w, bf16_t* __restrict__ ff,
                                                             bf16_t* __restrict__ fb, int N, int Kd) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= N * Kd) return;
  const int j = idx & 7, l = (idx >> 3) & 63, f = idx >> 9;
  {
    const int S = Kd / 32, t = f / S, s = f % S;
    ff[idx] = f2bf(w[(size_t)(t * 16 + (l & 15)) * Kd + s * 32 + 8 * (l >> 4) + j]);
  }
  {
    const int S = N / 32, t = f / S, s = f % S;
    fb[idx] = f2bf(w[(size_t)(s * 32 + 8 * (l >> 4) + j) * Kd + t * 16 + (l & 15)]);
  }
}

template <int NT, int NW, int NGL>
void launch_bwd(int B, const void* const* p, int K, float* slab, hipStream_t st) {
  hipLaunchKernelGGL((glob_bwd_kernel<NT, NW, NGL>), dim3((B + RB - 1) / RB), dim3(NW * 64), 0, st, (const float*)p[0],
                     (const float*)p[1], (const float*)p[2], (const bf16x8*)p[3], (const float*)p[4],
                     (const float*)p[5], (const float*)p[6], (const float*)p[7], (const bf16x8*)p[8],
                     (const float*)p[9], (const float*)p[10], (const float*)p[11], (const float*)p[12],
                     (const float*)p[13], (const float*)p[14], K, (const bf16x8*)p[15], (float*)p[16],
                     (float*)p[17], (bf16_t*)p[18], (bf16_t*)p[19], (bf16_t*)p[20], (float*)p[21], (float*)p[22],
                     (float*)p[23], (float*)p[24], (float*)p[25], (float*)p[26], (float*)p[27], (float*)p[28], B,
                     slab, K);
}
}  // namespace

// G in {256, 512}; NGL in {0, 128} (the local width C = 128 of the paper configuration).
static int pbx_glob_supported(int G, int NGL) {   // mirrored by global_track.glob_fused_ok
  return (G == 256 || G == 512) && (NGL == 0 || NGL == 128);
}

extern "C" int pbx_colsum_add_ld(const float* src, int rows, int cols, int ld, float* dst, const float* scale,
                                 hipStream_t st);

// p: dg2, dgb, pregl, fglT, xh2, r2, n2w, pre2, f2T, xh1, r1, n1w, pre1, vsum, wp, f1T, dg, dvs, du1, du2, dugl,
//    db1, dn1w, dn1b, db2, dn2w, dn2b, dbgl, dwp   (29 pointers)
// slab (nullable, deterministic mode): [ceil(B / 16)][6 G + NGL + K] fp32 column-sum partials, folded into
// the eight gradient destinations in a fixed order
PBX_EXPORT int pbx_glob_bwd(const void* const* p, int B, int G, int NGL, int K, float* slab, hipStream_t st) {
  if (!pbx_glob_supported(G, NGL) || B < 1 || K < 1 || K > 512) return (int)hipErrorInvalidValue;
  // 8 waves (a 16-wave build does not fit 128 VGPRs; a 4-wave form measured no better beside conv_dgrad4)
  if (G == 512) (NGL ? launch_bwd<4, 8, 128> : launch_bwd<4, 8, 0>)(B, p, K, slab, st);
  else (NGL ? launch_bwd<2, 8, 128> : launch_bwd<2, 8, 0>)(B, p, K, slab, st);
  int rc = pbx_launch_status();
  if (rc != 0 || slab == nullptr) return rc;
  const int rows = (B + RB - 1) / RB, ld = 6 * G + NGL + K;
  float* dst[8] = {(float*)p[21], (float*)p[22], (float*)p[23], (float*)p[24], (float*)p[25], (float*)p[26],
                   (float*)p[27], (float*)p[28]};
  const int off[8] = {0, G, 2 * G, 3 * G, 4 * G, 5 * G, 6 * G, 6 * G + NGL};
  const int len[8] = {G, G, G, G, G, G, NGL, K};
  for (int i = 0; i < 8 && rc == 0; ++i)
    if (len[i] > 0 && dst[i] != nullptr) rc = pbx_colsum_add_ld(slab + off[i], rows, len[i], ld, dst[i], nullptr, st);
  return rc;
}

// fragment images of W [N][Kd] (N, Kd multiples of 32; N*Kd bf16 each)
PBX_EXPORT int pbx_pack_glob_frags(const float* w, void* ff, void* fb, int N, int Kd, hipStream_t st) {
  if (N % 32 || Kd % 32) return (int)hipErrorInvalidValue;
  const int n = N * Kd;
  hipLaunchKernelGGL(pack_glob_frags_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w, (bf16_t*)ff, (bf16_t*)fb,
                     N, Kd);
  return pbx_launch_status();
}
