// Small fp32 GEMMs of the paper-semantics attention query path, with the operand layouts and epilogues
// fused in (reference intent: ProteinBERT/modules.py:49-60 -- q = tanh(g Wq) feeds the softmax over
// positions, so it is kept at fp32 accuracy).
//
//   forward   q = tanh(g Wq)             g [B][G] fp32, Wq [H][G][Kd] read in place as [G][H*Kd]
//                                        -> q and qs = q / sqrt(Kd) (both [B][H*Kd])
//   backward  dqpre = dqs s (1 - q^2)    applied while the operand tile is staged (never stored)
//             dg   = dqpre Wq^T          [B][H*Kd] x [H*Kd][G]
//             dWq += g^T dqpre           [G][B] x [B][H*Kd], accumulated into the [H][G][Kd] gradient
//
// These replace, per block, ~35 PyTorch launches of the bf16 hi/lo split form (casts, subtractions,
// concatenations, a split-K MFMA GEMM and its reduction, the permuted gradient adds).  Plain fp32 FMA
// (exact fp32 accumulation): the products are 67-134 MFLOP each.  The work is spread as split-K: a
// 32 x 32 output tile per 64-thread workgroup (4 x 4 per thread) over a 64-deep K slice, partial sums to
// a [S][M][N] workspace, then one finishing pass sums the S slices in a fixed order (deterministic) and
// applies the epilogue (store / tanh + scale / permuted accumulate).
#include "common.h"

namespace {
constexpr int TM = 32, TN = 32, TK = 32, KSLICE = 64;

enum AMode { A_ROW = 0, A_COL = 1, A_DQPRE = 2 };          // A[m][k] / A[k][m] / dqs (1 - q^2) s, [M][K]
enum BMode { B_WQ = 1, B_WQT = 2, B_DQPRE = 3 };           // Wq as [G][H Kd] / as [H Kd][G] / dqpre [K][N]

struct SgArgs {
  const float* a;
  const float* a2;
  const float* b;
  const float* b2;
  int lda, G, Kd;
  float s;
  float* part;          // [S][M][N]
  int M, N, K;
};

template <int AM, int BM_>
__global__ void __launch_bounds__(64) sgemm_part_kernel(SgArgs p) {
  __shared__ float as[TK][TM + 1];
  __shared__ float bs[TK][TN + 1];
  const int tid = threadIdx.x, tx = tid & 7, ty = tid >> 3;     // 8 x 8 threads, 4 x 4 outputs each
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  const int k_begin = blockIdx.z * KSLICE, k_end = min(p.K, k_begin + KSLICE);
  // this thread always stages column cc (m for A, n for B) of rows r0 + 2 i: per-column terms once
  const int cc = tid & 31, r0 = tid >> 5;
  const int am = m0 + cc, bn = n0 + cc;
  const bool am_ok = am < p.M, bn_ok = bn < p.N;
  size_t bcol = 0;
  if (BM_ == B_WQ) bcol = ((size_t)(bn / p.Kd) * p.G) * p.Kd + bn % p.Kd;     // + k Kd
  if (BM_ == B_WQT) bcol = (size_t)bn * p.Kd;                                 // + (k / Kd) G Kd + k % Kd
  float acc[4][4] = {};
  for (int k0 = k_begin; k0 < k_end; k0 += TK) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = r0 + 2 * i;
      const int k = k0 + r;
      const bool kok = k < k_end;
      float av = 0.f, bv = 0.f;
      if (kok && am_ok) {
        if (AM == A_ROW) av = p.a[(size_t)am * p.lda + k];
        if (AM == A_COL) av = p.a[(size_t)k * p.lda + am];
        if (AM == A_DQPRE) {
          const size_t o = (size_t)am * p.K + k;
          const float qq = p.a2[o];
          av = p.a[o] * p.s * (1.f - qq * qq);
        }
      }
      if (kok && bn_ok) {
        if (BM_ == B_WQ) bv = p.b[bcol + (size_t)k * p.Kd];
        if (BM_ == B_WQT) bv = p.b[bcol + (size_t)(k / p.Kd) * p.G * p.Kd + k % p.Kd];
        if (BM_ == B_DQPRE) {
          const size_t o = (size_t)k * p.N + bn;
          const float qq = p.b2[o];
          bv = p.b[o] * p.s * (1.f - qq * qq);
        }
      }
      as[r][cc] = av;
      bs[r][cc] = bv;
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < TK; ++kk) {
      float a4[4], b4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a4[i] = as[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b4[j] = bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a4[i], b4[j], acc[i][j]);
    }
    __syncthreads();
  }
  float* out = p.part + (size_t)blockIdx.z * p.M * p.N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n < p.N) out[(size_t)m * p.N + n] = acc[i][j];
    }
  }
}

// sum the S slices in order, then: epi 0 c[m][n] = v; 1 c = tanh(v), c2 = tanh(v) s; 2 c[(h G + m) Kd + kd] += v
__global__ void __launch_bounds__(256) sgemm_finish_kernel(const float* __restrict__ part, int S, int M, int N,
                                                           int epi, float* __restrict__ c, float* __restrict__ c2,
                                                           float s, int G, int Kd) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * N) return;
  float v = 0.f;
  for (int z = 0; z < S; ++z) v += part[(size_t)z * M * N + idx];
  if (epi == 0) {
    c[idx] = v;
  } else if (epi == 1) {
    const float t = tanhf(v);
    c[idx] = t;
    c2[idx] = t * s;
  } else {
    const int m = idx / N, n = idx - m * N;
    c[((size_t)(n / Kd) * G + m) * Kd + n % Kd] += v;
  }
}

template <int AM, int BM_>
int run(SgArgs p, int epi, float* c, float* c2, hipStream_t st) {
  if (p.M < 1 || p.N < 1 || p.K < 1 || p.G < 1 || p.Kd < 1) return (int)hipErrorInvalidValue;
  const int S = (p.K + KSLICE - 1) / KSLICE;
  hipLaunchKernelGGL((sgemm_part_kernel<AM, BM_>), dim3((p.N + TN - 1) / TN, (p.M + TM - 1) / TM, S), dim3(64), 0, st,
                     p);
  hipLaunchKernelGGL(sgemm_finish_kernel, dim3((p.M * p.N + 255) / 256), dim3(256), 0, st, p.part, S, p.M, p.N, epi,
                     c, c2, p.s, p.G, p.Kd);
  return pbx_launch_status();
}
}  // namespace

// workspace floats needed by the three launchers below: ceil(K / 64) * M * N of the largest product
PBX_EXPORT int pbx_sg_query_ws(int B, int G, int H, int Kd) {
  const long hk = (long)H * Kd;
  const long fwd = (G + KSLICE - 1) / KSLICE * (long)B * hk;
  const long dg = (hk + KSLICE - 1) / KSLICE * (long)B * G;
  const long dw = (B + KSLICE - 1) / KSLICE * (long)G * hk;
  const long mx = fwd > dg ? (fwd > dw ? fwd : dw) : (dg > dw ? dg : dw);
  return mx < 0x7fffffffL ? (int)mx : -1;
}

// q = tanh(g Wq), qs = q s:  g [B][G], Wq [H][G][Kd] -> q, qs [B][H*Kd]
PBX_EXPORT int pbx_sg_query_fwd(const float* g, const float* wq, float* q, float* qs, float* ws, int B, int G, int H,
                                int Kd, float s, hipStream_t st) {
  SgArgs p{g, nullptr, wq, nullptr, G, G, Kd, s, ws, B, H * Kd, G};
  return run<A_ROW, B_WQ>(p, 1, q, qs, st);
}

// dg = dqpre Wq^T with dqpre = dqs s (1 - q^2):  dqs, q [B][H*Kd] -> dg [B][G]
PBX_EXPORT int pbx_sg_query_dg(const float* dqs, const float* q, const float* wq, float* dg, float* ws, int B, int G,
                               int H, int Kd, float s, hipStream_t st) {
  SgArgs p{dqs, q, wq, nullptr, 0, G, Kd, s, ws, B, G, H * Kd};
  return run<A_DQPRE, B_WQT>(p, 0, dg, nullptr, st);
}

// dWq[h][g][kd] += sum_b g[b][g] dqpre[b][h Kd + kd]:  g [B][G], dqs, q [B][H*Kd], dwq [H][G][Kd]
PBX_EXPORT int pbx_sg_query_dwq(const float* g, const float* dqs, const float* q, float* dwq, float* ws, int B, int G,
                                int H, int Kd, float s, hipStream_t st) {
  SgArgs p{g, nullptr, dqs, q, G, G, Kd, s, ws, G, H * Kd, B};
  return run<A_COL, B_DQPRE>(p, 2, dwq, nullptr, st);
}

// ------------------------------------------------------------------------------------------------
// The fused attention kernels' K/V weight image and the K/V weight-gradient scatter, one launch each
// (replacing a permute-cat-cast chain of three PyTorch launches and two strided adds per block).
namespace {
__global__ void __launch_bounds__(256) pa_wimg_kernel(const float* __restrict__ wk, const float* __restrict__ wv,
                                                      unsigned short* __restrict__ img, int H, int C, int K, int VD) {
  // img [H][K + VD][C] bf16: row j < K is Wk[h][:, j], row K + j is Wv[h][:, j]
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long n = (long)H * (K + VD) * C;
  if (idx >= n) return;
  const int c = (int)(idx % C);
  const long hr = idx / C;
  const int r = (int)(hr % (K + VD)), h = (int)(hr / (K + VD));
  const float v = r < K ? wk[((size_t)h * C + c) * K + r] : wv[((size_t)h * C + c) * VD + (r - K)];
  img[idx] = f2bf(v);
}

__global__ void __launch_bounds__(256) pa_dwkv_add_kernel(const float* __restrict__ dwcat, float* __restrict__ dwk,
                                                          float* __restrict__ dwv, int H, int C, int K, int VD) {
  // dwcat [C][H K + H VD]: dWk[h][c][k] += dwcat[c][h K + k], dWv[h][c][v] += dwcat[c][H K + h VD + v]
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long nk = (long)H * C * K, n = nk + (long)H * C * VD;
  if (idx >= n) return;
  const int N = H * (K + VD);
  if (idx < nk) {
    const int k = (int)(idx % K);
    const long hc = idx / K;
    const int c = (int)(hc % C), h = (int)(hc / C);
    dwk[idx] += dwcat[(size_t)c * N + h * K + k];
  } else {
    const long j = idx - nk;
    const int v = (int)(j % VD);
    const long hc = j / VD;
    const int c = (int)(hc % C), h = (int)(hc / C);
    dwv[j] += dwcat[(size_t)c * N + H * K + h * VD + v];
  }
}
}  // namespace

PBX_EXPORT int pbx_pa_wimg(const float* wk, const float* wv, void* img, int H, int C, int K, int VD, hipStream_t st) {
  const long n = (long)H * (K + VD) * C;
  if (n <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pa_wimg_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, wk, wv,
                     (unsigned short*)img, H, C, K, VD);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_pa_dwkv_add(const float* dwcat, float* dwk, float* dwv, int H, int C, int K, int VD,
                               hipStream_t st) {
  const long n = (long)H * C * (K + VD);
  if (n <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pa_dwkv_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dwcat, dwk, dwv, H, C,
                     K, VD);
  return pbx_launch_status();
}
