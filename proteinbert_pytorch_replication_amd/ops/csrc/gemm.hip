// In-tree MFMA GEMMs for the small / skinny library-shaped products of ProteinBERT:
// the [B, 8943] x [8943, 512] GO-input and GO-output products, their weight gradients (a K = B
// reduction) and the global-track weight gradients dW = dU^T X.  hipBLASLt ran these at 10-66 us
// per call (profiles/r2_v8_concurrent_steps.txt); they are M,N <= 9k, K <= 9k, bf16 operands with
// fp32 accumulation.
//
//   C[M][N] (+)= sum_k op(A)[m][k] op(B)[k][n]
//   TA = 0: A[m][k] = A[m * lda + k]     TA = 1: A[m][k] = A[k * lda + m]
//   TB = 0: B[k][n] = B[k * ldb + n]     TB = 1: B[k][n] = B[n * ldb + k]
//
// Tile 128 x 128 per workgroup (4 waves, 64 x 64 each = 2 x 2 v_mfma_f32_32x32x16_bf16 tiles), K in
// chunks of 128.  Both operands are staged through LDS as 256-B-row swizzled tiles (mfma.h swz256):
// the operand whose K runs along memory is stored [m|n][k] and read by rows (ds_read_b128); the other
// is stored [k][m|n] and read transposed (ds_read_b64_tr_b16), so every layout is one coalesced 16-B
// global load per lane and conflict-free LDS reads.  The next K chunk is loaded into registers while
// the current one is in the MFMAs.  Split-K (grid.z) writes fp32 partial slabs that pbx_gemm_reduce
// sums in a fixed order: every result is deterministic (no float atomics).
//
// EPI_GO: the GO-annotation head of the reference loss fused into the GEMM epilogue
// (ProteinBERT/modules.py:286-293, utils.py:294): z = acc + bias, p = sigmoid(z), BCE(p, y) with
// PyTorch's log clamp (>= -100), weighted by w[b] / (B A); writes dz = dL/dz (bf16, the operand of
// the backward GEMMs), per-(row tile, column) partial sums of dz (the bias gradient, folded by the
// caller) and per-workgroup loss partials.  z itself is never stored.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int BT = 128;   // tile rows / cols
constexpr int BK = 128;   // K chunk
constexpr int TILE = BT * 256;   // bytes of one staged operand tile

enum { EPI_STORE = 0, EPI_GO = 1 };

struct GoArgs {
  const float* bias;      // [N]
  const float* y;         // [M][ldy] targets
  long ldy;
  const float* wrow;      // per-row weight (w[b]) ...
  const float* wfull;     // ... or a full [M][ldy] weight (one of the two)
  bf16_t* dz;             // [M][lddz]
  long lddz;
  float* dbias_part;      // [ceil(M / BT)][N]
  float* loss_part;       // [gridDim.x * gridDim.y]
  float inv_mn;           // 1 / (M N)
};

// One operand tile (rows r0.., K chunk k0..) into LDS.  KMAJ: K runs along memory (A row / B col) ->
// LDS [row][k]; else -> LDS [k][row].  ALIGNED: 16-B vector loads (ld % 8 == 0, 16-B base).
template <bool KMAJ, bool ALIGNED>
struct Stager {
  uint4 v[8];   // 2048 16-B chunks per tile / 256 threads
  __device__ __forceinline__ void load(const bf16_t* __restrict__ p, long ld, int rows, int K, int r0, int k0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int a = idx >> 4, c = (idx & 15) * 8;   // LDS row a, 8-element chunk c
      // KMAJ: row = r0 + a, k = k0 + c.. ; else: k = k0 + a, row = r0 + c..
      const int row = KMAJ ? r0 + a : r0 + c;
      const int kk = KMAJ ? k0 + c : k0 + a;
      if (ALIGNED) {
        const bool ok = KMAJ ? (row < rows && kk < K) : (kk < K && row < rows);
        // the chunk is entirely valid or entirely outside (rows / K multiples of 8 on this path)
        v[i] = ok ? *reinterpret_cast<const uint4*>(p + (KMAJ ? (size_t)row * ld + kk : (size_t)kk * ld + row))
                  : make_uint4(0u, 0u, 0u, 0u);
      } else {
        unsigned short e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int rr = KMAJ ? row : row + j, kj = KMAJ ? kk + j : kk;
          e[j] = (rr < rows && kj < K) ? p[KMAJ ? (size_t)rr * ld + kj : (size_t)kj * ld + rr] : (unsigned short)0;
        }
        v[i] = make_uint4(e[0] | (unsigned)e[1] << 16, e[2] | (unsigned)e[3] << 16, e[4] | (unsigned)e[5] << 16,
                          e[6] | (unsigned)e[7] << 16);
      }
    }
  }
  __device__ __forceinline__ void store(unsigned char* t) const {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = threadIdx.x + 256 * i;
      *reinterpret_cast<uint4*>(t + swz256(idx >> 4, idx & 15)) = v[i];
    }
  }
};

// MFMA operand fragment of row/col block `blk` (32 wide) at k-step kk from a staged tile
template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag(const unsigned char* t, int blk, int kk, int r, int h, int q, int tc) {
  if (KMAJ) return lds_frag(t, swz256(blk * 32 + r, kk * 2 + h));
  const int rlo = kk * 16 + 8 * h + q;
  const int col = blk * 32 + tc;
  return cat_tr(lds_tr(t, swz256e(rlo, col)), lds_tr(t, swz256e(rlo + 4, col)));
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_reduce_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// The K loop of one 128 x 128 output tile (rows m0.., cols n0.., K chunks kc0 .. kc1) into acc.
template <int TA, int TB, bool AL_A, bool AL_B>
__device__ __forceinline__ void gemm_mainloop(f32x16_t (&acc)[2][2], unsigned char* smem, const bf16_t* __restrict__ A,
                                              long lda, const bf16_t* __restrict__ B, long ldb, int M, int N, int K,
                                              int m0, int n0, int kc0, int kc1) {
  unsigned char* As = smem;
  unsigned char* Bs = smem + TILE;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int wm = w >> 1, wn = w & 1;
  constexpr bool AK = TA == 0, BKM = TB == 1;     // K runs along memory
  Stager<AK, AL_A> sa;
  Stager<BKM, AL_B> sb;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();
  if (kc0 < kc1) {
    sa.load(A, lda, M, K, m0, kc0 * BK);
    sb.load(B, ldb, N, K, n0, kc0 * BK);
  }
  for (int kc = kc0; kc < kc1; ++kc) {
    __syncthreads();                       // previous chunk's fragments consumed
    sa.store(As);
    sb.store(Bs);
    __syncthreads();
    if (kc + 1 < kc1) {                    // next chunk in flight during the MFMAs
      sa.load(A, lda, M, K, m0, (kc + 1) * BK);
      sb.load(B, ldb, N, K, n0, (kc + 1) * BK);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const bf16x8 a0 = frag<AK>(As, wm * 2, kk, r, h, q, tc), a1 = frag<AK>(As, wm * 2 + 1, kk, r, h, q, tc);
      const bf16x8 b0 = frag<BKM>(Bs, wn * 2, kk, r, h, q, tc), b1 = frag<BKM>(Bs, wn * 2 + 1, kk, r, h, q, tc);
      acc[0][0] = mfma32(a0, b0, acc[0][0]);
      acc[0][1] = mfma32(a0, b1, acc[0][1]);
      acc[1][0] = mfma32(a1, b0, acc[1][0]);
      acc[1][1] = mfma32(a1, b1, acc[1][1]);
    }
  }
}

// D layout: lane (r, h), register e -> row (e & 3) + 8 (e >> 2) + 4 h, column r of each 32 x 32 tile.
// accumulate: all 64 reads of C are issued before the first store (C is not restrict, so a fused
// load-add-store per element serialises 64 memory round trips: 42 vs 15 us on a cold 512^3 GEMM)
__device__ __forceinline__ void gemm_store(f32x16_t (&acc)[2][2], float* dst, long ldc, int M, int N, int m0, int n0,
                                           int accumulate) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  if (accumulate) {
    float old[2][2][16];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 64 + j * 32 + r;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          old[i][j][e] = (n < N && m < M) ? __builtin_nontemporal_load(dst + (size_t)m * ldc + n) : 0.f;
        }
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] += old[i][j][e];
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + r;
      if (n >= N) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m < M) dst[(size_t)m * ldc + n] = acc[i][j][e];
      }
    }
}

template <int TA, int TB, bool AL_A, bool AL_B, int EPI>
__global__ void __launch_bounds__(256, 2) gemm_kernel(const bf16_t* __restrict__ A, long lda, const bf16_t* __restrict__ B,
                                                      long ldb, float* __restrict__ C, long ldc, int M, int N, int K,
                                                      int kchunks_per_split, int accumulate, GoArgs go) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * BT, n0 = blockIdx.x * BT;
  const int nkc = (K + BK - 1) / BK;
  const int kc0 = blockIdx.z * kchunks_per_split;
  const int kc1 = min(nkc, kc0 + kchunks_per_split);
  f32x16_t acc[2][2];
  gemm_mainloop<TA, TB, AL_A, AL_B>(acc, smem, A, lda, B, ldb, M, N, K, m0, n0, kc0, kc1);
  if constexpr (EPI == EPI_STORE) {
    gemm_store(acc, C + (size_t)blockIdx.z * M * ldc, ldc, M, N, m0, n0, accumulate);   // split-K slab z
  } else {
    // GO head.  The 128 x 128 fp32 tile goes through LDS (row stride 132 floats) so the epilogue
    // runs on row-contiguous 8-column chunks: 2 x 16-B loads of y, one 16-B dz store, per thread a fixed
    // 8-column group (tid & 15) over 8 rows -> column sums in registers, folded over the 16 row groups
    constexpr int TS = BT + 4;
    float* ft = reinterpret_cast<float*>(smem);
    __syncthreads();                                  // staging tiles no longer read
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          ft[(wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h) * TS + wn * 64 + j * 32 + r] = acc[i][j][e];
    __syncthreads();
    const int c8 = tid & 15, rg = tid >> 4;           // columns n0 + 8 c8 .. +7, rows rg + 16 k
    const int nb = n0 + 8 * c8;
    float bc[8], dcol[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bc[e] = nb + e < N ? go.bias[nb + e] : 0.f;
      dcol[e] = 0.f;
    }
    const bool full = nb + 8 <= N && (go.ldy % 4) == 0 && ((uintptr_t)go.y & 15) == 0;
    const bool dzv = (go.lddz % 8) == 0 && ((uintptr_t)go.dz & 15) == 0;
    float lsum = 0.f;
#pragma unroll 2
    for (int k = 0; k < 8; ++k) {
      const int rl = rg + 16 * k, m = m0 + rl;
      if (m >= M) break;
      const float4 z0 = *reinterpret_cast<const float4*>(ft + rl * TS + 8 * c8);
      const float4 z1 = *reinterpret_cast<const float4*>(ft + rl * TS + 8 * c8 + 4);
      const float zz[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
      float yy[8], wv[8];
      const float* yrow = go.y + (size_t)m * go.ldy + nb;
      if (full) {
        const float4 a = *reinterpret_cast<const float4*>(yrow), b = *reinterpret_cast<const float4*>(yrow + 4);
        yy[0] = a.x; yy[1] = a.y; yy[2] = a.z; yy[3] = a.w; yy[4] = b.x; yy[5] = b.y; yy[6] = b.z; yy[7] = b.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) yy[e] = nb + e < N ? yrow[e] : 0.f;
      }
      if (go.wrow != nullptr) {
        const float wr = go.wrow[m];
#pragma unroll
        for (int e = 0; e < 8; ++e) wv[e] = wr;
      } else {
        const float* wr = go.wfull + (size_t)m * go.ldy + nb;
#pragma unroll
        for (int e = 0; e < 8; ++e) wv[e] = nb + e < N ? wr[e] : 0.f;
      }
      float g[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float p = 1.0f / (1.0f + __expf(-(zz[e] + bc[e])));
        const float lp = fmaxf(__logf(p), -100.f), l1p = fmaxf(__logf(1.0f - p), -100.f);
        const bool ok = nb + e < N;
        lsum += ok ? wv[e] * -(yy[e] * lp + (1.0f - yy[e]) * l1p) * go.inv_mn : 0.f;
        const float pq = p * (1.0f - p);
        g[e] = ok ? wv[e] * go.inv_mn * (p - yy[e]) * pq / fmaxf(pq, 1e-12f) : 0.f;
      }
      const uint4 q = packq8(g);
      if (dzv && nb + 8 <= go.lddz) {                // pad columns [N, lddz) are written as zeros
        *reinterpret_cast<uint4*>(go.dz + (size_t)m * go.lddz + nb) = q;
      } else {
        const unsigned short* qs = reinterpret_cast<const unsigned short*>(&q);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (nb + e < go.lddz) go.dz[(size_t)m * go.lddz + nb + e] = qs[e];
      }
      float gr[8];
      unpack8(q, gr);                                // the bias gradient sums the stored (bf16) dz
#pragma unroll
      for (int e = 0; e < 8; ++e) dcol[e] += gr[e];
    }
    // column sums over the 16 row groups: through LDS (reuse the tile after a barrier)
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) ft[rg * TS + 8 * c8 + e] = dcol[e];
    __syncthreads();
    if (tid < BT) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) a += ft[k * TS + tid];
      const int n = n0 + tid;
      if (n < N) go.dbias_part[(size_t)blockIdx.y * N + n] = a;
    }
    float* red = ft + 16 * TS;
    const float lt = block_sum256(lsum, red);
    if (tid == 0) go.loss_part[blockIdx.y * gridDim.x + blockIdx.x] = lt;
  }
}

// C[m][n] (+)= sum_z slab[z][m][n]  (fixed order); VEC: N and ldc multiples of 4 (16-B accesses)
template <bool VEC>
__global__ void __launch_bounds__(256) gemm_reduce_kernel(const float* __restrict__ slab, int S, float* __restrict__ C,
                                                          long ldc, int M, int N, int accumulate) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long n4 = (N + 3) / 4;
  if (idx >= (long)M * n4) return;
  const int m = (int)(idx / n4), n = (int)(idx - (idx / n4) * n4) * 4;
  if (VEC) {
    const size_t zs = (size_t)M * N;
    const float4* p = reinterpret_cast<const float4*>(slab + (size_t)m * N + n);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int z = 0;
    for (; z + 4 <= S; z += 4) {                 // four slabs in flight per step, summed in slab order
      const float4 a = p[(z * zs) / 4], b = p[((z + 1) * zs) / 4], c = p[((z + 2) * zs) / 4],
                   d = p[((z + 3) * zs) / 4];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
      s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
      s.x += c.x; s.y += c.y; s.z += c.z; s.w += c.w;
      s.x += d.x; s.y += d.y; s.z += d.z; s.w += d.w;
    }
    for (; z < S; ++z) {
      const float4 a = p[(z * zs) / 4];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
    float4* c = reinterpret_cast<float4*>(C + (size_t)m * ldc + n);
    if (accumulate) {
      const float4 o = *c;
      s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
    }
    *c = s;
    return;
  }
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int z = 0; z < S; ++z) {
    const float* p = slab + ((size_t)z * M + m) * N + n;
#pragma unroll
    for (int e = 0; e < 4; ++e) s[e] += n + e < N ? p[e] : 0.f;
  }
  float* c = C + (size_t)m * ldc + n;
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (n + e < N) c[e] = accumulate ? c[e] + s[e] : s[e];
}

// Up to 4 independent GEMMs of one transpose / alignment class in ONE launch: grid.z = problem,
// (grid.x, grid.y) = the largest problem's tiles (smaller problems' surplus tiles exit at once).  The
// global-track weight gradients of a block (dW1, dW2, dWgl: K = B rows, accumulated into the arena)
// were three split-K GEMMs + three slab folds on the weight-gradient stream; at K = B = 512 one
// pass per output tile without split-K is cheaper than the slabs, and one launch instead of six.
struct GemmBatch {
  const bf16_t* A[4];
  const bf16_t* B[4];
  float* C[4];
  long lda[4], ldb[4], ldc[4];
  int M[4], N[4], K[4];
};

template <int TA, int TB, bool AL_A, bool AL_B>
__global__ void __launch_bounds__(256, 2) gemm_batch_kernel(GemmBatch gb, int accumulate) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int z = blockIdx.z;
  const int M = gb.M[z], N = gb.N[z], K = gb.K[z];
  const int m0 = blockIdx.y * BT, n0 = blockIdx.x * BT;
  if (m0 >= M || n0 >= N) return;                  // workgroup-uniform
  f32x16_t acc[2][2];
  gemm_mainloop<TA, TB, AL_A, AL_B>(acc, smem, gb.A[z], gb.lda[z], gb.B[z], gb.ldb[z], M, N, K, m0, n0, 0,
                                    (K + BK - 1) / BK);
  gemm_store(acc, gb.C[z], gb.ldc[z], M, N, m0, n0, accumulate);
}

template <int TA, int TB, bool AL_A, bool AL_B>
int launch_batch(const GemmBatch& gb, int n, int accumulate, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_batch_kernel<TA, TB, AL_A, AL_B>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 2 * TILE);
    attr = true;
  }
  int mt = 1, nt = 1;
  for (int i = 0; i < n; ++i) {
    mt = max(mt, (gb.M[i] + BT - 1) / BT);
    nt = max(nt, (gb.N[i] + BT - 1) / BT);
  }
  hipLaunchKernelGGL((gemm_batch_kernel<TA, TB, AL_A, AL_B>), dim3(nt, mt, n), dim3(256), 2 * TILE, st, gb, accumulate);
  return pbx_launch_status();
}

template <int TA, int TB, bool AL_A, bool AL_B, int EPI>
int launch(const void* A, long lda, const void* B, long ldb, float* C, long ldc, int M, int N, int K, int splitk,
           int accumulate, const GoArgs& go, hipStream_t st) {
  constexpr int lds = EPI == EPI_GO ? BT * (BT + 4) * 4 : 2 * TILE;     // GO: the fp32 tile for the epilogue
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_kernel<TA, TB, AL_A, AL_B, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const int nkc = (K + BK - 1) / BK;
  const int per = (nkc + splitk - 1) / splitk;
  const int sk = (nkc + per - 1) / per;   // no empty splits
  dim3 grid((N + BT - 1) / BT, (M + BT - 1) / BT, sk);
  hipLaunchKernelGGL((gemm_kernel<TA, TB, AL_A, AL_B, EPI>), grid, dim3(256), lds, st, (const bf16_t*)A, lda,
                     (const bf16_t*)B, ldb, C, ldc, M, N, K, per, accumulate, go);
  return pbx_launch_status();
}

template <int TA, int TB, int EPI>
int dispatch_al(bool aa, bool ab, const void* A, long lda, const void* B, long ldb, float* C, long ldc, int M, int N,
                int K, int splitk, int accumulate, const GoArgs& go, hipStream_t st) {
  if (aa && ab) return launch<TA, TB, true, true, EPI>(A, lda, B, ldb, C, ldc, M, N, K, splitk, accumulate, go, st);
  if (aa) return launch<TA, TB, true, false, EPI>(A, lda, B, ldb, C, ldc, M, N, K, splitk, accumulate, go, st);
  if (ab) return launch<TA, TB, false, true, EPI>(A, lda, B, ldb, C, ldc, M, N, K, splitk, accumulate, go, st);
  return launch<TA, TB, false, false, EPI>(A, lda, B, ldb, C, ldc, M, N, K, splitk, accumulate, go, st);
}

// 16-B vector loads are legal when the base is 16-B aligned and the leading dimension and the extent
// along the contiguous axis are multiples of 8 elements (a chunk is then wholly in or out of range),
// or the caller guarantees the contiguous axis is zero-padded to a multiple of 8 (`padded`)
bool aligned(const void* p, long ld, int contig_extent, bool padded) {
  return ((size_t)p & 15) == 0 && ld % 8 == 0 && (padded || contig_extent % 8 == 0);
}
}  // namespace

// C (+)= op(A) op(B); splitk > 1: C must be a [splitk][M][N] fp32 scratch slab (ldc = N), then
// pbx_gemm_reduce folds it.  ta / tb: 0 / 1 as in the header comment.  pad bit 0 / 1: A / B is
// zero-padded along its contiguous axis to a multiple of 8 elements (16-B loads may read the pad).
PBX_EXPORT int pbx_gemm(const void* A, long lda, int ta, const void* B, long ldb, int tb, float* C, long ldc, int M, int N,
                        int K, int splitk, int accumulate, int pad, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || splitk < 1 || (splitk > 1 && ldc != N)) return (int)hipErrorInvalidValue;
  const GoArgs go{};
  const bool aa = aligned(A, lda, ta == 0 ? K : M, pad & 1), ab = aligned(B, ldb, tb == 1 ? K : N, pad & 2);
  if (ta == 0 && tb == 0) return dispatch_al<0, 0, EPI_STORE>(aa, ab, A, lda, B, ldb, C, ldc, M, N, K, splitk, accumulate, go, st);
  if (ta == 0 && tb == 1) return dispatch_al<0, 1, EPI_STORE>(aa, ab, A, lda, B, ldb, C, ldc, M, N, K, splitk, accumulate, go, st);
  if (ta == 1 && tb == 0) return dispatch_al<1, 0, EPI_STORE>(aa, ab, A, lda, B, ldb, C, ldc, M, N, K, splitk, accumulate, go, st);
  return dispatch_al<1, 1, EPI_STORE>(aa, ab, A, lda, B, ldb, C, ldc, M, N, K, splitk, accumulate, go, st);
}

PBX_EXPORT int pbx_gemm_reduce(const float* slab, int S, float* C, long ldc, int M, int N, int accumulate,
                               hipStream_t st) {
  const long n = (long)M * ((N + 3) / 4);
  const bool vec = N % 4 == 0 && ldc % 4 == 0 && ((size_t)C & 15) == 0 && ((size_t)slab & 15) == 0;
  hipLaunchKernelGGL(vec ? gemm_reduce_kernel<true> : gemm_reduce_kernel<false>, dim3((unsigned)((n + 255) / 256)),
                     dim3(256), 0, st, slab, S, C, ldc, M, N, accumulate);
  return pbx_launch_status();
}

// Fused GO head (reference semantics): x [M = B][K = G] bf16 row-major, w [N = A][K] bf16 (the head
// weight's bf16 mirror), bias [A] fp32, y [B][ldy] fp32 targets, weights per row (wrow) or full
// (wfull, [B][ldy]).  Outputs: dz [B][lddz] bf16 (columns A .. lddz zeroed), dbias_part
// [ceil(B / 128)][A], loss_part [ceil(B / 128) ceil(A / 128)] (each already divided by B A).
PBX_EXPORT int pbx_go_head_fused(const void* x, long ldx, const void* w, long ldw, const float* bias, const float* y,
                                 long ldy, const float* wrow, const float* wfull, void* dz, long lddz, float* dbias_part,
                                 float* loss_part, int M, int N, int K, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || (wrow == nullptr) == (wfull == nullptr)) return (int)hipErrorInvalidValue;
  GoArgs go{bias, y, ldy, wrow, wfull, (bf16_t*)dz, lddz, dbias_part, loss_part, 1.0f / ((float)M * (float)N)};
  const bool aa = aligned(x, ldx, K, false), ab = aligned(w, ldw, K, false);
  return dispatch_al<0, 1, EPI_GO>(aa, ab, x, ldx, w, ldw, nullptr, 0, M, N, K, 1, 0, go, st);
}

// n (<= 4) GEMMs C_i (+)= op(A_i) op(B_i) of one (ta, tb) class in one launch (no split-K).
// Arrays: A, B, C device pointers; lda, ldb, ldc, M, N, K per problem.
PBX_EXPORT int pbx_gemm_batch(int n, const void* const* A, const long* lda, const void* const* B, const long* ldb,
                              float* const* C, const long* ldc, const int* M, const int* N, const int* K, int ta, int tb,
                              int accumulate, hipStream_t st) {
  if (n < 1 || n > 4) return (int)hipErrorInvalidValue;
  GemmBatch gb{};
  bool aa = true, ab = true;
  for (int i = 0; i < n; ++i) {
    if (M[i] <= 0 || N[i] <= 0 || K[i] <= 0) return (int)hipErrorInvalidValue;
    gb.A[i] = (const bf16_t*)A[i];
    gb.B[i] = (const bf16_t*)B[i];
    gb.C[i] = C[i];
    gb.lda[i] = lda[i];
    gb.ldb[i] = ldb[i];
    gb.ldc[i] = ldc[i];
    gb.M[i] = M[i];
    gb.N[i] = N[i];
    gb.K[i] = K[i];
    aa = aa && aligned(A[i], lda[i], ta == 0 ? K[i] : M[i], false);
    ab = ab && aligned(B[i], ldb[i], tb == 1 ? K[i] : N[i], false);
  }
#define PBX_GB(TA_, TB_)                                                        \
  if (ta == TA_ && tb == TB_) {                                                  \
    if (aa && ab) return launch_batch<TA_, TB_, true, true>(gb, n, accumulate, st);   \
    if (aa) return launch_batch<TA_, TB_, true, false>(gb, n, accumulate, st);        \
    if (ab) return launch_batch<TA_, TB_, false, true>(gb, n, accumulate, st);        \
    return launch_batch<TA_, TB_, false, false>(gb, n, accumulate, st);               \
  }
  PBX_GB(1, 0)
  PBX_GB(0, 0)
  PBX_GB(0, 1)
  PBX_GB(1, 1)
#undef PBX_GB
  return (int)hipErrorInvalidValue;
}
