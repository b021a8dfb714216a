// Conv weight gradient, LDS-DMA pipelined form (SURVEY K3 backward; reference conv layers
// ProteinBERT/modules.py:185-199 -- there it is autograd's cuDNN wgrad).
//
//   dW[co][ci][k] = sum_{b,pos} dy[b][pos][co] * x[b][pos + (k - 4) d][ci],   db[co] = sum dy[b][pos][co]
//
// One workgroup (8 waves, ONE per CU) owns one (conv, 64-co half) "type" and a contiguous run of
// 128-position tiles ("chunk").  Wave w owns input channels 32(w&3).. for both 32-co tiles and
// taps 0-4 (waves 0-3) or 5-8 (waves 4-7): <= 10 x 32x32 fp32 accumulators, so two waves share a
// SIMD within 256 registers each, and every x fragment read from LDS feeds two MFMAs (the previous
// form, one 32-co tile per wave, needed one LDS fragment per MFMA and staged synchronously: ~19 %
// of MFMA peak).  (One wave per SIMD holding all 9 taps = 288 accumulator registers does not fit
// the 256 AGPRs: hipcc shuffles accumulators through VGPR copies around every MFMA.)
//
// Staging is asynchronous global->LDS DMA (global_load_lds_dwordx4, 1 KiB per wave instruction,
// lane-linear destination) into two LDS buffers: the loads of tile t+1 are issued before the MFMAs
// of tile t, and one barrier per tile retires them.  The x tile keeps the swz256 image of the other
// kernels by permuting the per-lane SOURCE chunk (the destination of a DMA cannot be permuted);
// rows outside the sequence (conv zero padding) read a 16-byte zero block.
//
// Partials go to fp32 slabs in tap-major layout [chunk][conv][k][co][ci] (each store instruction
// covers 2 x 128 contiguous bytes); wgrad2_reduce sums the chunks in fixed order (deterministic)
// and adds into the torch layouts [co][ci][k] (the flat-arena .grad views).
#include "mfma.h"
#include <stdlib.h>

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;

constexpr int BM = 128;          // positions per tile
constexpr int KS = 9;

__device__ __attribute__((aligned(16))) unsigned int g_zero16[4];   // zero-initialised device global
__device__ __attribute__((aligned(16))) unsigned int g_ones16[4] = {~0u, ~0u, ~0u, ~0u};   // token -1 (no token)

// One 1-KiB LDS-DMA wave instruction: lane i's 16 source bytes land at lds_base + 16 i.  Issued as
// inline asm so hipcc does not treat every later ds_read as a possible alias of the in-flight DMA
// (with the builtin it waits vmcnt(0) before the first LDS read after the issue, serialising the
// prefetch with the MFMAs); completion is waited explicitly before the barrier that publishes it.
__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_base) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}

// The tile loop of one wave: NTAP taps k0.. of input-channel tile cig, both 32-co tiles.
template <int NTAP, int BIAS, typename StageF>   // BIAS: 0 none, 1 / 2: sum co tile 0 / 1
__device__ __forceinline__ void wgrad_tiles(unsigned char* smem, int buf_bytes, long t0, long t1, StageF& stage,
                                            f32x16_t (&acc0)[5], f32x16_t (&acc1)[5], float& bsum, int halo,
                                            int d, int k0, int cig, int lane) {
  const int h = lane >> 5, q = tr_q(lane), tc = tr_c(lane);
  // LDS byte offsets at kk = 0; K-step kk adds kk * 16 rows (swz256's XOR depends on row & 15 only)
  const int aoff = (8 * h + q) * 64 + tc * 2;
  int xoff[NTAP], xoff4[NTAP];
#pragma unroll
  for (int j = 0; j < NTAP; ++j) {
    const int rb = halo + 8 * h + q + (k0 + j - KS / 2) * d;
    xoff[j] = BM * 128 + swz256e(rb, cig * 32 + tc);
    xoff4[j] = BM * 128 + swz256e(rb + 4, cig * 32 + tc);
  }
  if (t0 < t1) stage(t0, smem);
  for (long tile = t0; tile < t1; ++tile) {
    unsigned char* cur = smem + ((tile - t0) & 1) * buf_bytes;
    unsigned char* nxt = smem + (((tile - t0) & 1) ^ 1) * buf_bytes;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of `cur` landed
    __syncthreads();                                   // ... every wave's; `nxt` no longer read
    if (tile + 1 < t1) stage(tile + 1, nxt);
    // (K-step kk, tap j) steps s = kk * NTAP + j: the x fragment of step s + 2 (and the dy fragments
    // of the next K-step) are read while the MFMA pair of step s runs -- a 3-slot register ring that
    // keeps two LDS reads in flight ahead of the MFMAs without the VGPRs of a whole K-step
    constexpr int NS = (BM / 16) * NTAP;
    bf16x8 fa0[2], fa1[2], fb[3];
    auto read_a = [&](int kk) {
      const unsigned char* c = cur + kk * 16 * 64;     // dy rows advance 16 x 64 B
      fa0[kk & 1] = cat_tr(lds_tr(c, aoff), lds_tr(c, aoff + 256));
      fa1[kk & 1] = cat_tr(lds_tr(c, BM * 64 + aoff), lds_tr(c, BM * 64 + aoff + 256));
    };
    auto read_b = [&](int st) {
      const unsigned char* cx = cur + (st / NTAP) * 16 * 256;   // x rows advance 16 x 256 B
      fb[st % 3] = cat_tr(lds_tr(cx, xoff[st % NTAP]), lds_tr(cx, xoff4[st % NTAP]));
    };
    read_a(0);
    read_b(0);
    read_b(1);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int kk = st / NTAP, j = st % NTAP;
      if (st + 2 < NS) {
        if ((st + 2) % NTAP == 0) read_a((st + 2) / NTAP);
        read_b(st + 2);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (BIAS != 0 && j == 0) {
        typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
        const u32x4 u = __builtin_bit_cast(u32x4, BIAS == 2 ? fa1[kk & 1] : fa0[kk & 1]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          bsum += __builtin_bit_cast(float, u[e] << 16) + __builtin_bit_cast(float, u[e] & 0xffff0000u);
      }
      acc0[j] = mfma32(fa0[kk & 1], fb[st % 3], acc0[j]);
      acc1[j] = mfma32(fa1[kk & 1], fb[st % 3], acc1[j]);
    }
  }
}

// LDS buffer layout: dy sub-tile 0 [BM][64 B] | dy sub-tile 1 [BM][64 B] | x [XRM][256 B] swz256
__global__ void __launch_bounds__(512, 1) wgrad2_kernel(const bf16_t* __restrict__ dy0, const bf16_t* __restrict__ dy1,
                                                        const bf16_t* __restrict__ x, float* __restrict__ slab,
                                                        float* __restrict__ bslab, int B, int L, int dil1,
                                                        int nconv, int R, int buf_bytes, int xlo, int xhi) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ntypes = nconv * 2;
  int type, chunk;
  if ((R & 7) == 0) {
    // the types of one chunk stage the same x rows: ids congruent mod 8 -> one XCD's L2
    const int id = blockIdx.x, j = id >> 3;
    chunk = (j / ntypes) * 8 + (id & 7);
    type = j - (j / ntypes) * ntypes;
  } else {
    chunk = blockIdx.x / ntypes;
    type = blockIdx.x - chunk * ntypes;
  }
  const int cv = type >> 1, half = type & 1;
  const bf16_t* dy = cv ? dy1 : dy0;
  const int d = cv ? dil1 : 1;
  const int halo = (KS / 2) * d;
  const int XR = BM + 2 * halo;               // x rows per tile (multiple of 4: 2*halo = 8d)
  // wave index through readfirstlane: hipcc cannot prove threadIdx.x / 64 uniform, and the staging
  // loop and the tap split branch on it
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  // wave w: input channels (w & 3)*32.. for taps k0 .. k0+NTAP-1 (waves 0-3: taps 0-4, 4-7: taps 5-8)
  const int cig = w & 3;
  const int k0 = w < 4 ? 0 : 5;
  const int ntap = w < 4 ? 5 : 4;     // (the tile loop takes them as template / argument)
  const int T = (L + BM - 1) / BM;
  const long NT = (long)B * T;
  const long t0 = NT * chunk / R, t1 = NT * (chunk + 1) / R;

  // issue the DMA of one tile into buffer `buf` (instructions dealt round-robin to the 8 waves)
  auto stage = [&](long tile, unsigned char* buf) {
    const int b = (int)(tile / T), t = (int)(tile - (tile / T) * T);
    const int pos0 = t * BM;
    const size_t sbase = (size_t)b * L * CH;
    const int n = 16 + XR / 4;
    for (int i = w; i < n; i += 8) {
      if (i < 16) {                            // dy: 16 rows x 64 B per instruction
        const int sub = i >> 3, row = (i & 7) * 16 + (lane >> 2);
        const int pos = pos0 + row;
        const void* src = pos < L ? (const void*)(dy + sbase + (size_t)pos * CH + half * 64 + sub * 32 + (lane & 3) * 8)
                                  : (const void*)g_zero16;
        glds16(src, buf + sub * (BM * 64) + (i & 7) * 1024);
      } else {                                 // x: 4 rows x 256 B per instruction, swz256 image
        const int j = i - 16, row = j * 4 + (lane >> 4);
        const int chunk16 = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
        const int pos = pos0 - halo + row;
        const void* src = (pos >= -xlo && pos < L + xhi)
                              ? (const void*)(x + ((ptrdiff_t)b * (L + xlo + xhi) + xlo + pos) * CH + chunk16 * 8)
                              : (const void*)g_zero16;
        glds16(src, buf + BM * 128 + j * 1024);
      }
    }
  };

  f32x16_t acc0[5], acc1[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    acc0[j] = zero16();
    acc1[j] = zero16();
  }
  float bsum = 0.f;
  // bias partials: wave 0 -> co tile 0, wave 1 -> co tile 1 (summed from their A fragments)
  if (w == 0)
    wgrad_tiles<5, 1>(smem, buf_bytes, t0, t1, stage, acc0, acc1, bsum, halo, d, 0, cig, lane);
  else if (w == 1)
    wgrad_tiles<5, 2>(smem, buf_bytes, t0, t1, stage, acc0, acc1, bsum, halo, d, 0, cig, lane);
  else if (w < 4)
    wgrad_tiles<5, 0>(smem, buf_bytes, t0, t1, stage, acc0, acc1, bsum, halo, d, 0, cig, lane);
  else
    wgrad_tiles<4, 0>(smem, buf_bytes, t0, t1, stage, acc0, acc1, bsum, halo, d, 5, cig, lane);
  // tap-major slab [chunk][conv][k][co][ci]; lane -> ci (32 lanes = 128 contiguous bytes)
  float* dst = slab + ((size_t)chunk * nconv + cv) * KS * CH * CH + cig * 32 + r;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    if (j < ntap) {
      const int k = k0 + j;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int co = half * 64 + (i & 3) + 8 * (i >> 2) + 4 * h;
        dst[((size_t)k * CH + co) * CH] = acc0[j][i];
        dst[((size_t)k * CH + co + 32) * CH] = acc1[j][i];
      }
    }
  }
  if (w < 2) {
    bsum += __shfl_xor(bsum, 32, 64);
    if (h == 0) bslab[((size_t)chunk * nconv + cv) * CH + half * 64 + w * 32 + r] = bsum;
  }
}

// sum the R tap-major slabs (fixed order) and ADD into weight [co][ci][KS] and bias [co].
// 256 threads = 64 float4 columns x 4 R-quarters (8 loads in flight each); the quarters are combined
// through LDS in a fixed order (deterministic).  Blocks >= nblk_w reduce the bias slabs.
__global__ void __launch_bounds__(256) wgrad2_reduce_kernel(const float4* __restrict__ slab,
                                                            const float* __restrict__ bslab, float* __restrict__ dw0,
                                                            float* __restrict__ dw1, float* __restrict__ db0,
                                                            float* __restrict__ db1, int R, int nconv) {
  constexpr int per4 = KS * CH * CH / 4;
  const int total4 = nconv * per4;
  const int nblk_w = (total4 + 63) / 64;
  const int tid = threadIdx.x, col = tid & 63, part = tid >> 6;
  if ((int)blockIdx.x >= nblk_w) {             // bias: one thread per output, R in order
    const int idx = ((int)blockIdx.x - nblk_w) * 256 + tid;
    if (idx < nconv * CH) {
      float s = 0.f;
      for (int rr = 0; rr < R; ++rr) s += bslab[(size_t)rr * nconv * CH + idx];
      float* db = idx >= CH ? db1 : db0;
      if (db != nullptr) db[idx % CH] += s;
    }
    return;
  }
  __shared__ float4 red[4][64];
  const int idx = blockIdx.x * 64 + col;
  const int r0 = R * part / 4, r1 = R * (part + 1) / 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (idx < total4) {
    int rr = r0;
    for (; rr + 8 <= r1; rr += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(size_t)(rr + u) * total4 + idx];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w;
      }
    }
    for (; rr < r1; ++rr) {
      const float4 a = slab[(size_t)rr * total4 + idx];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
  }
  red[part][col] = s;
  __syncthreads();
  if (part == 0 && idx < total4) {
#pragma unroll
    for (int p = 1; p < 4; ++p) {
      const float4 a = red[p][col];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
    const int cv = idx >= per4;
    const int rem = idx - cv * per4;
    const int k = rem / (CH * CH / 4), co = (rem / (CH / 4)) % CH, ci = (rem % (CH / 4)) * 4;
    float* dw = (cv ? dw1 : dw0) + ((size_t)co * CH + ci) * KS + k;
    dw[0] += s.x;
    dw[KS] += s.y;
    dw[2 * KS] += s.z;
    dw[3 * KS] += s.w;
  }
}

bool wgrad2_attr_set = false;
}  // namespace

// KS = 9 only.  slab: R * nconv * 9 * 128 * 128 floats; bslab: R * nconv * 128 floats.
// xlo / xhi: x carries neighbouring shards' rows ([B][xlo + L + xhi][128], context parallelism); 0 / 0 otherwise.
PBX_EXPORT int pbx_wgrad2x(const void* dy0, const void* dy1, const void* x, float* slab, float* bslab, float* dw0,
                           float* dw1, float* db0, float* db1, int B, int L, int dil1, int nconv, int R, int xlo,
                           int xhi, hipStream_t st) {
  if (nconv < 1 || nconv > 2 || R < 1 || dil1 < 1 || xlo < 0 || xhi < 0) return (int)hipErrorInvalidValue;
  const int halo_max = (KS / 2) * (nconv > 1 ? dil1 : 1);
  const int buf = BM * 128 + (BM + 2 * halo_max) * 256;
  if (2 * buf > 163840) return (int)hipErrorInvalidValue;
  if (!wgrad2_attr_set) {
    (void)hipFuncSetAttribute((const void*)wgrad2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    wgrad2_attr_set = true;
  }
  hipLaunchKernelGGL(wgrad2_kernel, dim3(nconv * 2 * R), dim3(512), 2 * buf, st, (const bf16_t*)dy0,
                     (const bf16_t*)dy1, (const bf16_t*)x, slab, bslab, B, L, dil1, nconv, R, buf, xlo, xhi);
  const int total4 = nconv * KS * CH * CH / 4;
  const int nblk = (total4 + 63) / 64 + (nconv * CH + 255) / 256;
  hipLaunchKernelGGL(wgrad2_reduce_kernel, dim3(nblk), dim3(256), 0, st, (const float4*)slab,
                     bslab, dw0, dw1, db0, db1, R, nconv);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_wgrad2(const void* dy0, const void* dy1, const void* x, float* slab, float* bslab, float* dw0,
                          float* dw1, float* db0, float* db1, int B, int L, int dil1, int nconv, int R,
                          hipStream_t st) {
  return pbx_wgrad2x(dy0, dy1, x, slab, bslab, dw0, dw1, db0, db1, B, L, dil1, nconv, R, 0, 0, st);
}

// ------------------------------------------------------------------------------------------------
// Weight gradient of the first block's convolutions, whose input is the token embedding
// x[pos] = bf16(E[tok[pos]]) (reference modules.py:249-253,300 feeding :185-199): through the token
// one-hot instead of the 128 input channels,
//   dW[co][ci][k] = sum_pos dpre[pos][co] x[pos + s_k][ci] = sum_v bf16(E[v][ci]) S_k[v][co],
//   S_k[v][co]    = sum_{src : tok[src] = v} dpre[src - s_k][co]      (s_k = (k - 4) d; zero padding)
// S is a one-hot GEMM (M = 32 token rows, K = source positions, N = 128 channels: a quarter of the
// 128-input-channel product's MFMA work, the embed_bwd pattern of ln.hip with 9 shifted B operands per
// K-step), E^T S is 2 x 9 x 128 x 128 x V.  Same fp32-accumulated sums as wgrad2, in another order;
// deterministic (per-workgroup slab, fixed-order fold).  Replaces the step's exposed tail (the first
// block's wgrad2 runs after every other backward kernel).
namespace {
constexpr int TBM = 128;   // source positions per tile

// Workgroup: 8 waves, wave w = (conv w >> 2, 32-channel tile w & 3), 9 tap accumulators each.
// LDS buffer (double-buffered, DMA-staged): narrow dpre rows [TBM + 8][256 B] | wide dpre rows
// [TBM + 8 d][256 B] (swz256) | the tile's tokens (int64, one 1-KiB DMA)
__global__ void __launch_bounds__(512, 1) wgrad_tok_kernel(const long long* __restrict__ tok,
                                                           const bf16_t* __restrict__ dy0,
                                                           const bf16_t* __restrict__ dy1, float* __restrict__ slab,
                                                           int B, int L, int dil1, int R, int V, int buf_bytes) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int cv = w >> 2, ct = w & 3;
  const int d = cv ? dil1 : 1;
  const int hal0 = KS / 2, hal1 = (KS / 2) * dil1;
  const int rows0 = TBM + 2 * hal0, rows1 = TBM + 2 * hal1;
  const int T = (L + TBM - 1) / TBM;
  const long NT = (long)B * T;
  const long t0 = NT * blockIdx.x / R, t1 = NT * (blockIdx.x + 1) / R;

  auto stage = [&](long tile, unsigned char* buf) {
    const int b = (int)(tile / T), t = (int)(tile - (tile / T) * T);
    const int pos0 = t * TBM;
    const size_t sbase = (size_t)b * L * CH;
    const int n0 = rows0 / 4, n1 = rows1 / 4;
    for (int i = w; i <= n0 + n1; i += 8) {
      if (i == n0 + n1) {                      // tokens pos0 .. pos0 + 127: 2 per lane (L even)
        const int p = pos0 + 2 * lane;
        const void* src = p < L ? (const void*)(tok + (size_t)b * L + p) : (const void*)g_ones16;
        glds16(src, buf + (rows0 + rows1) * 256);
        continue;
      }
      const int c = i >= n0;
      const int j = c ? i - n0 : i;
      const int hal = c ? hal1 : hal0;
      const bf16_t* dy = c ? dy1 : dy0;
      const int row = j * 4 + (lane >> 4);
      const int chunk16 = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
      const int pos = pos0 - hal + row;
      const void* src = (pos >= 0 && pos < L) ? (const void*)(dy + sbase + (size_t)pos * CH + chunk16 * 8)
                                              : (const void*)g_zero16;
      glds16(src, buf + (c ? rows0 * 256 : 0) + j * 1024);
    }
  };

  f32x16_t acc[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) acc[k] = zero16();
  const int hal = cv ? hal1 : hal0;
  const int colb = ct * 32 + tc;
  // per-lane B-fragment byte offsets at k-step 0: B[k = src][col = co] = dpre[src - s_k][co] of tap k is
  // tile row hal + (4 - k) d + kb*16 + 8h + j; swz256's XOR depends on row & 15 only, so k-step kb adds
  // kb * 4096 B (an immediate of the unrolled k-step loop) -- no per-read address arithmetic
  const int cvb = cv ? rows0 * 256 : 0;
  int boff[KS], boff4[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int rb = hal + (KS / 2 - k) * d + 8 * h + q;
    boff[k] = cvb + swz256e(rb, colb);
    boff4[k] = cvb + swz256e(rb + 4, colb);
  }
  const int toff = (rows0 + rows1) * 256 + 8 * h * 8;   // this lane's 8 source tokens (int64) at k-step 0
  if (t0 < t1) stage(t0, smem);
  for (long tile = t0; tile < t1; ++tile) {
    unsigned char* cur = smem + ((tile - t0) & 1) * buf_bytes;
    unsigned char* nxt = smem + (((tile - t0) & 1) ^ 1) * buf_bytes;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of `cur` landed
    __syncthreads();                                   // ... every wave's; `nxt` no longer read
    if (tile + 1 < t1) stage(tile + 1, nxt);
    // (k-step kb, tap k) steps s = kb * 9 + k: the B fragment of step s + 2 is read while the MFMA of
    // step s runs (3-slot ring); the one-hot A operand of k-step kb + 1 (A[i = v][k = src] = [tok == v],
    // lane's v = r; positions >= L were staged as token -1) is built during taps 3..7 of k-step kb
    constexpr int NS = (TBM / 16) * KS;
    bf16x8 fb[3], fa[2];
    unsigned tk[8];
    auto read_b = [&](int st) {
      const unsigned char* c = cur + (st / KS) * 4096;
      fb[st % 3] = cat_tr(lds_tr(c, boff[st % KS]), lds_tr(c, boff4[st % KS]));
    };
    auto read_tok = [&](int kb) {
      const unsigned* tp = reinterpret_cast<const unsigned*>(cur + toff + kb * 128);
#pragma unroll
      for (int j = 0; j < 8; ++j) tk[j] = tp[2 * j];          // low words (tokens < 32, or -1)
    };
    auto make_a = [&](int kb) {
      typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = (tk[2 * e] == (unsigned)r ? 0x3F80u : 0u) | (tk[2 * e + 1] == (unsigned)r ? 0x3F800000u : 0u);
      fa[kb & 1] = __builtin_bit_cast(bf16x8, o);
    };
    read_tok(0);
    make_a(0);
    read_b(0);
    read_b(1);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int kb = st / KS, k = st % KS;
      if (st + 2 < NS) read_b(st + 2);
      if (k == 3 && kb + 1 < TBM / 16) read_tok(kb + 1);
      if (k == 7 && kb + 1 < TBM / 16) make_a(kb + 1);
      __builtin_amdgcn_sched_barrier(0);
      acc[k] = mfma32(fa[kb & 1], fb[st % 3], acc[k]);
    }
  }
  // slab [R][2][KS][V][128]: D row = token v, column = channel
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int v = (i & 3) + 8 * (i >> 2) + 4 * h;
      if (v < V) slab[((((size_t)blockIdx.x * 2 + cv) * KS + k) * V + v) * CH + ct * 32 + r] = acc[k][i];
    }
}

// dW_c[co][ci][k] += sum_v bf16(E[v][ci]) S[c][k][v][co] ; db_c[co] += sum_v S[c][4][v][co]
// (the centre tap reads every position).  One workgroup per (conv, co), thread = ci.
// W0 / W1 / dEslab (the embedding gradient's conv part, pbx_embed_dpre): this workgroup's share of
//   dE[v][ci] = sum_c sum_co sum_k bf16(W_c[co][ci][k]) S[c][k][v][co]
// (the transposed convolution of dpre summed over the source positions with token v) goes to slab row
// blockIdx.x, folded in a fixed order by the caller.
__global__ void __launch_bounds__(128) wgrad_tok_finish_kernel(const float* __restrict__ S, const float* __restrict__ E,
                                                               float* __restrict__ dw0, float* __restrict__ dw1,
                                                               float* __restrict__ db0, float* __restrict__ db1,
                                                               int V, const float* __restrict__ W0,
                                                               const float* __restrict__ W1, float* __restrict__ dEslab) {
  __shared__ float sv[KS * 32];
  const int c = blockIdx.x / CH, co = blockIdx.x % CH, ci = threadIdx.x;
  for (int i = threadIdx.x; i < KS * V; i += 128) {
    const int k = i / V, v = i % V;
    sv[k * 32 + v] = S[(((size_t)c * KS + k) * V + v) * CH + co];
  }
  __syncthreads();
  float o[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) o[k] = 0.f;
  for (int v = 0; v < V; ++v) {
    const float e = bfround(E[v * CH + ci]);
#pragma unroll
    for (int k = 0; k < KS; ++k) o[k] = fmaf(e, sv[k * 32 + v], o[k]);
  }
  float* dw = (c ? dw1 : dw0) + ((size_t)co * CH + ci) * KS;
#pragma unroll
  for (int k = 0; k < KS; ++k) dw[k] += o[k];
  if (ci == 0) {
    float s = 0.f;
    for (int v = 0; v < V; ++v) s += sv[(KS / 2) * 32 + v];
    (c ? db1 : db0)[co] += s;
  }
  if (dEslab != nullptr) {
    const float* wr = (c ? W1 : W0) + ((size_t)co * CH + ci) * KS;
    float wk[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) wk[k] = bfround(wr[k]);
    for (int v = 0; v < V; ++v) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < KS; ++k) a = fmaf(wk[k], sv[k * 32 + v], a);
      dEslab[((size_t)blockIdx.x * V + v) * CH + ci] = a;
    }
  }
}

bool wgrad_tok_attr_set = false;
}  // namespace

extern "C" int pbx_colsum_add(const float* src, int rows, int cols, float* dst, const float* scale, hipStream_t st);
extern "C" int pbx_colsum_set(const float* src, int rows, int cols, float* dst, const float* scale, hipStream_t st);

// Rows of the per-workgroup slab pbx_wgrad_tok needs ([R][2][9][V][128] fp32).
PBX_EXPORT int pbx_wgrad_tok_rows(int B, int L) {
  constexpr int cap = 256;   // (128: +50 % time)
  const long NT = (long)B * ((L + TBM - 1) / TBM);
  return (int)(NT < cap ? NT : cap);
}

// Both convolutions of a block whose input is bf16(E[tok]) (KS = 9, L even, V <= 32): slab as
// pbx_wgrad_tok_rows x 2 x 9 x V x 128 floats, S 2 x 9 x V x 128 floats (scratch); dW / db accumulated.
// W0 / W1 / dE / dEslab (all null, or all set): also dE += the conv part of the embedding gradient (see
// the finish kernel; W_c: the fp32 conv weights [128][128][9]; dEslab: 2 x 128 x V x 128 floats scratch).
PBX_EXPORT int pbx_wgrad_tok(const void* tok, const void* dy0, const void* dy1, const float* E, float* slab, float* S,
                             float* dw0, float* dw1, float* db0, float* db1, int B, int L, int dil1, int V,
                             const float* W0, const float* W1, float* dE, float* dEslab, hipStream_t st) {
  if (V < 1 || V > 32 || dil1 < 1 || (L & 1) || B < 1 || L < 1) return (int)hipErrorInvalidValue;
  if ((dE == nullptr) != (W0 == nullptr) || (dE == nullptr) != (W1 == nullptr) || (dE == nullptr) != (dEslab == nullptr))
    return (int)hipErrorInvalidValue;
  const int buf = (2 * TBM + 8 + 8 * dil1) * 256 + 1024;
  if (2 * buf > 163840) return (int)hipErrorInvalidValue;
  if (!wgrad_tok_attr_set) {
    (void)hipFuncSetAttribute((const void*)wgrad_tok_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    wgrad_tok_attr_set = true;
  }
  const int R = pbx_wgrad_tok_rows(B, L);
  hipLaunchKernelGGL(wgrad_tok_kernel, dim3(R), dim3(512), 2 * buf, st, (const long long*)tok, (const bf16_t*)dy0,
                     (const bf16_t*)dy1, slab, B, L, dil1, R, V, buf);
  const int cols = 2 * KS * V * CH;
  int rc = pbx_colsum_set(slab, R, cols, S, nullptr, st);
  if (rc != 0) return rc;
  hipLaunchKernelGGL(wgrad_tok_finish_kernel, dim3(2 * CH), dim3(128), 0, st, S, E, dw0, dw1, db0, db1, V, W0, W1,
                     dEslab);
  if (dE == nullptr) return pbx_launch_status();
  rc = pbx_launch_status();
  if (rc != 0) return rc;
  return pbx_colsum_add(dEslab, 2 * CH, V * CH, dE, nullptr, st);
}
