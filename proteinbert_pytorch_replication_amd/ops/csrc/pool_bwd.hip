// Attention-pool backward, weight-stationary form (reference semantics).
//
// Reference: ProteinBERT/modules.py:49-60,87-92,219.  In reference semantics every head reduces to
// (1/K) sum_l GELU(h2 Wv_j), so the pool's input gradient is
//   dh2[b][pos][c] = dh2_in[b][pos][c] + sum_j Wv[j][c] dv[b][j] GELU'(h2[b][pos] . Wv[j])
// with GELU' stored by the forward (ln.hip ln_attn_fwd2, `gfrag`: bf16 MFMA B-operand fragments).
//
// Why a second form next to attn_bwd2 (ln.hip): attn_bwd2 keeps the whole [512 x 128] Wv in LDS
// (128 KB, one workgroup per CU, nothing else co-resident) and re-scales every streamed GELU'
// fragment by dv on the VALU (unpack, 8 multiplies, repack per fragment): 132 us alone, ~200 us beside
// the aux-stream conv weight gradient it cannot share a CU with, MFMA busy 0.11.
//
// Here dv is folded into the STATIONARY operand instead: a workgroup owns tiles of ONE sample, so
// A = (Wv^T diag(dv_b)) is built once per workgroup and held in registers -- wave w keeps the 32-channel
// slice c = 32w..32w+31 (NJ/16 fragments, 128 VGPRs at NJ = 512) -- and the streamed GELU' tile is the
// MFMA B operand exactly as the forward wrote it, with no VALU on the hot path.  A 32-position tile's
// GELU' fragments (NJ/16 x 1 KiB) are shared by the 4 waves: they arrive by global->LDS DMA into a
// double buffer (2 x 32 KB), so the next tile streams in while this one runs its MFMAs; the epilogue
// operands (dh2_in, s2 rows, LN2 gamma) are loaded at the top of the tile and land during its MFMAs.  64 KB of LDS and
// <= 256 VGPRs: two workgroups per CU, and a CU keeps room for a co-resident weight-gradient workgroup.
//
// Work: grid (nsplit, B); workgroup (s, b) owns the 32-position tiles [s tpw, (s+1) tpw) of sample b.
// LayerNorm-2 backward partials are written per (tile, wave): sums2[b][4 TW][2], TW = ceil(L / 32).
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int BML = 32;    // tile of the s2 (mean, M2) partials written by ln_linear_fwd (ln.hip)

// one 1-KiB global->LDS DMA wave instruction (lane i's 16 bytes land at lds_base + 16 i); inline asm
// so hipcc does not make later ds_reads wait for it.  Retires in vmcnt order with the wave's loads.
__device__ __forceinline__ void glds16_p(const void* src, unsigned char* lds_base) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

struct EpiOps {            // one lane's epilogue operands of one tile: 4 groups of 4 channels
  uint2 d[4], s[4];
  float4 g[4];
};

// CONSTS (a workgroup owns a whole sample, tpw >= ceil(L / 32)): the workgroup also writes the sample's
// LayerNorm-2 / LayerNorm-1 backward constants consts[b] = (mean2, rstd2, m1, m2, mean1, rstd1, 0, 0) --
// what ln2_consts_kernel (ln.hip) derives from the per-tile partials in a launch of its own -- and zeroes
// row b of the [B, 128] accumulator the LN1 finalize adds into.  m1 / m2 sum the waves' per-tile partials
// in a fixed order (deterministic).
template <int NJT, bool CONSTS>
__global__ void __launch_bounds__(256, 2) attn_bwd4_kernel(
    const bf16x8* __restrict__ gfrag, const bf16_t* __restrict__ s2, const float* __restrict__ st2,
    const float* __restrict__ g2, const bf16_t* __restrict__ dh2_in, const float* __restrict__ dv,
    const bf16x8* __restrict__ wvt, bf16_t* __restrict__ dh2, float* __restrict__ sums2, int L, int tpw,
    float eps, const float* __restrict__ st1, int T1, int BM1, float* __restrict__ consts, float* __restrict__ zero128) {
  constexpr int NJ = NJT * 32;
  constexpr int NF = 2 * NJT;                 // 16-deep k-steps (1-KiB fragments) per tile
  constexpr int FPW = NF / 4;                 // fragments each wave DMAs per tile
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];   // 2 x NF KiB
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int b = blockIdx.y;
  const int TW = (L + 31) / 32;
  const int TWG = 2 * ((L + 63) / 64);        // 32-position tiles per sample in gfrag
  const int T2 = (L + BML - 1) / BML;
  const int t0 = blockIdx.x * tpw;
  const int t1 = min(t0 + tpw, TW);
  if (t0 >= TW) return;                       // workgroup-uniform
  const bf16x8* gs = gfrag + (size_t)b * TWG * NF * 64 + w * FPW * 64 + lane;
  auto dma = [&](int t, int buf) {
    const bf16x8* src = gs + (size_t)t * NF * 64;
    unsigned char* dst = smem + buf * NF * 1024 + w * FPW * 1024;
#pragma unroll
    for (int k = 0; k < FPW; ++k) glds16_p(src + k * 64, dst + k * 1024);
  };
  const bf16_t* dsrc = dh2_in != nullptr ? dh2_in : s2;   // branch-free loads; masked by dmask
  const float dmask = dh2_in != nullptr ? 1.f : 0.f;
  auto epi_load = [&](int t, EpiOps& e) {
    const int pc = min(t * 32 + r, L - 1);
    const size_t roff = ((size_t)b * L + pc) * CH;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ci0 = w * 32 + 8 * g + 4 * h;
      e.d[g] = *reinterpret_cast<const uint2*>(dsrc + roff + ci0);
      e.s[g] = *reinterpret_cast<const uint2*>(s2 + roff + ci0);
      e.g[g] = *reinterpret_cast<const float4*>(g2 + (size_t)pc * CH + ci0);
    }
  };
  dma(t0, 0);
  // per-sample store windows (num_records = the sample's bytes; out-of-range lanes' stores are dropped)
  const __amdgpu_buffer_rsrc_t dh2r =
      __builtin_amdgcn_make_buffer_rsrc(dh2 + (size_t)b * L * CH, (short)0, L * CH * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t sumr =
      __builtin_amdgcn_make_buffer_rsrc(sums2 + (size_t)b * TW * 8, (short)0, TW * 32, 0x00020000);

  // stationary operand: A[c][j] = Wv[j][c] dv[b][j] for c = 32w + r, from the packed Wv^T fragments
  // (pbx_pack_wvt_frag: k-step i, element jj <-> j = 16 i + 8 (jj >> 2) + 4 h + (jj & 3), the K order
  // of the stored GELU' fragments), scaled by dv in fp32 and rounded once
  bf16x8 a[NF];
  {
    // dv row of sample b: lane l holds dv[8 l .. 8 l + 7]; fragment i takes its 8 factors from lanes
    // 2i (j = 16i..16i+7) and 2i+1 (16i+8..) by readlane (wave-uniform lane index): 8 VGPRs, not 256
    const float* dvb = dv + (size_t)b * NJ + 8 * (lane & (NJ / 8 - 1));
    const float4 dl = *reinterpret_cast<const float4*>(dvb), dh = *reinterpret_cast<const float4*>(dvb + 4);
    const float dreg[8] = {dl.x, dl.y, dl.z, dl.w, dh.x, dh.y, dh.z, dh.w};
    const uint4* wp = reinterpret_cast<const uint4*>(wvt) + (size_t)w * NF * 64 + lane;
#pragma unroll
    for (int i = 0; i < NF; ++i) a[i] = __builtin_bit_cast(bf16x8, wp[i * 64]);
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      float v[8];
      unpack8(__builtin_bit_cast(uint4, a[i]), v);
      float d8[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // element e (j = 16i + 4h + e) and 4 + e (j = 16i + 8 + 4h + e)
        const float a0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dreg[e]), 2 * i));
        const float a1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dreg[4 + e]), 2 * i));
        const float b0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dreg[e]), 2 * i + 1));
        const float b1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dreg[4 + e]), 2 * i + 1));
        d8[e] = h ? a1 : a0;
        d8[4 + e] = h ? b1 : b0;
      }
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) v[jj] *= d8[jj];
      a[i] = pack8(v);
      __builtin_amdgcn_sched_barrier(0);      // keep the 16 readlanes of a fragment next to their use
    }
  }
  float mean, rstd;
  wave_ln_stats(st2 + (size_t)b * T2 * 2, T2, BML, L, CH, eps, mean, rstd);
  float wsa = 0.f, wsc = 0.f;                 // CONSTS: this wave's partial sums over the sample's tiles

  auto step = [&](int t, int buf) {
    // this wave's DMA of tile t has landed: after it the wave issued only tile t-1's epilogue loads
    // (consumed, so already waited for) and its 5 stores (4 dh2 + 1 partial), which may stay in flight -- on gfx950
    // stores count in vmcnt, and waiting for them (vmcnt(0)) serialised every tile behind its stores.
    // Then s_barrier: every wave's DMA landed and tile t-1's buffer is no longer read (the asm blocks
    // keep the compiler's LDS accesses on their side; no workgroup fence, which would drain the stores)
    if (t == t0)
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(5)\n\ts_barrier" ::: "memory");
    if (t + 1 < t1) dma(t + 1, buf ^ 1);
    EpiOps cur;                                          // in flight during the MFMAs
    epi_load(t, cur);
    const unsigned char* bb = smem + buf * NF * 1024 + lane * 16;
    f32x16_t y = zero16();
    constexpr int PF = 4;                                // B fragments read ahead of their MFMA
    bf16x8 bq[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) bq[i] = lds_frag(bb, i * 1024);
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      y = mfma32(a[i], bq[i % PF], y);
      if (i + PF < NF) bq[i % PF] = lds_frag(bb, (i + PF) * 1024);
      __builtin_amdgcn_sched_barrier(0);
    }
    // dh2 = bf16(dh2_in + y); LayerNorm-2 backward partials (sum dxhat, sum dxhat xhat) of this wave.
    // All math first, then branch-free buffer stores (rows past L fall outside the buffer's range and are
    // dropped): a store under a branch makes the compiler's vmcnt tracking fall back to waiting for every
    // store at the next join, which serialised the next tile behind this one's stores.
    const int pos = t * 32 + r;
    const bool okb = pos < L;
    float sa = 0.f, sc = 0.f;
    u32x2 ov[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float din[4], sv[4], o[4];
      unpack4(cur.d[g], din);
      unpack4(cur.s[g], sv);
      const float gg[4] = {cur.g[g].x, cur.g[g].y, cur.g[g].z, cur.g[g].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = bfround(fmaf(din[e], dmask, y[4 * g + e]));
        const float xh = (sv[e] - mean) * rstd;
        const float dxh = o[e] * gg[e];
        sa += okb ? dxh : 0.f;
        sc += okb ? dxh * xh : 0.f;
      }
      const uint2 q = packq4(o);
      ov[g] = (u32x2){q.x, q.y};
    }
    sa = wave_reduce_sum(sa);
    sc = wave_reduce_sum(sc);
    if constexpr (CONSTS) {
      wsa += sa;
      wsc += sc;
    }
    __builtin_amdgcn_sched_barrier(0);
    const int vo = okb ? (pos * CH + w * 32 + 4 * h) * 2 : 0x7ffffff0;
#pragma unroll
    for (int g = 0; g < 4; ++g) __builtin_amdgcn_raw_buffer_store_b64(ov[g], dh2r, vo + 16 * g, 0, 0);
    const u32x2 sv2 = {__float_as_uint(sa), __float_as_uint(sc)};
    __builtin_amdgcn_raw_buffer_store_b64(sv2, sumr, lane == 0 ? ((t * 4 + w) * 8) : 0x7ffffff0, 0, 0);
  };
  for (int t = t0; t < t1; ++t) step(t, (t - t0) & 1);
  if constexpr (CONSTS) {
    // every DMA was consumed by its tile; the buffers are free once all waves are past their last tile
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    float* red = reinterpret_cast<float*>(smem);
    if (lane == 0) {
      red[2 * w] = wsa;
      red[2 * w + 1] = wsc;
    }
    __syncthreads();
    if (w == 0) {
      const float inv = 1.0f / (float)(L * CH);
      const float m1 = (red[0] + red[2] + red[4] + red[6]) * inv;
      const float m2 = (red[1] + red[3] + red[5] + red[7]) * inv;
      float mean1, rstd1;
      wave_ln_stats(st1 + (size_t)b * T1 * 2, T1, BM1, L, CH, eps, mean1, rstd1);
      if (lane == 0) {
        float4* c = reinterpret_cast<float4*>(consts + (size_t)b * 8);
        c[0] = make_float4(mean, rstd, m1, m2);
        c[1] = make_float4(mean1, rstd1, 0.f, 0.f);
      }
    } else if (w == 1) {
      *reinterpret_cast<float2*>(zero128 + (size_t)b * CH + 2 * lane) = make_float2(0.f, 0.f);
    }
  }
}
// Wv [NJ][128] bf16 -> Wv^T A-operand fragments [ct = c / 32][i = NJ / 16][lane][8]:
// element jj of lane (r, h) = Wv[16 i + 8 (jj >> 2) + 4 h + (jj & 3)][32 ct + r]
__global__ void __launch_bounds__(256) pack_wvt_frag_kernel(const bf16_t* __restrict__ wv, bf16_t* __restrict__ out,
                                                            int NJ) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= NJ * CH) return;
  const int jj = idx & 7, lane = (idx >> 3) & 63, fi = idx >> 9;
  const int NF = NJ / 16;
  const int i = fi % NF, ct = fi / NF;
  const int r = lane & 31, h = lane >> 5;
  const int j = 16 * i + 8 * (jj >> 2) + 4 * h + (jj & 3);
  out[idx] = wv[(size_t)j * CH + 32 * ct + r];
}
}  // namespace

PBX_EXPORT int pbx_pack_wvt_frag(const void* wv, void* out, int NJ, hipStream_t st) {
  if (NJ % 16 != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_wvt_frag_kernel, dim3((NJ * CH + 255) / 256), dim3(256), 0, st, (const bf16_t*)wv,
                     (bf16_t*)out, NJ);
  return pbx_launch_status();
}

static bool pool4_attrs_set = false;

static int attn_bwd4_launch(const void* gfrag, const void* s2, const float* st2, const float* g2, const void* dh2_in,
                            const float* dv, const void* wvt, void* dh2, float* sums2, int B, int L, int NJ, float eps,
                            int tpw, const float* st1, int T1, int BM1, float* consts, float* zero128, hipStream_t st) {
  if ((NJ != 256 && NJ != 512) || B < 1 || L < 1) return (int)hipErrorInvalidValue;
  const bool fuse = consts != nullptr;
  const auto kern = NJ == 512 ? (fuse ? attn_bwd4_kernel<16, true> : attn_bwd4_kernel<16, false>)
                              : (fuse ? attn_bwd4_kernel<8, true> : attn_bwd4_kernel<8, false>);
  if (!pool4_attrs_set) {
    (void)hipFuncSetAttribute((const void*)attn_bwd4_kernel<16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    (void)hipFuncSetAttribute((const void*)attn_bwd4_kernel<8, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    (void)hipFuncSetAttribute((const void*)attn_bwd4_kernel<16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    (void)hipFuncSetAttribute((const void*)attn_bwd4_kernel<8, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    pool4_attrs_set = true;
  }
  const int TW = (L + 31) / 32;
  if (fuse) {
    tpw = TW;                                 // one workgroup per sample
  } else if (tpw <= 0) {
    // >= ~4 workgroups per CU-pair slot over the grid, whole samples when B alone fills the chip
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const long want = 4L * ncu;
    const int nsplit = (int)((want + B - 1) / B);
    tpw = (TW + nsplit - 1) / nsplit;
    if (tpw < 2) tpw = 2;
  }
  if (tpw > TW) tpw = TW;
  const int nsplit = (TW + tpw - 1) / tpw;
  const int lds = 2 * (NJ / 16) * 1024;
  hipLaunchKernelGGL(kern, dim3(nsplit, B), dim3(256), lds, st, (const bf16x8*)gfrag, (const bf16_t*)s2, st2, g2,
                     (const bf16_t*)dh2_in, dv, (const bf16x8*)wvt, (bf16_t*)dh2, sums2, L, tpw, eps, st1, T1, BM1,
                     consts, zero128);
  return pbx_launch_status();
}

// B samples; gfrag as written by pbx_ln_attn_fwd2; dv [B][NJ] fp32 (one gradient row per sample);
// wvt: pbx_pack_wvt_frag image of Wv; sums2 [B][4 ceil(L/32)][2]; tpw <= 0: tiles per workgroup chosen here.
PBX_EXPORT int pbx_attn_bwd4(const void* gfrag, const void* s2, const float* st2, const float* g2,
                             const void* dh2_in, const float* dv, const void* wvt, void* dh2, float* sums2,
                             int B, int L, int NJ, float eps, int tpw, hipStream_t st) {
  return attn_bwd4_launch(gfrag, s2, st2, g2, dh2_in, dv, wvt, dh2, sums2, B, L, NJ, eps, tpw, nullptr, 0, 0, nullptr,
                          nullptr, st);
}

// pbx_attn_bwd4 with one workgroup per sample that also writes consts [B][8] (the ln2_consts_kernel output:
// pbx_ln2_linear_bwd then runs with consts_ready = 1) and zeroes zero128 [B][128]; st1 [B][T1][2]: the
// LayerNorm-1 (mean, M2) tile partials (tile BM1).
PBX_EXPORT int pbx_attn_bwd4c(const void* gfrag, const void* s2, const float* st2, const float* g2,
                              const void* dh2_in, const float* dv, const void* wvt, void* dh2, float* sums2,
                              int B, int L, int NJ, float eps, const float* st1, int T1, int BM1, float* consts,
                              float* zero128, hipStream_t st) {
  if (consts == nullptr || zero128 == nullptr || st1 == nullptr) return (int)hipErrorInvalidValue;
  return attn_bwd4_launch(gfrag, s2, st2, g2, dh2_in, dv, wvt, dh2, sums2, B, L, NJ, eps, 0, st1, T1, BM1, consts,
                          zero128, st);
}
