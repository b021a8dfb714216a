// Attention pool, recompute form (SURVEY K7 + the LayerNorm-2 apply of K5/K6, reference semantics).
//
// Reference: ProteinBERT/modules.py:49-60,87-92,219 (global attention) and :162-164,214-217 (the second
// (L, C) LayerNorm).  In reference semantics every head reduces to (1/K) sum_l GELU(h2 Wv_j) (SURVEY
// A.2 Q1) and the head weights are untrained buffers, so the pool is
//   forward : h2 = LN_(L,C)(s2) (the block output) ; vpart[b][t][j] = sum_{pos in tile t} GELU(h2[pos] . Wv[j])
//   backward: dh2[pos][c] = dh2_in[pos][c] + sum_j Wv[j][c] dv[b][j] GELU'(h2[pos] . Wv[j])
// plus the LayerNorm-2 backward partials (sum dxhat, sum dxhat xhat) per (sample, tile).
//
// Design (MI355X-first, replaces the stored-GELU' pair of rounds 2-4, whose forward wrote and whose
// backward streamed a [B, L, 512] bf16 GELU' tensor -- 537 MB each way per block at B = 1024):
//   * one workgroup per CU (8 waves, two per SIMD), the whole bf16 Wv (512 x 128, 128 KB) staged once
//     into a swizzled LDS image; a workgroup owns ONE 32-position tile and walks a group of samples, so
//     the tile's [L, C] LayerNorm affine rows are staged into the remaining LDS once as well;
//   * forward: s2 rows -> LN2 apply (fp32 affine from LDS) -> h2 (stored: block output) -> MFMA against
//     Wv -> GELU (logistic form fitted to the erf GELU; the A&S erf form in the exact-GELU build) -> column sums, all in
//     registers (no ln2_apply pass, no GELU' store);
//   * backward: h2 rows -> zT = Wv h2^T (MFMA) -> u = dv * GELU'(zT) on the VALU -> dh2^T += Wv^T u (MFMA).
//     The D layout of zT (lane = position, rows 8 g + 4 h + e of a 32-row block) IS the B operand of the
//     second product when its K order is permuted to {16 s + 8 (jj >> 2) + 4 h + (jj & 3)}, which the
//     transposed Wv reads deliver: the two GEMMs meet in registers, nothing goes through LDS or HBM.
//     The GELU' of block jt runs in the shadow of block jt+1's MFMAs (and of the partner wave's).
//   * LayerNorm-2 backward partials: sum dh2 g2 and sum dh2 (h2 - b2) (= g2 xhat up to the bf16 rounding
//     of h2), so the backward needs neither s2 nor the statistics; h2 comes from the B fragments already
//     in registers (a lane-half exchange puts them in the accumulator layout).
// HBM per block (B = 1024, L = 512): forward 268 MB (s2 in, h2 out), backward 403 MB (h2, dh2_in in,
// dh2 out) -- vs ~1.5 GB for the stored-GELU' pair.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int BML = 32;      // tile of the s2 (mean, M2) partials written by ln_linear_fwd (ln.hip)
constexpr int TP = 32;       // positions per tile (one MFMA tile)
constexpr int NWV = 8;       // waves per workgroup
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// stage a [rows x 128] bf16 matrix into a swz256 LDS image (whole workgroup)
__device__ __forceinline__ void stage_rows(unsigned char* dst, const bf16_t* __restrict__ w, int rows) {
  stage_chunks(
      rows * 16, [&](int idx) { return *reinterpret_cast<const uint4*>(w + (size_t)idx * 8); },
      [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(dst + swz256(idx >> 4, idx & 15)) = v; });
}

// fp32 [32 pos][128 ch] affine image, 16-B chunks XOR-swizzled by (pos & 15): a ds_read_b128 lane group
// (16 positions, one chunk) hits 16 distinct bank quads
__device__ __forceinline__ int aff_off(int pos, int chunk) {   // float offset; chunk = ch / 4 (0..31)
  return pos * CH + ((chunk ^ (pos & 15)) << 2);
}
// bf16 [32 pos][128 ch] affine image, 16-B units (8 channels) XOR-swizzled by (pos & 15): a ds_read_b128
// lane group (16 positions, one unit) hits 16 distinct bank quads
__device__ __forceinline__ int affy_off(int pos, int unit4) {   // bf16 offset of 4-channel unit (0..31)
  return pos * CH + ((((unit4 >> 1) ^ (pos & 15)) << 3) | ((unit4 & 1) << 2));
}

__device__ __forceinline__ float4 lds_f4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Pin 8 values at this point of the instruction stream (an empty volatile asm that "modifies" them): the
// SelectionDAG scheduler otherwise sinks pure VALU next to its first use, across sched_barriers.
__device__ __forceinline__ void pin8(float* a) {
  asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]));
}

// Backward operand type.  Fitted-GELU build: both backward GEMMs run on v_mfma_f32_32x32x16_f16 with an f16
// Wv image, so GELU' is evaluated on packed-f16 VALU (v_pk_* f16: two values per ~4-cycle issue slot instead of
// one per fp32 instruction) and u = dv GELU' is the f16 B operand as it stands.  dv is scaled per sample by a
// power of two (max |dv| -> [0.5, 1)) so u stays in the f16 normal range; the epilogue undoes it exactly.
// Entries of u more than 2^14 below the sample's max |dv| lose precision as f16 subnormals and 2^24 below it
// flush to zero: an absolute error <= 2^-24 max |dv| per term, far below the bf16 rounding of dh2
// (tests/test_hip_pool.py, dv spanning 1e-6 .. 1).  Exact-GELU build (PBX_GELU_EXACT): bf16 operands and the
// A&S erf GELU' in fp32.
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
#if !PBX_GELU_EXACT
typedef __attribute__((ext_vector_type(8))) _Float16 opx8;
__device__ __forceinline__ f32x16_t mfma_b(const opx8& a, const opx8& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
#else
typedef bf16x8 opx8;
__device__ __forceinline__ f32x16_t mfma_b(const opx8& a, const opx8& b, const f32x16_t& c) { return mfma32(a, b, c); }
#endif
__device__ __forceinline__ opx8 as_op(const bf16x8& v) { return __builtin_bit_cast(opx8, v); }
__device__ __forceinline__ opx8 as_op(const uint4& v) { return __builtin_bit_cast(opx8, v); }
// 8 bf16 -> 8 f16 (RNE; exact for |x| in [6.1e-5, 65504], the range of the pool's operands)
__device__ __forceinline__ uint4 bf16x8_to_f16x8(const uint4& q) {
  float v[8];
  unpack8(q, v);
  uint4 o;
  unsigned* ow = reinterpret_cast<unsigned*>(&o);
#pragma unroll
  for (int i = 0; i < 4; ++i) ow[i] = __builtin_bit_cast(unsigned, (h2_t){(_Float16)v[2 * i], (_Float16)v[2 * i + 1]});
  return o;
}
__device__ __forceinline__ h2_t h2_of(unsigned u) { return __builtin_bit_cast(h2_t, u); }
__device__ __forceinline__ unsigned u_of(h2_t v) { return __builtin_bit_cast(unsigned, v); }
// exp2 / rcp of 4 f16 pairs: the low halves, then the high halves by SDWA into WORD_1 with the low half
// preserved -- no v_pack per pair, and every transcendental's result is read >= 3 instructions later (the
// trailing s_nop covers the last ones for the instruction after the block: trans-forwarding hazard)
#define PBX_TRANS_H4(OP, x)                                                                                 \
  do {                                                                                                      \
    unsigned i0_ = u_of(x[0]), i1_ = u_of(x[1]), i2_ = u_of(x[2]), i3_ = u_of(x[3]), o0_, o1_, o2_, o3_;  \
    asm volatile(OP "_e32 %0, %4\n\t" OP "_e32 %1, %5\n\t" OP "_e32 %2, %6\n\t" OP "_e32 %3, %7\n\t"           \
                 OP "_sdwa %0, %4 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"            \
                 OP "_sdwa %1, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"            \
                 OP "_sdwa %2, %6 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"            \
                 OP "_sdwa %3, %7 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"            \
                 "s_nop 0"                                                                                  \
                 : "=&v"(o0_), "=&v"(o1_), "=&v"(o2_), "=&v"(o3_)                                            \
                 : "v"(i0_), "v"(i1_), "v"(i2_), "v"(i3_));                                                 \
    x[0] = h2_of(o0_); x[1] = h2_of(o1_); x[2] = h2_of(o2_); x[3] = h2_of(o3_);                             \
  } while (0)

__device__ __forceinline__ void pinh4(h2_t* a) {
  asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
}

// GELU cores (measured on one box, B = 1024, L = 512, round 5, profiles/r5/pool_gelu_cores_ab.txt):
//   forward : A&S-erf 203-206 us (exact build) | 2-term logistic (max |err| 2.9e-4, vpart rel 1.2e-4) 159 us |
//             no GELU at all (ablation, removed) 114 us
//   backward: A&S-erf GELU' 294-296 us (exact build) | f16 logistic GELU' 245 us alone

// sample range of workgroup row blockIdx.y
__device__ __forceinline__ void sample_range(int B, int& b0, int& b1) {
  const int nbg = gridDim.y;
  b0 = (int)((long)B * blockIdx.y / nbg);
  b1 = (int)((long)B * (blockIdx.y + 1) / nbg);
}

// (mean, rstd) of one sample from its (mean, M2) tile partials, T2 <= 128 (two per lane, prefetched)
__device__ __forceinline__ void stats_from(float2 pm0, float2 pm1, int lane, int T2, int L, float eps, float& mean,
                                           float& rstd) {
  float n = 0.f, m = 0.f, M2 = 0.f;
  if (lane < T2) chan_merge(n, m, M2, (float)(min(BML, L - lane * BML) * CH), pm0.x, pm0.y);
  if (lane + 64 < T2) chan_merge(n, m, M2, (float)(min(BML, L - (lane + 64) * BML) * CH), pm1.x, pm1.y);
  wave_chan(n, m, M2);
  mean = m;
  rstd = rsqrtf(M2 / n + eps);
}

// =============================================================================================
// forward: grid (ceil(L / 32), sample groups), 512 threads.  Wave w processes samples b0 + w + 8 i of
// the workgroup's position tile; the next sample's s2 rows and LN statistics partials are loaded while
// this one runs its MFMA / GELU loop (one exposed HBM round trip per wave, not per item).
// vpart [B][ceil(L/32)][NJ].
template <int NJT>
__global__ void __launch_bounds__(64 * NWV) pool_fwd_kernel(
    const bf16_t* __restrict__ s2, const float* __restrict__ st2, const float* __restrict__ g2,
    const float* __restrict__ be2, const bf16_t* __restrict__ wv, bf16_t* __restrict__ h2,
    float* __restrict__ vpart, int B, int L, float eps) {
  constexpr int NJ = NJT * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;                                            // Wv, NJ x 256 B
  float* aff = reinterpret_cast<float*>(smem + NJ * 256);              // gamma [32][128], beta [32][128]
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int tp = blockIdx.x, p0 = tp * TP;
  const int TW = gridDim.x;
  int b0, b1;
  sample_range(B, b0, b1);
  stage_rows(ws, wv, NJ);
  for (int i = tid; i < 2 * TP * 32; i += 64 * NWV) {
    const int which = i >> 10, pr = (i >> 5) & 31, chunk = i & 31;
    const int p = p0 + pr;
    const float* src = (which ? be2 : g2) + (size_t)min(p, L - 1) * CH + chunk * 4;
    float4 v = *reinterpret_cast<const float4*>(src);
    if (p >= L) v = make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(aff + which * TP * CH + aff_off(pr, chunk)) = v;
  }
  __syncthreads();
  const int pos = p0 + r;
  const bool ok = pos < L;
  const int pc = min(pos, L - 1);
  const int T2 = (L + BML - 1) / BML;
  const bool big_t2 = T2 > 128;                                        // statistics loaded per item
  const int vo = ok ? pos * CH * 2 : 0x7ffffff0;     // rows past L fall outside the buffer: stores dropped
  int b = b0 + w;
  if (b >= b1) return;
  // item loads (clamped, branch-free: a load under a branch costs the compiler's vmcnt tracking)
  uint4 q[8];
  float2 pm0, pm1;
  auto load_item = [&](int bb) {
    const bf16_t* src = s2 + ((size_t)bb * L + pc) * CH + 8 * h;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) q[kk] = *reinterpret_cast<const uint4*>(src + kk * 16);
    const float* stb = st2 + (size_t)bb * T2 * 2;
    pm0 = *reinterpret_cast<const float2*>(stb + 2 * min(lane, T2 - 1));
    pm1 = *reinterpret_cast<const float2*>(stb + 2 * min(lane + 64, T2 - 1));
  };
  load_item(b);
  for (; b < b1; b += NWV) {
    float mean, rstd;
    if (big_t2) wave_ln_stats(st2 + (size_t)b * T2 * 2, T2, BML, L, CH, eps, mean, rstd);
    else stats_from(pm0, pm1, lane, T2, L, eps, mean, rstd);
    const float nmr = -mean * rstd;
    // the affine rows are loop-invariant: an opaque offset keeps the compiler from hoisting their 32 LDS
    // reads out of the sample loop (128 VGPRs held across it -> spills)
    int zo = 0;
    asm volatile("" : "+v"(zo));
    const float* gam = aff + zo;
    const float* bet = aff + TP * CH + zo;
    const __amdgpu_buffer_rsrc_t hr =
        __builtin_amdgcn_make_buffer_rsrc(h2 + (size_t)b * L * CH, (short)0, L * CH * 2, 0x00020000);
    bf16x8 hf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      float sv[8], v[8];
      unpack8(q[kk], sv);
      const int c0 = 4 * kk + 2 * h;   // 16-B chunk of channels kk*16 + 8h
      const float4 ga = lds_f4(gam + aff_off(r, c0)), gb4 = lds_f4(gam + aff_off(r, c0 + 1));
      const float4 ba = lds_f4(bet + aff_off(r, c0)), bb4 = lds_f4(bet + aff_off(r, c0 + 1));
      const float g8[8] = {ga.x, ga.y, ga.z, ga.w, gb4.x, gb4.y, gb4.z, gb4.w};
      const float be8[8] = {ba.x, ba.y, ba.z, ba.w, bb4.x, bb4.y, bb4.z, bb4.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaf(fmaf(sv[e], rstd, nmr), g8[e], be8[e]);   // 0 past L (affine 0)
      const uint4 o = packq8(v);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){o.x, o.y, o.z, o.w}, hr, vo + 16 * h, kk * 32, 0);
      hf[kk] = __builtin_bit_cast(bf16x8, o);
    }
    load_item(min(b + NWV, b1 - 1));                 // next item, in flight during the GEMM loop
    float* vrow = vpart + ((size_t)b * TW + tp) * NJ;
    // D[pos][j]: lane = column j = 32 jt + r, 16 positions in registers -> column sums in-lane
    auto epi = [&](const f32x16_t& c, int jt) {
      f32x2 xv[8], gv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = (f32x2){c[2 * i], c[2 * i + 1]};
      gelu_scalar_n<8, 0>(xv, gv, nullptr);
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s += gv[i].x + gv[i].y;
      s += __shfl_xor(s, 32, 64);
      if (h == 0) vrow[jt * 32 + r] = s;
    };
    // software-pipelined column blocks: the MFMA chain of block jt is interleaved, one MFMA at a time, with
    // the GELU / column-sum stages of block jt-1 (sched_barrier-pinned groups), so each wave's stream is a
    // VALU stream with an MFMA every ~30 VALU instructions: neither wave leaves its VALU idle behind 8
    // back-to-back MFMAs, and the two waves of a SIMD share the matrix pipe without queueing on it.
    // Loop body = two blocks (no accumulator copies), branch-free.
    bf16x8 wf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) wf[kk] = lds_frag(ws, swz256(r, kk * 2 + h));
    // one step: c_new = MFMA chain of the block whose fragments are in wf (then wf <- block jn's), while
    // the GELU of c_old (block jo) is summed into vrow
    auto step = [&](f32x16_t& cn, const f32x16_t& co, int jo, int jn) {
      const unsigned char* nb = ws + jn * 32 * 256;
      float x[16], t[16], e[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = co[i];
      cn = zero16();
#define POOL_MF(kk)                                                     \
      cn = mfma32(hf[kk], wf[kk], cn);                                  \
      asm volatile("" : "+v"(cn));                                      \
      wf[kk] = lds_frag(nb, swz256(r, (kk) * 2 + h));                   \
      __builtin_amdgcn_sched_barrier(0);
#if !PBX_GELU_EXACT
      // logistic form: GELU(x) ~ x sigma(x k(t)), t = x^2, k = 1.59934 + 0.0696829 t, fitted (minimax on
      // [-14, 14]) to the exact erf GELU: max |err| 2.9e-4, 7 VALU per value; x / (1 + exp2(-log2(e) x k(t)))
      POOL_MF(0)
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = x[i] * x[i];
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(1)
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = fmaf(t[i], -0.10053117f, -2.3073633f) * x[i];
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(2)
#pragma unroll
      for (int i = 0; i < 16; ++i) e[i] = __builtin_amdgcn_exp2f(t[i]);
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(3)
#pragma unroll
      for (int i = 0; i < 16; ++i) e[i] = __builtin_amdgcn_rcpf(e[i] + 1.0f);
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(4)
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) sm = fmaf(x[i], e[i], sm);
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(5)
#pragma unroll
      for (int i = 8; i < 16; ++i) sm = fmaf(x[i], e[i], sm);
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(6)
#else
      POOL_MF(0)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        t[i] = fmaf(fabsf(x[i]), 0.23164190f, 1.0f);
        e[i] = (x[i] * -0.72134752044448170f) * x[i];
      }
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(1)
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = __builtin_amdgcn_rcpf(t[i]);
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(2)
#pragma unroll
      for (int i = 0; i < 16; ++i) e[i] = __builtin_amdgcn_exp2f(e[i]);
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(3)
      float pl[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) pl[i] = fmaf(t[i], fmaf(t[i], -0.5307027145f, 0.7265760135f), -0.7107068705f);
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(4)
#pragma unroll
      for (int i = 0; i < 16; ++i) pl[i] = fmaf(t[i], fmaf(t[i], pl[i], 0.142248368f), -0.127414796f);
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(5)
#pragma unroll
      for (int i = 0; i < 16; ++i) pl[i] = fmaf(pl[i] * t[i], e[i], 0.5f);   // h = 0.5 erf(|x| / sqrt 2)
      __builtin_amdgcn_sched_barrier(0);
      POOL_MF(6)
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) sm += fmaf(fabsf(x[i]), pl[i], x[i] * 0.5f);   // GELU
      __builtin_amdgcn_sched_barrier(0);
#endif
      POOL_MF(7)
#undef POOL_MF
      sm += __shfl_xor(sm, 32, 64);
      if (h == 0) vrow[jo * 32 + r] = sm;
    };
    auto chain = [&](int jn) {   // first block: no GELU to overlap
      f32x16_t c = zero16();
      const unsigned char* nb = ws + jn * 32 * 256;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        c = mfma32(hf[kk], wf[kk], c);
        wf[kk] = lds_frag(nb, swz256(r, kk * 2 + h));
      }
      return c;
    };
    f32x16_t c0 = chain(1), c1;
#pragma unroll 1
    for (int jt = 1; jt < NJT - 1; jt += 2) {
      step(c1, c0, jt - 1, jt + 1);
      step(c0, c1, jt, jt + 2 < NJT ? jt + 2 : NJT - 1);
    }
    step(c1, c0, NJT - 2, NJT - 1);   // block NJT-1 (its fragments already in wf; the reload is unused)
    epi(c1, NJT - 1);
  }
}

// =============================================================================================
// backward: grid (ceil(L / 32), sample groups), 512 threads.  sums2 [B][ceil(L/32)][2].
// LDS: Wv image, the tile's bf16 affine rows (16 KB) and one dv row per wave (NJ fp32).  The next item's
// h2 rows and dv row are loaded before this item's epilogue, its dh2_in rows two column blocks before the
// loop ends.
template <int NJT>
__global__ void __launch_bounds__(64 * NWV) pool_bwd_kernel(
    const bf16_t* __restrict__ h2, const float* __restrict__ g2, const float* __restrict__ be2,
    const bf16_t* __restrict__ dh2_in, const float* __restrict__ dv, int dv_tiles, const bf16_t* __restrict__ wv,
    bf16_t* __restrict__ dh2, float* __restrict__ sums2, int B, int L) {
  constexpr int NJ = NJT * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;                                            // Wv, NJ x 256 B
  bf16_t* affh = reinterpret_cast<bf16_t*>(smem + NJ * 256);           // bf16 gamma [32][128], beta [32][128]
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  float* dvs = reinterpret_cast<float*>(smem + NJ * 256 + 2 * TP * CH * 2) + w * NJ;   // this wave's dv row
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int tp = blockIdx.x, p0 = tp * TP;
  const int TW = gridDim.x;
  int b0, b1;
  sample_range(B, b0, b1);
#if !PBX_GELU_EXACT
  stage_chunks(
      NJ * 16, [&](int idx) { return bf16x8_to_f16x8(*reinterpret_cast<const uint4*>(wv + (size_t)idx * 8)); },
      [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(ws + swz256(idx >> 4, idx & 15)) = v; });
#else
  stage_rows(ws, wv, NJ);
#endif
  for (int i = tid; i < 2 * TP * 32; i += 64 * NWV) {
    const int which = i >> 10, pr = (i >> 5) & 31, unit = i & 31;
    const int p = p0 + pr;
    const float* src = (which ? be2 : g2) + (size_t)min(p, L - 1) * CH + unit * 4;
    const float4 v = *reinterpret_cast<const float4*>(src);
    const float vv[4] = {v.x, v.y, v.z, v.w};
    *reinterpret_cast<uint2*>(affh + which * TP * CH + affy_off(pr, unit)) = packq4(vv);
  }
  // Wv^T fragment offsets (transposed reads) at 16-step 0; step i adds 16 i rows = 4096 i bytes
  int woff[4], woff8[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    woff[ct] = swz256e(4 * h + q, ct * 32 + tc);
    woff8[ct] = swz256e(4 * h + q + 8, ct * 32 + tc);
  }
  __syncthreads();
  const int pos = p0 + r;
  const bool ok = pos < L;
  const int pc = min(pos, L - 1);
  const bf16_t* dsrc = dh2_in != nullptr ? dh2_in : h2;    // branch-free loads, masked by dmask
  const float dmask = dh2_in != nullptr ? 1.f : 0.f;
  const int vo = ok ? pos * CH * 2 : 0x7ffffff0;          // rows past L: stores dropped
  const int dv_tile = dv_tiles > 1 ? tp : 0;
  int b = b0 + w;
  if (b >= b1) return;
  uint4 hq[8];
  float4 dvr[NJ / 256];
  auto load_item = [&](int bb) {
    const bf16_t* src = h2 + ((size_t)bb * L + pc) * CH + 8 * h;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) hq[kk] = *reinterpret_cast<const uint4*>(src + kk * 16);
#pragma unroll
    for (int k = 0; k < NJ / 256; ++k)
      dvr[k] = *reinterpret_cast<const float4*>(dv + ((size_t)bb * dv_tiles + dv_tile) * NJ + 256 * k + 4 * lane);
  };
  load_item(b);
  for (; b < b1; b += NWV) {
    opx8 hf[8];
    const uint4 zq = make_uint4(0u, 0u, 0u, 0u);
#if !PBX_GELU_EXACT
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      u32x4 c = __builtin_bit_cast(u32x4, bf16x8_to_f16x8(ok ? hq[kk] : zq));
      asm volatile("" : "+v"(c));     // materialised here: sunk into the loop it would keep hq live (spills)
      hf[kk] = __builtin_bit_cast(opx8, c);
    }
    // this sample's dv row as f16 pairs, scaled by 2^-ex so that max |dv| lands in [0.5, 1)
    float dvmax = 0.f;
#pragma unroll
    for (int k = 0; k < NJ / 256; ++k)
      dvmax = fmaxf(dvmax, fmaxf(fmaxf(fabsf(dvr[k].x), fabsf(dvr[k].y)), fmaxf(fabsf(dvr[k].z), fabsf(dvr[k].w))));
    dvmax = wave_reduce_max(dvmax);
    const int dvex = dvmax > 0.f ? __builtin_amdgcn_frexp_expf(dvmax) : 0;
    const float dvscale = ldexpf(1.0f, -dvex), dvinv = ldexpf(1.0f, dvex);
#pragma unroll
    for (int k = 0; k < NJ / 256; ++k) {
      const float4 d = dvr[k];
      *reinterpret_cast<uint2*>(reinterpret_cast<unsigned*>(dvs) + 128 * k + 2 * lane) =
          make_uint2(u_of(__builtin_bit_cast(h2_t, __builtin_amdgcn_cvt_pkrtz(d.x * dvscale, d.y * dvscale))),
                     u_of(__builtin_bit_cast(h2_t, __builtin_amdgcn_cvt_pkrtz(d.z * dvscale, d.w * dvscale))));
    }
#else
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) hf[kk] = as_op(ok ? hq[kk] : zq);
#pragma unroll
    for (int k = 0; k < NJ / 256; ++k) *reinterpret_cast<float4*>(dvs + 256 * k + 4 * lane) = dvr[k];
    constexpr float dvinv = 1.0f;
#endif
    const size_t roff = ((size_t)b * L + pc) * CH;
    f32x16_t y[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) y[ct] = zero16();
    // One step = block jt's GELU' (VALU) + its two 4-MFMA slices of dh2^T += Wv^T u, interleaved (pinned
    // sched_barrier groups) with the 8-MFMA chain of block jn's zT = Wv h2^T: the wave's stream is VALU
    // with an MFMA every ~15 VALU instructions.  Block jt's zT (zo) is complete when the step starts.
    auto bstep = [&](f32x16_t& zn, const f32x16_t& zo, int jt, int jn, bool next) {
      const unsigned char* ab = ws + jn * 32 * 256;
      const unsigned char* w0 = ws + 4096 * (2 * jt);
      const unsigned char* w1 = w0 + 4096;
#if !PBX_GELU_EXACT
      // dv of this lane's rows j = 32 jt + 8 i + 4 h + (0..3), i = 0..3: f16 pairs (j, j + 1)
      const unsigned* dvjh = reinterpret_cast<const unsigned*>(dvs) + jt * 16 + 2 * h;
      const uint2 ddh[4] = {*reinterpret_cast<const uint2*>(dvjh), *reinterpret_cast<const uint2*>(dvjh + 4),
                            *reinterpret_cast<const uint2*>(dvjh + 8), *reinterpret_cast<const uint2*>(dvjh + 12)};
#else
      const float* dvj = dvs + jt * 32 + 4 * h;
      const float4 dd[4] = {*reinterpret_cast<const float4*>(dvj), *reinterpret_cast<const float4*>(dvj + 8),
                            *reinterpret_cast<const float4*>(dvj + 16), *reinterpret_cast<const float4*>(dvj + 24)};
#endif
      opx8 fa[8], fb[4], fc[4];
      auto tr = [&](const unsigned char* wsi, int ct) {
        return as_op(cat_tr(lds_tr(wsi, woff[ct]), lds_tr(wsi, woff8[ct])));
      };
      if (next) {
        fa[0] = as_op(lds_frag(ab, swz256(r, h)));
        fa[1] = as_op(lds_frag(ab, swz256(r, 2 + h)));
      }
      zn = zero16();
      opx8 bu0, bu1;
#if PBX_GELU_EXACT
      float t[8], e[8], pl[8];
#endif
      // GELU' stages of the 8 values of 16-step s (regs 8 s .. 8 s + 7 of zo), Zelen-Severo form of
      // A&S 7.1.26: e = phi(x), Phi = 0.5 + sign(x) h, GELU' = Phi + x phi
#if !PBX_GELU_EXACT
      // logistic GELU' (common.h gelu_logistic_n constants) on packed f16, 4 pairs (j, j + 1) per 16-step s:
      //   s = 1 / (1 + exp2(x (C0 + C1 t))), t = x^2, GELU' = s + x s (1 - s) (K0 + K1 t)
      // x is clamped to [-8, 8] first (GELU' is saturated there: s is exactly 0 or 1 in f16), so t <= 64 and
      // x (K0 + K1 t) stays finite: no 0 * inf, whatever the pre-activation
      h2_t xh[4], th[4], eh[4], kh[4];
      // each stage runs one operation over the 4 independent pairs before the next (a dependent packed-f16
      // op right after its producer costs an s_nop)
      auto stA = [&](int s) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          xh[k] = __builtin_bit_cast(h2_t, __builtin_amdgcn_cvt_pkrtz(zo[8 * s + 2 * k], zo[8 * s + 2 * k + 1]));
#pragma unroll
        for (int k = 0; k < 4; ++k)
          xh[k] = __builtin_elementwise_max(__builtin_elementwise_min(xh[k], (h2_t){8.0f16, 8.0f16}),
                                            (h2_t){-8.0f16, -8.0f16});
#pragma unroll
        for (int k = 0; k < 4; ++k) th[k] = xh[k] * xh[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) eh[k] = th[k] * (h2_t){-0.10053117f16, -0.10053117f16} + (h2_t){-2.3073633f16, -2.3073633f16};
#pragma unroll
        for (int k = 0; k < 4; ++k) eh[k] = eh[k] * xh[k];
        pinh4(xh);
        pinh4(th);
        pinh4(eh);
      };
      auto stB = [&]() { PBX_TRANS_H4("v_exp_f16", eh); };
      auto stC = [&]() {
#pragma unroll
        for (int k = 0; k < 4; ++k) eh[k] = eh[k] + (h2_t){1.0f16, 1.0f16};
        PBX_TRANS_H4("v_rcp_f16", eh);
      };
      auto stD = [&]() {   // x (K0 + K1 t)
#pragma unroll
        for (int k = 0; k < 4; ++k) kh[k] = th[k] * (h2_t){0.20904868f16, 0.20904868f16} + (h2_t){1.5993424f16, 1.5993424f16};
#pragma unroll
        for (int k = 0; k < 4; ++k) kh[k] = kh[k] * xh[k];
        pinh4(kh);
      };
      auto stE = [&](int s) {
        h2_t s1[4], u[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) s1[k] = eh[k] - eh[k] * eh[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = kh[k] * s1[k] + eh[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint2 dq2 = ddh[2 * s + (k >> 1)];
          u[k] = u[k] * h2_of((k & 1) ? dq2.y : dq2.x);
        }
        pinh4(u);
        return as_op(make_uint4(u_of(u[0]), u_of(u[1]), u_of(u[2]), u_of(u[3])));
      };
#else
      auto stA = [&](int s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float x = zo[8 * s + i];
          t[i] = fmaf(fabsf(x), 0.23164190f, 1.0f);
          e[i] = fmaf(x * x, -0.72134752044448170f, -1.3257480647361592f);
        }
        pin8(t);
        pin8(e);
      };
      auto stB = [&]() {
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = __builtin_amdgcn_rcpf(t[i]);
        pin8(t);
      };
      auto stC = [&]() {
#pragma unroll
        for (int i = 0; i < 8; ++i) e[i] = __builtin_amdgcn_exp2f(e[i]);
        pin8(e);
      };
      auto stD = [&]() {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float p = fmaf(t[i], -1.3302744295891233f, 1.8212559791077754f);
          p = fmaf(t[i], p, -1.7814779365698128f);
          p = fmaf(t[i], p, 0.3565637812489156f);
          pl[i] = fmaf(t[i], p, -0.31938153025994087f);
        }
        pin8(pl);
      };
      auto stE = [&](int s) {
        float u[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float x = zo[8 * s + i];
          const float hh = fmaf(pl[i] * t[i], e[i], 0.5f);
          const float Phi = copysignf(hh, x) + 0.5f;
          const float4 d = dd[2 * s + (i >> 2)];
          const float dj = (i & 3) == 0 ? d.x : (i & 3) == 1 ? d.y : (i & 3) == 2 ? d.z : d.w;
          u[i] = fmaf(x, e[i], Phi) * dj;
        }
        pin8(u);
        return as_op(pack8(u));
      };
#endif
#define SB __builtin_amdgcn_sched_barrier(0);
// the empty volatile asm pins each MFMA into its group (MFMA nodes carry no chain, so the DAG scheduler
// would otherwise cluster them in front of the first sched_barrier)
#define PIN(v) asm volatile("" : "+v"(v));
#define G1(k) if (next) { zn = mfma_b(fa[k], hf[k], zn); PIN(zn) if ((k) + 2 < 8) fa[(k) + 2] = as_op(lds_frag(ab, swz256(r, 2 * ((k) + 2) + h))); }
      SB
      G1(0) stA(0); SB
      G1(1) stB(); SB
      G1(2) stC(); SB
      G1(3) stD(); SB
      G1(4) bu0 = stE(0); fb[0] = tr(w0, 0); fb[1] = tr(w0, 1); SB
      G1(5) stA(1); SB
      G1(6) stB(); fb[2] = tr(w0, 2); SB
      G1(7) stC(); fb[3] = tr(w0, 3); SB
      y[0] = mfma_b(fb[0], bu0, y[0]); PIN(y[0]) fc[0] = tr(w1, 0); stD(); SB
      y[1] = mfma_b(fb[1], bu0, y[1]); PIN(y[1]) fc[1] = tr(w1, 1); SB
      y[2] = mfma_b(fb[2], bu0, y[2]); PIN(y[2]) fc[2] = tr(w1, 2); bu1 = stE(1); SB
      y[3] = mfma_b(fb[3], bu0, y[3]); PIN(y[3]) fc[3] = tr(w1, 3); SB
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) y[ct] = mfma_b(fc[ct], bu1, y[ct]);
      SB
#undef G1
#undef PIN
#undef SB
    };
    f32x16_t z0 = zero16(), z1;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) z0 = mfma_b(as_op(lds_frag(ws, swz256(r, kk * 2 + h))), hf[kk], z0);
#pragma unroll 1
    for (int jt = 0; jt < NJT - 2; jt += 2) {
      bstep(z1, z0, jt, jt + 1, true);
      bstep(z0, z1, jt + 1, jt + 2, true);
    }
    // epilogue operand dh2_in in the B-fragment channel layout (lane (r, h): channels 16 K + 8 h + 0..7), loads
    // in flight during the last two blocks
    uint2 dq[16];        // (8-B loads: 16-B ones need aligned register quads, which spill here)
#pragma unroll
    for (int q = 0; q < 16; ++q) dq[q] = *reinterpret_cast<const uint2*>(dsrc + roff + 16 * (q >> 1) + 8 * h + 4 * (q & 1));
    bstep(z1, z0, NJT - 2, NJT - 1, true);
    bstep(z0, z1, NJT - 1, NJT - 1, false);
    load_item(min(b + NWV, b1 - 1));                 // next item: in flight during the epilogue
    // dh2^T in the B-fragment layout too: y[ct][4 g + e] is channel ct*32 + 8 g + 4 h + e; a permlane32 swap
    // of the (g, g + 1) registers leaves lane half h with g = 2 m + h of both halves, i.e. channels
    // ct*32 + 16 m + 8 h + {e, 4 + e}.  Then h2 is hf itself, and dh2_in / dh2 / the affine rows move as
    // 16-B rows (8 buffer_store_b128 per lane instead of 16 b64: the store issue was the epilogue's bound)
    int rh = r;                                  // opaque: keeps the affine LDS addresses inside the loop
    asm volatile("" : "+v"(rh));
    const bf16_t* gamh = affh + rh * CH;
    const bf16_t* beth = gamh + TP * CH;
    const __amdgpu_buffer_rsrc_t dr =
        __builtin_amdgcn_make_buffer_rsrc(dh2 + (size_t)b * L * CH, (short)0, L * CH * 2, 0x00020000);
    float sa = 0.f, sc = 0.f;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int ct = kk >> 1, m = kk & 1;
      float o[8], din[8], hh[8], gg[8], bb[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(y[ct][8 * m + e]),
                                                         __float_as_uint(y[ct][8 * m + 4 + e]), false, false);
        o[e] = __uint_as_float(sw[0]);
        o[4 + e] = __uint_as_float(sw[1]);
      }
      const int uo = (((2 * kk + h) ^ (rh & 15)) << 3);         // 16-B unit 2 kk + h of row rh (affy layout)
      unpack4(dq[2 * kk], din);
      unpack4(dq[2 * kk + 1], din + 4);
#if !PBX_GELU_EXACT
      {
        const uint4 hb = __builtin_bit_cast(uint4, hf[kk]);     // zero past L
        const unsigned hw[4] = {hb.x, hb.y, hb.z, hb.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const h2_t v = h2_of(hw[i]);
          hh[2 * i] = (float)v.x;
          hh[2 * i + 1] = (float)v.y;
        }
      }
#else
      unpack8(__builtin_bit_cast(uint4, hf[kk]), hh);             // zero past L
#endif
      unpack8(*reinterpret_cast<const uint4*>(gamh + uo), gg);
      unpack8(*reinterpret_cast<const uint4*>(beth + uo), bb);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = bfround(fmaf(din[e], dmask, o[e] * dvinv));
        sa = fmaf(o[e], gg[e], sa);
        sc = fmaf(o[e], hh[e] - bb[e], sc);
      }
      const uint4 oq = packq8(o);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){oq.x, oq.y, oq.z, oq.w}, dr, vo + 16 * h, kk * 32, 0);
      __builtin_amdgcn_sched_barrier(0);   // one 16-B row at a time (hoisted affine reads of all 8 spill)
    }
    sa = wave_reduce_sum(ok ? sa : 0.f);
    sc = wave_reduce_sum(ok ? sc : 0.f);
    if (lane == 0) *reinterpret_cast<float2*>(sums2 + ((size_t)b * TW + tp) * 2) = make_float2(sa, sc);
  }
}

bool pool_attrs_set = false;
void set_pool_attrs() {
  if (pool_attrs_set) return;
  (void)hipFuncSetAttribute((const void*)pool_fwd_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)pool_fwd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)pool_bwd_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)pool_bwd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  pool_attrs_set = true;
}

int num_cus_pool() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
  }
  return n;
}

dim3 pool_grid(int B, int L) {
  const int TW = (L + TP - 1) / TP;
  int ng = (num_cus_pool() + TW - 1) / TW;             // one workgroup per CU (LDS-bound)
  ng = ng < 1 ? 1 : (ng > B ? B : ng);
  return dim3(TW, ng);
}
}  // namespace

// s2 [B, L, 128] bf16; st2 [B][ceil(L/32)][2] (mean, M2) tile partials; g2 / be2 [L, 128] fp32;
// wv [NJ, 128] bf16 (NJ = 256 or 512); h2 [B, L, 128] bf16 out; vpart [B][ceil(L/32)][NJ] fp32 out.
PBX_EXPORT int pbx_pool_fwd(const void* s2, const float* st2, const float* g2, const float* be2, const void* wv,
                            void* h2, float* vpart, int B, int L, int NJ, float eps, hipStream_t st) {
  if ((NJ != 256 && NJ != 512) || B < 1 || L < 1) return (int)hipErrorInvalidValue;
  set_pool_attrs();
  const int lds = NJ * 256 + 2 * TP * CH * 4;
  const auto kern = NJ == 512 ? pool_fwd_kernel<16> : pool_fwd_kernel<8>;
  hipLaunchKernelGGL(kern, pool_grid(B, L), dim3(64 * NWV), lds, st, (const bf16_t*)s2, st2, g2, be2,
                     (const bf16_t*)wv, (bf16_t*)h2, vpart, B, L, eps);
  return pbx_launch_status();
}

// h2 [B, L, 128] bf16 (the forward's output); dh2_in (nullable) [B, L, 128] bf16; dv [B][dv_tiles][NJ] fp32:
// the vpart gradient, one row per sample (dv_tiles = 1: every tile's row has the same gradient, as when
// the consumer sums the tiles) or per tile (dv_tiles = ceil(L/32)); dh2 [B, L, 128] bf16 out;
// sums2 [B][ceil(L/32)][2] fp32 out: (sum dh2 g2, sum dh2 (h2 - b2)) per (sample, 32-position tile).
PBX_EXPORT int pbx_pool_bwd(const void* h2, const float* g2, const float* be2, const void* dh2_in, const float* dv,
                            int dv_tiles, const void* wv, void* dh2, float* sums2, int B, int L, int NJ,
                            hipStream_t st) {
  const int TW = (L + TP - 1) / TP;
  if ((NJ != 256 && NJ != 512) || B < 1 || L < 1 || (dv_tiles != 1 && dv_tiles != TW)) return (int)hipErrorInvalidValue;
  set_pool_attrs();
  const int lds = NJ * 256 + 2 * TP * CH * 2 + NWV * NJ * 4;
  const auto kern = NJ == 512 ? pool_bwd_kernel<16> : pool_bwd_kernel<8>;
  hipLaunchKernelGGL(kern, pool_grid(B, L), dim3(64 * NWV), lds, st, (const bf16_t*)h2, g2, be2,
                     (const bf16_t*)dh2_in, dv, dv_tiles, (const bf16_t*)wv, (bf16_t*)dh2, sums2, B, L);
  return pbx_launch_status();
}

