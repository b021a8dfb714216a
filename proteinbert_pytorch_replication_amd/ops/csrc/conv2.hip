// Dual-dilation residue convolutions with weights streamed as MFMA fragments.
//
// Reference: ProteinBERT/modules.py:124-147 (Conv1d C->C, k=9, dilation 1 and 5, padding "same",
// each + GELU) and :205-212 (x + narrow + wide + broadcast(global->local), LayerNorm over (L, C)).
//
// Why weights are streamed (the round-1 form staged all 590 KB of both convs' weights through LDS:
// global -> VGPR -> ds_write -> barrier -> ds_read for only 256 positions, a barrier every weight
// step and one workgroup per CU, MFMA busy ~25 %, profiles/r1_hip_v5_*): here the weights are re-packed once per step (pbx_pack_conv_frag, 2 x 295 KB bf16) into the exact
// per-lane order of a v_mfma_f32_32x32x16_bf16 A operand, so one wave loads a whole 32x16 fragment
// with ONE coalesced 1-KB global_load_dwordx4 (an L2 hit: every XCD keeps the 0.6 MB resident).
// Only the activation tile lives in LDS; the main loop has no barrier and no LDS writes, each wave
// runs independently with its A fragments prefetched two K-steps ahead, and a workgroup needs
// < 80 KB of LDS and <= 128 VGPRs, so two workgroups (16 waves) share a CU.
//
//   conv_fwd3   : 128 positions / workgroup; waves 0-3 = narrow conv, 4-7 = wide conv; wave q owns
//                 output channels q*32..+32 for all 128 positions (4 accumulators of 32x32).
//                 Epilogue: the pre-activations staged through LDS; all 8 waves then write
//                 s1 = x + GELU(pre_n) + GELU(pre_w) + gb and (training) GELU'(pre_n), GELU'(pre_w)
//                 with row-contiguous 16-B stores, plus the tile's LayerNorm (mean, M2) partial.
//   (the data gradient is conv4.hip conv_dgrad4)
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int BM = 128;               // positions per workgroup
constexpr int FRAG = 64 * 8;          // bf16 per packed fragment (64 lanes x 8)
constexpr int OT = BM * 256;          // bytes of one [BM][128] bf16 staging tile

// Workgroup -> (sample, tile) id.  The dispatcher deals workgroups to the 8 XCDs round-robin by id
// (blockIdx % 8 labels the blocks that share an XCD's L2), so the bijective remap
// (cdna_hip_programming.md T1) gives each XCD a contiguous run of tiles: neighbouring tiles of one
// sample, whose +-20-row halos overlap, then read those rows through the same L2.  +0.5 % on the step,
// 6/6 same-box rounds against the identity map (profiles/r2_v8_xcd_remap_ab.txt).
__device__ __forceinline__ int tile_id() {
  const int n = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// Packed fragment index (in fragments) of (tap k, K-block kb of 16, M-block mb of 32); lane offset
// added by the reader.  Forward: M = output channel, K = input channel.  Dgrad: M = input channel,
// K = output channel.
__device__ __forceinline__ int frag_index(int k, int kb, int mb) { return (k * 8 + kb) * 4 + mb; }

// TBM = 128 positions per workgroup: two workgroups per CU at <= 128 VGPRs (a 256-position form, one
// workgroup per CU with every weight fragment feeding 8 MFMAs, measured slower in the full step)
template <bool STORE>   // STORE: write GELU'(pre) of both convs for the backward (training forward)
__global__ void __launch_bounds__(512, 4) conv_fwd3_kernel(
    const bf16_t* __restrict__ x, const bf16x8* __restrict__ fwn, const bf16x8* __restrict__ fww,
    const float* __restrict__ bn, const float* __restrict__ bw, const float* __restrict__ gb,
    bf16_t* __restrict__ pre_n, bf16_t* __restrict__ pre_w, bf16_t* __restrict__ s1,
    float* __restrict__ stats, int L, int KS, int dil, const long long* __restrict__ tok,
    const bf16_t* __restrict__ emb, int xlo, int xhi) {
  constexpr int TBM = BM;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NPT = TBM / 32;                               // 32-position MFMA tiles per wave
  constexpr int TOT = TBM * 256;                              // bytes of one [TBM][128] bf16 tile
  const int T = (L + TBM - 1) / TBM;
  const int tid0 = tile_id();
  const int b = tid0 / T, t = tid0 - (tid0 / T) * T;
  const int pos0 = t * TBM;
  const int half = KS >> 1;
  const int halo = half * dil;
  const int XR = TBM + 2 * halo;
  unsigned char* xs = smem;                                   // XR x 256 B (swz256)
  unsigned char* ot = smem + XR * 256;                        // [TBM][128] bf16 staging tile
  float* bsm = reinterpret_cast<float*>(ot + TOT);            // bn | bw | gb[b] | LN scratch
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int cv = w >> 2, cq = w & 3;
  // xlo / xhi: rows of the neighbouring sequence shards stored around each sample's L rows (context
  // parallelism): logical positions -xlo .. L + xhi - 1 are real, anything beyond is the zero padding
  const bf16_t* xsmp = x + ((size_t)b * (xlo + L + xhi) + xlo) * CH;
  const bf16x8* fw = (cv ? fww : fwn) + cq * 64;            // wave-uniform; + frag_index(k, kb, 0) * 64 + lane
  const int NI = KS * 8;                                      // K-steps: taps x 16-channel blocks
  // A-fragment ring: step it uses fr[it & 3], the load for step it + 3 is in flight meanwhile (the
  // loop is unrolled by the ring size so the ring never rotates registers, which would make the
  // compiler wait for the newest load every step)
  bf16x8 fr[4];
  fr[0] = fw[lane];
  fr[1] = fw[256 + lane];
  fr[2] = fw[512 + lane];
  if (tid < 3 * CH) bsm[tid] = tid < CH ? bn[tid] : tid < 2 * CH ? bw[tid - CH] : gb[(size_t)b * CH + tid - 2 * CH];
  // tok != nullptr (the first block, pbx_conv_fwd3t): the input rows are the embedding rows emb[tok]
  // (bf16 [V][128]), gathered here -- the [B, L, 128] embedding output is never materialised
  const long long* toks = tok != nullptr ? tok + (size_t)b * L : nullptr;
  stage_chunks(
      XR * 16,
      [&](int idx) {
        const int pos = pos0 - halo + (idx >> 4);
        if (pos < -xlo || pos >= L + xhi) return make_uint4(0u, 0u, 0u, 0u);
        const bf16_t* row = toks != nullptr ? emb + (size_t)toks[pos] * CH : xsmp + (size_t)pos * CH;
        return *reinterpret_cast<const uint4*>(row + (idx & 15) * 8);
      },
      [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(xs + swz256(idx >> 4, idx & 15)) = v; });
  __syncthreads();

  f32x16_t acc[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) acc[i] = zero16();
  const int d = cv ? dil : 1;
  // tap loop outside, the 8 channel blocks of a tap unrolled: the swz256 byte offset of (row rb + 32 pt,
  // chunk 2 kb + h) is rowb + 8192 pt + ((32 kb) ^ gs) with rowb / gs fixed per tap, so a step costs one
  // v_xad_u32 instead of the ~7 VALU of the general swizzle; the weight fragment address is a scalar
  // base + the lane offset (no per-step 64-bit vector add)
  // B fragments (the x rows) are read one K-step ahead into a 2-deep register ring, so an MFMA never
  // waits on the LDS read issued right before it (the previous form read them in front of their own
  // MFMAs: an s_waitcnt lgkmcnt per MFMA pair, the LDS latency exposed on every step)
  bf16x8 bq[2][NPT];
  auto rows_of = [&](int k, int& rowb, int& gs) {
    const int rb = halo + r + (k - half) * d;
    rowb = rb << 8;
    gs = (h ^ (((rb & 3) << 2) | ((rb >> 2) & 3))) << 4;
  };
  int rowb, gs;
  rows_of(0, rowb, gs);
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) bq[0][pt] = lds_frag(xs, (0 ^ gs) + rowb + pt * 8192);
  for (int k = 0; k < KS; ++k) {
    int rowbn, gsn;
    rows_of(min(k + 1, KS - 1), rowbn, gsn);
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      const int it = k * 8 + kb;
      const bf16x8* fwk = fw + min(it + 3, NI - 1) * 256;   // scalar base
      fr[(kb + 3) & 3] = fwk[lane];
      const int noff = kb < 7 ? ((32 * (kb + 1)) ^ gs) + rowb : (0 ^ gsn) + rowbn;
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) bq[(kb + 1) & 1][pt] = lds_frag(xs, noff + pt * 8192);
      __builtin_amdgcn_sched_barrier(0);          // keep both prefetches ahead of this step's MFMAs
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) acc[pt] = mfma32(fr[kb & 3], bq[kb & 1][pt], acc[pt]);
    }
    rowb = rowbn;
    gs = gsn;
  }

  // ---- epilogue: acc[pt][4g + e] = (co = cq*32 + 8g + 4h + e, pos = pt*32 + r) ------------------
  // Both pre-activation tiles are staged in LDS (narrow -> ot, wide -> over the x tile, whose 4 rows
  // per thread are read into registers first), then all 512 threads take 4 (row, 16-B chunk) units
  // each: pre_n / pre_w stores, s1 = x + GELU(pre_n) + GELU(pre_w) + gb with interleaved packed GELU
  // chains, and the LayerNorm (mean, M2) partial -- balanced over the 8 waves (the narrow waves
  // alone used to evaluate all 2 x 16K GELUs of the tile while the wide waves idled).
  const int vrows = min(TBM, L - pos0);
  uint4 xq[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int idx = tid + 512 * i;
    xq[i] = *reinterpret_cast<const uint4*>(xs + swz256(halo + (idx >> 4), idx & 15));
  }
  __syncthreads();                                // every wave is done with the x tile
  {
    unsigned char* dst = cv ? smem : ot;
    const float* bias = bsm + cv * CH;
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ch0 = cq * 32 + 8 * g + 4 * h;
        const float4 bv = *reinterpret_cast<const float4*>(bias + ch0);
        const float v[4] = {acc[pt][4 * g] + bv.x, acc[pt][4 * g + 1] + bv.y, acc[pt][4 * g + 2] + bv.z,
                            acc[pt][4 * g + 3] + bv.w};
        *reinterpret_cast<uint2*>(dst + swz256e(pt * 32 + r, ch0)) = packq4(v);
      }
  }
  __syncthreads();
  // s1 = x + GELU(pre_n) + GELU(pre_w) + gb in packed pairs; the LayerNorm partial of the tile as
  // plain (sum, sum of squares) of the stored bf16 values -- per row, masked once -- merged to
  // (mean, M2) by one thread at the end (the per-thread / per-lane Chan merges cost a division each)
  f32x2 s2v = {0.f, 0.f};                          // (sum, sum of squares)
  const float4 g0 = *reinterpret_cast<const float4*>(bsm + 2 * CH + (tid & 15) * 8);
  const float4 g1 = *reinterpret_cast<const float4*>(bsm + 2 * CH + (tid & 15) * 8 + 4);
  const f32x2 gbp[4] = {(f32x2){g0.x, g0.y}, (f32x2){g0.z, g0.w}, (f32x2){g1.x, g1.y}, (f32x2){g1.z, g1.w}};
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int idx = tid + 512 * i;
    const int row = idx >> 4, c = idx & 15;
    const bool ok = row < vrows;
    const uint4 pnq = *reinterpret_cast<const uint4*>(ot + swz256(row, c));
    const uint4 pwq = *reinterpret_cast<const uint4*>(smem + swz256(row, c));
    const size_t off = ((size_t)b * L + pos0 + row) * CH + c * 8;
    float xv[8], pn[8], pw[8];
    unpack8(xq[i], xv);
    unpack8(pnq, pn);
    unpack8(pwq, pw);
    f32x2 gi[8], go[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      gi[e] = (f32x2){pn[2 * e], pn[2 * e + 1]};
      gi[4 + e] = (f32x2){pw[2 * e], pw[2 * e + 1]};
    }
    // scalar GELU stages: this epilogue runs beside the other waves' MFMAs, where packed-fp32 forms measured
    // slower.  Training: GELU AND GELU' from one shared core; GELU' is what the data gradient multiplies by,
    // so it is stored instead of the pre-activation and the data gradient evaluates no GELU' core
    // (gelu_n: the fitted logistic core, or the A&S erf core in the exact-GELU library -- common.h)
    if constexpr (STORE) {
      f32x2 gd[8];
      gelu_n<4, 2>(gi, go, gd);
      gelu_n<4, 2>(gi + 4, go + 4, gd + 4);
      float dn[8], dw[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dn[2 * e] = gd[e].x;
        dn[2 * e + 1] = gd[e].y;
        dw[2 * e] = gd[4 + e].x;
        dw[2 * e + 1] = gd[4 + e].y;
      }
      if (ok) {
        *reinterpret_cast<uint4*>(pre_n + off) = packq8(dn);
        *reinterpret_cast<uint4*>(pre_w + off) = packq8(dw);
      }
    } else {
      gelu_n<4, 0>(gi, go, nullptr);
      gelu_n<4, 0>(gi + 4, go + 4, nullptr);
    }
    float o[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      // no FMA contraction of the GELU product into these adds: conv_fwd5 (conv5.hip) rounds the same way
#pragma clang fp contract(off)
      const f32x2 v = (f32x2){xv[2 * e], xv[2 * e + 1]} + go[e] + go[4 + e] + gbp[e];
      o[2 * e] = v.x;
      o[2 * e + 1] = v.y;
    }
    const uint4 oq = packq8(o);
    if (ok) *reinterpret_cast<uint4*>(s1 + off) = oq;
    float orr[8];
    unpack8(oq, orr);                                // the stored (rounded) values
    f32x2 rs = {0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const f32x2 pv = {orr[e], orr[e + 1]};
      rs += (f32x2){pv.x + pv.y, pv.x * pv.x + pv.y * pv.y};
    }
    s2v += ok ? rs : (f32x2){0.f, 0.f};
  }
  float* scratch = bsm + 3 * CH;                  // 8 waves x (sum, sum of squares)
  {
    const float sa = wave_reduce_sum(s2v.x), sq = wave_reduce_sum(s2v.y);
    if (lane == 0) { scratch[2 * w] = sa; scratch[2 * w + 1] = sq; }
  }
  __syncthreads();
  if (tid == 0) {
    float sa = 0.f, sq = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) { sa += scratch[2 * i]; sq += scratch[2 * i + 1]; }
    const float n = (float)(vrows * CH), m = sa / n;
    stats[((size_t)b * T + t) * 2] = m;
    stats[((size_t)b * T + t) * 2 + 1] = fmaxf(sq - sa * m, 0.f);
  }
}

// fp32 torch conv weight [co][ci][KS] -> bf16 fragment images: fwd[k][kb][mb][lane][8] with
// (M = co = 32mb + (lane&31), K = ci = 16kb + 8(lane>>5) + j) and dgrad with M = ci, K = co.
__global__ void __launch_bounds__(256) pack_conv_frag_kernel(const float* __restrict__ w, bf16_t* __restrict__ pf,
                                                             bf16_t* __restrict__ pt, int KS) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= KS * CH * CH) return;
  const int j = idx & 7, lane = (idx >> 3) & 63, fi = idx >> 9;
  const int mb = fi & 3, kb = (fi >> 2) & 7, k = fi >> 5;
  const int m = mb * 32 + (lane & 31), kk = kb * 16 + 8 * (lane >> 5) + j;
  pf[idx] = f2bf(w[((size_t)m * CH + kk) * KS + k]);     // M = co, K = ci
  pt[idx] = f2bf(w[((size_t)kk * CH + m) * KS + k]);     // M = ci, K = co
}

int fwd3_lds(int KS, int dil, int tbm) {
  const int xt = (tbm + 2 * (KS / 2) * dil) * 256;  // x tile, later the pre_w staging tile
  const int ot = tbm * 256;
  return (xt > ot ? xt : ot) + ot + (3 * CH + 32) * 4;
}
}  // namespace

static bool conv3_attrs_set = false;
static void set_conv3_attrs() {
  if (conv3_attrs_set) return;
  (void)hipFuncSetAttribute((const void*)conv_fwd3_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)conv_fwd3_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  conv3_attrs_set = true;
}

// LayerNorm partials in `stats` are per 128-position tile: [B][ceil(L/128)][2].  fwn/fww: forward
// fragment images of the narrow/wide weights (pbx_pack_conv_frag); C = 128 channels; gb [B][128] fp32.
// pre_n / pre_w: GELU'(pre-activation) of the narrow / wide conv as bf16 (what the data gradient,
// conv4.hip conv_dgrad4, multiplies the incoming gradient by), or both null (inference: no backward).
// xlo / xhi: halo rows of the neighbouring sequence shards stored around each sample's L rows of x
// (context parallelism: x is [B][xlo + L + xhi][128]); 0 / 0 for a whole sequence.
static int conv_fwd3_launch(const void* x, const long long* tok, const void* emb, const void* fwn, const void* fww,
                            const float* bn, const float* bw, const float* gb, void* pre_n, void* pre_w, void* s1,
                            float* stats, int B, int L, int KS, int dil, int xlo, int xhi, hipStream_t st) {
  set_conv3_attrs();
  const int lds = fwd3_lds(KS, dil, BM);
  if (lds > 163840 || dil < 1 || KS < 2 || gb == nullptr || xlo < 0 || xhi < 0) return (int)hipErrorInvalidValue;
  if (tok != nullptr && (xlo || xhi)) return (int)hipErrorInvalidValue;
  const int T = (L + BM - 1) / BM;
  if ((pre_n == nullptr) != (pre_w == nullptr)) return (int)hipErrorInvalidValue;
  const auto kern = pre_n != nullptr ? conv_fwd3_kernel<true> : conv_fwd3_kernel<false>;
  hipLaunchKernelGGL(kern, dim3(B * T), dim3(512), lds, st, (const bf16_t*)x, (const bf16x8*)fwn,
                     (const bf16x8*)fww, bn, bw, gb, (bf16_t*)pre_n, (bf16_t*)pre_w, (bf16_t*)s1, stats, L, KS, dil,
                     tok, (const bf16_t*)emb, xlo, xhi);
  return pbx_launch_status();
}

// context-parallel form: x holds xlo / xhi halo rows of the neighbouring shards around each sample's L rows
PBX_EXPORT int pbx_conv_fwd3x(const void* x, const void* fwn, const void* fww, const float* bn, const float* bw,
                              const float* gb, void* pre_n, void* pre_w, void* s1, float* stats, int B, int L, int KS,
                              int dil, int xlo, int xhi, hipStream_t st) {
  return conv_fwd3_launch(x, nullptr, nullptr, fwn, fww, bn, bw, gb, pre_n, pre_w, s1, stats, B, L, KS, dil, xlo, xhi,
                          st);
}

// The first block (reference modules.py:249-253,300 feeding :185-212): x = emb[tok] gathered in the
// staging pass (tok [B][L] int64 < V, emb [V][128] bf16); otherwise pbx_conv_fwd3x.
PBX_EXPORT int pbx_conv_fwd3t(const long long* tok, const void* emb, const void* fwn, const void* fww, const float* bn,
                              const float* bw, const float* gb, void* pre_n, void* pre_w, void* s1, float* stats,
                              int B, int L, int KS, int dil, hipStream_t st) {
  if (tok == nullptr || emb == nullptr) return (int)hipErrorInvalidValue;
  return conv_fwd3_launch(nullptr, tok, emb, fwn, fww, bn, bw, gb, pre_n, pre_w, s1, stats, B, L, KS, dil, 0, 0, st);
}

// fwd / dgrad fragment images (KS * 128 * 128 bf16 each) of one fp32 [128][128][KS] conv weight
PBX_EXPORT int pbx_pack_conv_frag(const float* w, void* pf, void* pt, int KS, hipStream_t st) {
  const int n = KS * CH * CH;
  hipLaunchKernelGGL(pack_conv_frag_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w, (bf16_t*)pf, (bf16_t*)pt,
                     KS);
  return pbx_launch_status();
}

