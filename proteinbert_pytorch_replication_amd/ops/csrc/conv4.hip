// Dual-dilation residue convolution data gradient, optionally with the LayerNorm-1 backward
// finalize fused into its staging pass (K5).
//
// Reference: ProteinBERT/modules.py:124-147 (Conv1d C->C, k=9, dilation 1 and 5, padding "same",
// each + GELU) and :205-212 (x + narrow + wide + broadcast(global->local), LayerNorm over (L, C)) --
// the backward of that chain.  The forward is conv2.hip conv_fwd3.
//
// (A persistent, software-pipelined forward -- the epilogue of tile i-1 inside the K loop of tile i --
// lived here in rounds 3-4: equal in isolation, 3.3 % slower in the step; removed in round 5.)
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int BM = 128;              // positions per tile
constexpr int KS = 9;                // taps (the launcher refuses other sizes)
constexpr int NI = KS * 8;           // K-steps per tile (taps x 16-channel blocks)
constexpr int NPT = BM / 32;         // 32-position MFMA tiles per wave


// ------------------------------------------------------------------------------------------------
// Data gradient, one wave per 32 input channels over BOTH convolutions (reference modules.py:205-206
// backward):  dx[pos][ci] = ds1[pos][ci] + sum_conv sum_tap sum_co W[co][ci][tap] dpre_conv[pos - shift][co]
//
// (The round-2 form split the two convolutions over two wave groups and summed their fp32 partials through
// a 64 KB LDS tile with two extra barriers before the dx pass.)  Here each of the 4 waves runs the K loop of both convolutions (2 x 72 K-steps, 4 MFMAs each) into
// ONE accumulator set, so the cross-wave reduction disappears; the weight-fragment ring (buffer loads,
// scalar offsets) runs straight from the narrow into the wide image.  dpre = ds1 * GELU'(pre) tiles
// (GELU' stored by the forward) with their halos are staged once per workgroup; their central rows go
// to global for the weight gradient.  ~78 KB of LDS: two workgroups (8 waves) per CU.
//
// FIN (pbx_conv_dgrad4f): the LayerNorm-1 backward finalize is fused into the staging: dS1 is never
// stored -- each staged row computes dS1 = rstd1 (dh1 g1 - m1 - xhat1 m2) (bf16, as ln1_finalize
// rounds it) from dh1 / s1 and the per-sample statistics, the central rows' dS1 stay in registers for
// the dx = dS1 + conv^T epilogue, and their column sums go to dgb (one float atomic per channel and
// workgroup).  Saves the dS1 write + read and the finalize launch.  Whole sequences only (ilo = ihi = 0).
struct FinArgs {
  const bf16_t* dh1;
  const bf16_t* s1;
  const float* st1;       // [B][T1][2] LN1 (mean, M2) partials
  int T1, BM1;
  const float* sums1;     // [B][TS1][2] LN1 backward partials
  int TS1;
  const float* g1;        // [L][128] LN1 affine weight
  float* dgb;             // [B][128] accumulated
  float eps;
};

template <bool FIN>
__global__ void __launch_bounds__(256, 2) conv_dgrad4_kernel(
    const bf16_t* __restrict__ ds1, const bf16_t* __restrict__ gdn, const bf16_t* __restrict__ gdw,
    const bf16x8* __restrict__ ftn, const bf16x8* __restrict__ ftw, bf16_t* __restrict__ dx,
    bf16_t* __restrict__ dpre_n, bf16_t* __restrict__ dpre_w, int L, int dil, int ilo, int ihi, FinArgs fa) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = (L + BM - 1) / BM;
  int tid0;
  {
    const int n = gridDim.x, orig = blockIdx.x, xcd = orig & 7, qq = n >> 3, rr = n & 7;
    tid0 = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);   // XCD-contiguous tiles
  }
  const int b = tid0 / T, t = tid0 - (tid0 / T) * T;
  const int pos0 = t * BM;
  const int half = KS >> 1;
  const int halo_n = half, halo_w = half * dil;
  const int RN = BM + 2 * halo_n;
  unsigned char* an = smem;                       // RN x 256 B: dpre of the narrow conv (swz256)
  unsigned char* aw = smem + RN * 256;            // (BM + 2 halo_w) x 256 B: wide conv
  const int tid = threadIdx.x, lane = tid & 63, cq = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const size_t sbase = (size_t)b * L * CH;                          // outputs: [B][L][128]
  const ptrdiff_t ibase = ((ptrdiff_t)b * (L + ilo + ihi) + ilo) * CH;   // inputs: logical position 0
  const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16x8*>(ftn + cq * 64), (short)0, (NI * 4 - cq) * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16x8*>(ftw + cq * 64), (short)0, (NI * 4 - cq) * 1024, 0x00020000);
  auto wfrag = [&](int it) {      // K-step it of 2 NI: narrow image for it < NI, then the wide one
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
    const int li = it < NI ? it : it - NI;
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(it < NI ? rn : rw, lane * 16, li * 4096, 0);
    return __builtin_bit_cast(bf16x8, v);
  };
  bf16x8 fr[4];
  fr[0] = wfrag(0);
  fr[1] = wfrag(1);
  fr[2] = wfrag(2);

  // FIN: dS1 of the central rows (narrow-tile rows (tid >> 4) + 16 m - 4, channel chunk tid & 15) and
  // this thread's share of their column sums
  uint4 keep[9];
  float csum[8];
  float mean1 = 0.f, rstd1 = 0.f, m1 = 0.f, m2 = 0.f;
  if constexpr (FIN) {
    // per-sample LN1 constants, computed by every wave (no barrier)
    wave_ln_stats(fa.st1 + (size_t)b * fa.T1 * 2, fa.T1, fa.BM1, L, CH, fa.eps, mean1, rstd1);
    wave_bwd_consts(fa.sums1 + (size_t)b * fa.TS1 * 2, fa.TS1, 1.0f / (float)(L * CH), m1, m2);
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
  }
  // dS1 chunk operands of position pos (clamped to a valid row; masked by the caller)
  auto fin_load = [&](int pos, int c16, uint4& qd, uint4& qs, float4& ga, float4& gb) {
    const int p = min(max(pos, 0), L - 1);
    const size_t off = sbase + (size_t)p * CH + c16 * 8;
    qd = *reinterpret_cast<const uint4*>(fa.dh1 + off);
    qs = *reinterpret_cast<const uint4*>(fa.s1 + off);
    ga = *reinterpret_cast<const float4*>(fa.g1 + (size_t)p * CH + c16 * 8);
    gb = *reinterpret_cast<const float4*>(fa.g1 + (size_t)p * CH + c16 * 8 + 4);
  };
  auto fin_ds1 = [&](bool ok, const uint4& qd, const uint4& qs, const float4& ga, const float4& gb) {
    float dv[8], sv[8], o[8];
    unpack8(qd, dv);
    unpack8(qs, sv);
    const float g[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = ok ? rstd1 * (dv[e] * g[e] - m1 - (sv[e] - mean1) * rstd1 * m2) : 0.f;
    return packq8(o);
  };
  auto dpre_of = [&](const uint4& gq, const uint4& pq) {
    float g[8], pv[8], o[8];
    unpack8(gq, g);
    unpack8(pq, pv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = pv[e] * g[e];
    return packq8(o);
  };
  if constexpr (FIN) {
    // wide tile first: dS1 of each of its rows from dh1 / s1 / g1 -> dpre_w into aw; the rows the narrow
    // tile covers also park their dS1 in `an` (the narrow tile's own slot), so dh1 / s1 / g1 are read once
    const int nchw = (BM + 2 * halo_w) * 16;
    const int joff = halo_w - halo_n;                // wide row of narrow row 0
    for (int base = tid; base < nchw; base += 4 * 256) {
      uint4 qd[4], qs[4], pq[4];
      float4 ga[4], gb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = base + i * 256;
        const int pos = pos0 - halo_w + (idx >> 4);
        fin_load(pos, idx & 15, qd[i], qs[i], ga[i], gb[i]);
        pq[i] = *reinterpret_cast<const uint4*>(gdw + sbase + (size_t)min(max(pos, 0), L - 1) * CH + (idx & 15) * 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = base + i * 256;
        if (idx >= nchw) break;
        const int j = idx >> 4, ch = idx & 15;
        const int pos = pos0 - halo_w + j;
        const bool ok = pos >= 0 && pos < L;
        const uint4 dq = fin_ds1(ok, qd[i], qs[i], ga[i], gb[i]);
        const uint4 v = ok ? dpre_of(dq, pq[i]) : make_uint4(0u, 0u, 0u, 0u);
        if (ok && j >= halo_w && j < halo_w + BM)
          *reinterpret_cast<uint4*>(dpre_w + sbase + (size_t)pos * CH + ch * 8) = v;
        *reinterpret_cast<uint4*>(aw + swz256(j, ch)) = v;
        if (j >= joff && j < joff + RN) *reinterpret_cast<uint4*>(an + swz256(j - joff, ch)) = dq;
      }
    }
    __syncthreads();
    // narrow tile (RN = BM + 8 rows x 16 chunks): fully unrolled so the central rows' dS1 stay in
    // registers; each thread converts its own chunks of `an` in place (dS1 -> dpre_n)
    const int nch = RN * 16;
#pragma unroll
    for (int mb = 0; mb < 9; mb += 3) {
      uint4 pq[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int idx = tid + 256 * (mb + i);
        const int pos = pos0 - halo_n + (idx >> 4);
        pq[i] = *reinterpret_cast<const uint4*>(gdn + sbase + (size_t)min(max(pos, 0), L - 1) * CH + (idx & 15) * 8);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int m = mb + i;
        const int idx = tid + 256 * m;
        const int j = idx >> 4, ch = idx & 15;
        const int pos = pos0 - halo_n + j;
        const bool ok = idx < nch && pos >= 0 && pos < L;
        const uint4 dq = idx < nch ? *reinterpret_cast<const uint4*>(an + swz256(j, ch)) : make_uint4(0u, 0u, 0u, 0u);
        keep[m] = dq;
        if (ok && j >= halo_n && j < halo_n + BM) {
          float t[8];
          unpack8(dq, t);
#pragma unroll
          for (int e = 0; e < 8; ++e) csum[e] += t[e];
        }
        if (idx < nch) {
          const uint4 v = ok ? dpre_of(dq, pq[i]) : make_uint4(0u, 0u, 0u, 0u);
          if (ok && j >= halo_n && j < halo_n + BM)
            *reinterpret_cast<uint4*>(dpre_n + sbase + (size_t)pos * CH + ch * 8) = v;
          *reinterpret_cast<uint4*>(an + swz256(j, ch)) = v;
        }
      }
    }
  }
  // stage dpre = dS1 * GELU'(pre) of both convs with their halos; central rows also go to global
#pragma unroll 1
  for (int c = 0; c < (FIN ? 0 : 2); ++c) {
    const int halo = c ? halo_w : halo_n;
    const bf16_t* gd = c ? gdw : gdn;
    bf16_t* dpo = c ? dpre_w : dpre_n;
    unsigned char* tile = c ? aw : an;
    const int nch = (BM + 2 * halo) * 16;
    for (int base = tid; base < nch; base += 4 * 256) {
      uint4 gq[4], pq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = base + i * 256;
        const int pos = pos0 - halo + (idx >> 4);
        const bool ok = idx < nch && pos >= -ilo && pos < L + ihi;
        const ptrdiff_t off = ibase + (ptrdiff_t)(ok ? pos : 0) * CH + (idx & 15) * 8;
        gq[i] = ok ? *reinterpret_cast<const uint4*>(ds1 + off) : make_uint4(0u, 0u, 0u, 0u);
        pq[i] = ok ? *reinterpret_cast<const uint4*>(gd + off) : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = base + i * 256;
        if (idx >= nch) break;
        const int j = idx >> 4, ch = idx & 15;
        const int pos = pos0 - halo + j;
        float g[8], pv[8], o[8];
        unpack8(gq[i], g);
        unpack8(pq[i], pv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = pv[e] * g[e];
        const uint4 v = (pos >= -ilo && pos < L + ihi) ? packq8(o) : make_uint4(0u, 0u, 0u, 0u);
        if (pos >= 0 && pos < L && j >= halo && j < halo + BM)
          *reinterpret_cast<uint4*>(dpo + sbase + (size_t)pos * CH + ch * 8) = v;
        *reinterpret_cast<uint4*>(tile + swz256(j, ch)) = v;
      }
    }
  }
  __syncthreads();

  f32x16_t acc[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) acc[i] = zero16();
  // transposed conv: output row pos reads dpre row pos - (k - half) d, i.e. tile row halo + r - (k - half) d
  auto rows_of = [&](int c, int k, int& rowb, int& gs) {
    const int rb = (c ? halo_w : halo_n) + r - (k - half) * (c ? dil : 1);
    rowb = rb << 8;
    gs = (h ^ (((rb & 3) << 2) | ((rb >> 2) & 3))) << 4;
  };
  bf16x8 bq[2][NPT];
  int rowb, gs;
  rows_of(0, 0, rowb, gs);
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt) bq[0][pt] = lds_frag(an, (0 ^ gs) + rowb + pt * 8192);
#pragma unroll 1
  for (int c = 0; c < 2; ++c) {
    const unsigned char* as = c ? aw : an;
    for (int k = 0; k < KS; ++k) {
      // the step after this tap: next tap of this conv, or the wide conv's first tap
      const int cn = k + 1 < KS ? c : 1, kn = k + 1 < KS ? k + 1 : 0;
      const unsigned char* asn = cn ? aw : an;
      int rowbn, gsn;
      rows_of(cn, kn, rowbn, gsn);
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        const int it = c * NI + k * 8 + kb;
        fr[(kb + 3) & 3] = wfrag(min(it + 3, 2 * NI - 1));
        const unsigned char* nb = kb < 7 ? as : asn;
        const int noff = kb < 7 ? ((32 * (kb + 1)) ^ gs) + rowb : (0 ^ gsn) + rowbn;
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt) bq[(kb + 1) & 1][pt] = lds_frag(nb, noff + pt * 8192);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt) acc[pt] = mfma32(fr[kb & 3], bq[kb & 1][pt], acc[pt]);
      }
      rowb = rowbn;
      gs = gsn;
    }
  }

  // dx = ds1 + acc: the fp32 tile goes through LDS (over the dpre tiles) for row-contiguous 16-B accesses
  const int vrows = min(BM, L - pos0);
  float* ft = reinterpret_cast<float*>(smem);
  auto fidx = [&](int p, int c4) { return p * CH + ((c4 ^ (p & 31)) << 2); };
  __syncthreads();                                // every wave is done reading the dpre tiles
#pragma unroll
  for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c4 = (cq * 32 + 8 * g + 4 * h) >> 2;
      *reinterpret_cast<float4*>(ft + fidx(pt * 32 + r, c4)) =
          make_float4(acc[pt][4 * g], acc[pt][4 * g + 1], acc[pt][4 * g + 2], acc[pt][4 * g + 3]);
    }
  if constexpr (FIN) {
    // dgb partial: the 4 row groups of a wave by shuffles, then the 4 waves through LDS (past the tile)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      csum[e] += __shfl_xor(csum[e], 16, 64);
      csum[e] += __shfl_xor(csum[e], 32, 64);
    }
    float* dsum = ft + BM * CH;                    // [4 waves][128]
    if (lane < 16) {
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum[cq * CH + lane * 8 + e] = csum[e];
    }
  }
  __syncthreads();
  if constexpr (FIN) {
    if (tid < CH) {
      const float* dsum = ft + BM * CH;
      atomicAdd(fa.dgb + (size_t)b * CH + tid, dsum[tid] + dsum[CH + tid] + dsum[2 * CH + tid] + dsum[3 * CH + tid]);
    }
    // dx = dS1 (registers) + acc over the central rows
#pragma unroll
    for (int m = 0; m < 9; ++m) {
      const int row = (tid >> 4) + 16 * m - halo_n, cc = tid & 15;
      if (row < 0 || row >= vrows) continue;
      float gv[8], o[8];
      unpack8(keep[m], gv);
      const float4 f0 = *reinterpret_cast<const float4*>(ft + fidx(row, 2 * cc));
      const float4 f1 = *reinterpret_cast<const float4*>(ft + fidx(row, 2 * cc + 1));
      const float fv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = gv[e] + fv[e];
      *reinterpret_cast<uint4*>(dx + sbase + (size_t)(pos0 + row) * CH + cc * 8) = packq8(o);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < BM * 16 / 256; ++i) {
    const int idx = tid + 256 * i;
    const int row = idx >> 4, cc = idx & 15;
    if (row >= vrows) continue;
    const size_t off = sbase + (size_t)(pos0 + row) * CH + cc * 8;
    float gv[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(ds1 + ibase + (ptrdiff_t)(pos0 + row) * CH + cc * 8), gv);
    const float4 f0 = *reinterpret_cast<const float4*>(ft + fidx(row, 2 * cc));
    const float4 f1 = *reinterpret_cast<const float4*>(ft + fidx(row, 2 * cc + 1));
    const float fv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = gv[e] + fv[e];
    *reinterpret_cast<uint4*>(dx + off) = packq8(o);
  }
}

bool dgrad4_attr_set = false;
}  // namespace

int conv_dgrad4_lds(int dil) {
  const int a = (2 * BM + 8 * (1 + dil)) * 256;
  const int e = BM * CH * 4 + 4 * CH * 4;     // the fp32 dx tile + the FIN dgb partials
  return a > e ? a : e;
}

// KS = 9: gdn / gdw are the GELU'(pre) images the forward (pbx_conv_fwd3x / pbx_conv_fwd3t) stored.
// ilo / ihi: halo rows of ds1 and GELU' from the neighbouring shards (context parallelism; both inputs
// [B][ilo + L + ihi][128]); outputs dx, dpre_n, dpre_w are [B][L][128].  0 / 0 for a whole sequence.
PBX_EXPORT int pbx_conv_dgrad4x(const void* ds1, const void* gdn, const void* gdw, const void* ftn, const void* ftw,
                                void* dx, void* dpre_n, void* dpre_w, int B, int L, int KS_, int dil, int ilo, int ihi,
                                hipStream_t st) {
  const int lds = conv_dgrad4_lds(dil);
  if (KS_ != KS || dil < 1 || lds > 163840 || B < 1 || L < 1 || ilo < 0 || ihi < 0) return (int)hipErrorInvalidValue;
  if (!dgrad4_attr_set) {
    (void)hipFuncSetAttribute((const void*)conv_dgrad4_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    (void)hipFuncSetAttribute((const void*)conv_dgrad4_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    dgrad4_attr_set = true;
  }
  const int T = (L + BM - 1) / BM;
  hipLaunchKernelGGL(conv_dgrad4_kernel<false>, dim3(B * T), dim3(256), lds, st, (const bf16_t*)ds1,
                     (const bf16_t*)gdn, (const bf16_t*)gdw, (const bf16x8*)ftn, (const bf16x8*)ftw, (bf16_t*)dx,
                     (bf16_t*)dpre_n, (bf16_t*)dpre_w, L, dil, ilo, ihi, FinArgs{});
  return pbx_launch_status();
}

// pbx_conv_dgrad4x with the LayerNorm-1 backward finalize fused in (see FinArgs): dh1 / s1 [B][L][128]
// bf16, st1 [B][T1][2] / sums1 [B][TS1][2] the LN1 statistics and backward partials (as
// pbx_ln1_finalize), g1 [L][128]; dgb [B][128] accumulated.  dS1 itself is not written.
PBX_EXPORT int pbx_conv_dgrad4f(const void* dh1, const void* s1, const float* st1, int T1, int BM1, const float* sums1,
                                int TS1, const float* g1, const void* gdn, const void* gdw, const void* ftn,
                                const void* ftw, void* dx, void* dpre_n, void* dpre_w, float* dgb, int B, int L,
                                int KS_, int dil, float eps, hipStream_t st) {
  const int lds = conv_dgrad4_lds(dil);
  if (KS_ != KS || dil < 1 || lds > 163840 || B < 1 || L < 1 || T1 < 1 || BM1 < 1 || TS1 < 1)
    return (int)hipErrorInvalidValue;
  if (!dgrad4_attr_set) {
    (void)hipFuncSetAttribute((const void*)conv_dgrad4_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    (void)hipFuncSetAttribute((const void*)conv_dgrad4_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    dgrad4_attr_set = true;
  }
  const int T = (L + BM - 1) / BM;
  FinArgs fa{(const bf16_t*)dh1, (const bf16_t*)s1, st1, T1, BM1, sums1, TS1, g1, dgb, eps};
  hipLaunchKernelGGL(conv_dgrad4_kernel<true>, dim3(B * T), dim3(256), lds, st, nullptr, (const bf16_t*)gdn,
                     (const bf16_t*)gdw, (const bf16x8*)ftn, (const bf16x8*)ftw, (bf16_t*)dx, (bf16_t*)dpre_n,
                     (bf16_t*)dpre_w, L, dil, 0, 0, fa);
  return pbx_launch_status();
}

