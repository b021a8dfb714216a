// Conv data gradient with the LayerNorm-1 backward finalize (SURVEY K3 + K5), wave-specialised and
// persistent.  Same math and outputs as conv_dgrad4<FIN> (conv4.hip); reference ProteinBERT/modules.py:124-147,
// 205-212 (the backward of x + narrow + wide + broadcast, LayerNorm over (L, C)).
//
// Why: conv_dgrad4<FIN> runs three phases per 128-position tile -- a prologue that loads dh1 / s1 / g1 and
// both GELU' images for the tile and its halos, finalises dS1 and stages dpre = dS1 GELU' (HBM-bound), the
// MFMA loop over both convolutions, and the dx epilogue -- and the two workgroups sharing a CU run them in
// lockstep (stamps: 50K / 31K / 5K cycles per wave, profiles/r5/conv_phase_stamps.txt), so the matrix pipe
// idles through every prologue and HBM idles through every MFMA loop.  (A persistent form that ran the next
// tile's prologue inside the MFMA loop of the same waves lost: HBM loads and L2 weight fragments share one
// in-order vmcnt, so every weight wait also waited for HBM.)
//
// Here ONE workgroup per CU holds 4 MFMA waves (one per SIMD: weight fragments from L2, dpre fragments from
// LDS, then dx = dS1 + conv^T dpre straight from the accumulators) and NSW staging waves (dh1 / s1 / g1 /
// GELU' loads in a register ring that runs on across tiles, dS1 = LN1-backward finalise -> dx, dpre = dS1
// GELU' -> LDS + HBM, dgb column sums).  Two LDS buffers alternate -- the MFMA waves read tile i from
// buf[i & 1] while the staging waves fill buf[(i+1) & 1] -- and one barrier per tile hands them over.  The
// per-sample LN1 constants (mean, rstd, and the two backward means) come from a one-wave-per-sample pre-pass.
//
// Staging unit: (wide-tile row j, 16-B channel chunk c16); staging thread p owns NCU central units (rows
// halo_w + p/16 + RS m) and NHU halo units (rows p/16 + RS q of the 2 halo_w halo rows; the rest are empty),
// chunk p & 15.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int BM = 128;              // positions per tile
constexpr int KS = 9;
constexpr int NI = KS * 8;           // K-steps per convolution
constexpr int NPT = BM / 32;         // 32-position MFMA tiles per wave
#ifndef PBX_DGRAD5_NSW
#define PBX_DGRAD5_NSW 4
#endif
constexpr int NSW = PBX_DGRAD5_NSW;  // staging waves (after the 4 MFMA waves)
constexpr int NST = 64 * NSW;        // staging threads
constexpr int NTH = 256 + NST;
constexpr int RS = NST / 16;         // row stride of a staging thread's units
constexpr int NCU = BM / RS;         // central units per staging thread
constexpr int NHU = (64 + RS - 1) / RS;   // halo unit slots (2 halo_w = 8 dil <= 40 rows used for dil <= 5)
constexpr int NU = NCU + NHU;        // units per tile (12 for NSW = 4)
#ifndef PBX_DGRAD5_R
#define PBX_DGRAD5_R 4
#endif
constexpr int R = PBX_DGRAD5_R;      // staging load ring: R - 1 units in flight ahead of the one computed
static_assert(NU % R == 0, "the ring slot of a unit must not depend on the tile");
constexpr int RING = 12;             // MFMA waves: weight-fragment ring

#ifdef PBX_STAMPS   // instrumented builds only (tools/ubench/dgrad5stamps.py): per workgroup and wave, cycles per phase
__device__ unsigned long long pbx_dgrad5_stamps[256 * 16 * 8];
#define D5_STAMP(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); sacc[k] += t_ - slast; slast = t_; } while (0)
#else
#define D5_STAMP(k) do { } while (0)
#endif

struct Fin5 {
  const bf16_t* dh1;
  const bf16_t* s1;
  const float4* lnc;      // [B] (mean1, rstd1, m1, m2) from ln1_consts_kernel
  const float* g1;        // [L][128] LN1 affine weight
  float* dgb;             // [B][128] accumulated
};

struct UnitIn {                      // one unit's operands in flight
  uint4 dh, s, gw, gn;
  float4 ga, gb;
};

// Every global access of the kernel is a raw buffer op and every masked-out lane gets an out-of-range offset
// (loads return 0 and move nothing, stores and atomics are dropped): no branches, so the compiler's
// wait-count bookkeeping never meets a control-flow join and the load ring stays in flight across tiles.
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
constexpr unsigned OOB = 0x80000000u;  // every tensor here is < 2 GiB (checked by the launcher)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ uint4 ld16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float4 ld16f(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, unsigned off, const uint4& q) {
  u32x4 v;
  v.x = q.x; v.y = q.y; v.z = q.z; v.w = q.w;
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}

// per-sample LN1 constants, one wave per sample
__global__ void __launch_bounds__(256) ln1_consts_kernel(const float* __restrict__ st1, int T1, int BM1,
                                                         const float* __restrict__ sums1, int TS1, int B, int L,
                                                         float eps, float4* __restrict__ lnc) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float mean1, rstd1, m1, m2;
  wave_ln_stats(st1 + (size_t)b * T1 * 2, T1, BM1, L, CH, eps, mean1, rstd1);
  wave_bwd_consts(sums1 + (size_t)b * TS1 * 2, TS1, 1.0f / (float)(L * CH), m1, m2);
  if ((threadIdx.x & 63) == 0) lnc[b] = make_float4(mean1, rstd1, m1, m2);
}

__global__ void __launch_bounds__(NTH, 1) conv_dgrad5_kernel(
    const bf16_t* __restrict__ gdn, const bf16_t* __restrict__ gdw, const bf16x8* __restrict__ ftn,
    const bf16x8* __restrict__ ftw, bf16_t* __restrict__ dx, bf16_t* __restrict__ dpre_n,
    bf16_t* __restrict__ dpre_w, int L, int dil, int ntiles, Fin5 fa) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = (L + BM - 1) / BM;
  const int half = KS >> 1;
  const int halo_n = half, halo_w = half * dil;
  const int RN = BM + 2 * halo_n, RW = BM + 2 * halo_w;
  const int BUF = (RN + RW) * 256;                  // one buffer: narrow dpre | wide dpre (swz256)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int v0 = blockIdx.x;
  if (v0 >= ntiles) return;
  const int n = (ntiles - v0 + G - 1) / G;          // tiles of this workgroup: v0, v0 + G, ...
  auto tile_of = [&](int i) {     // XCD-contiguous runs of tiles (conv2.hip tile_id)
    const int v = v0 + i * G;
    const int xcd = v & 7, q = ntiles >> 3, rr = ntiles & 7;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (v >> 3);
  };
  auto buf = [&](int i) { return smem + (i & 1) * BUF; };
  const unsigned tbytes = (unsigned)(ntiles / T) * (unsigned)L * 256u;   // one [B, L, 128] bf16 tensor
  const __amdgpu_buffer_rsrc_t r_dx = rsrc(dx, tbytes);
#ifdef PBX_STAMPS
  unsigned long long sacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long slast = __builtin_amdgcn_s_memtime();
  auto stamps_out = [&]() {
    if (lane == 0 && blockIdx.x < 256) {
      unsigned long long* o = pbx_dgrad5_stamps + ((size_t)blockIdx.x * 16 + wave) * 8;
      for (int k = 0; k < 8; ++k) o[k] = sacc[k];
    }
  };
#else
  auto stamps_out = [&]() {};
#endif

  if (wave < 4) {
    // ===================== MFMA waves =====================
    const int cq = wave, r = lane & 31, h = lane >> 5;
#ifdef PBX_D5_PRIO
    __builtin_amdgcn_s_setprio(PBX_D5_PRIO);
#endif
    const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16x8*>(ftn + cq * 64), (short)0, (NI * 4 - cq) * 1024, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16x8*>(ftw + cq * 64), (short)0, (NI * 4 - cq) * 1024, 0x00020000);
    auto wfrag = [&](int it) {    // K-step it of 2 NI: narrow image for it < NI, then the wide one
      typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
      const int li = it < NI ? it : it - NI;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(it < NI ? rn : rw, lane * 16, li * 4096, 0);
      return __builtin_bit_cast(bf16x8, v);
    };
    int ro = r, ho = h;                              // lane terms, re-derived per tile (see below)
    // transposed conv: output row pos reads dpre row pos - (k - half) d, i.e. tile row halo + r - (k - half) d
    auto rows_of = [&](int c, int k, int& rowb, int& gs) {
      const int rb = (c ? halo_w : halo_n) + ro - (k - half) * (c ? dil : 1);
      rowb = rb << 8;
      gs = (ho ^ (((rb & 3) << 2) | ((rb >> 2) & 3))) << 4;
    };
    __syncthreads();                                 // P0: tile 0 staged
    D5_STAMP(7);
    for (int i = 0; i < n; ++i) {
      unsigned char* cur = buf(i);
      const int tile = tile_of(i);
      const int b = tile / T, pos0 = (tile - b * T) * BM;
      // an opaque zero: without it the 144 per-step LDS addresses are hoisted out of the tile loop as
      // invariants and held in (spilled) registers
      int zo;
      asm volatile("v_mov_b32 %0, 0" : "=v"(zo));
      ro = r + zo;
      ho = h + zo;
      f32x16_t acc[NPT];
#pragma unroll
      for (int t = 0; t < NPT; ++t) acc[t] = zero16();
      bf16x8 fr[RING];
#pragma unroll
      for (int s = 0; s < RING - 1; ++s) fr[s] = wfrag(s);
      // this lane's dS1 (the staging waves wrote it into dx before the barrier): rows t*32 + r, channels
      // cq*32 + 8 g + 4 h + 0..3 -- the accumulator layout; issued after the weight prologue, so the first
      // wait on it comes RING - 1 steps into the loop
      unsigned xo[NPT];
      u32x2 ds[NPT][4];
#pragma unroll
      for (int t = 0; t < NPT; ++t) {
        const int row = t * 32 + r;
        xo[t] = row < L - pos0 ? (((unsigned)(b * L + pos0 + row)) * CH + cq * 32 + 4 * h) * 2u : OOB;
#pragma unroll
        for (int g = 0; g < 4; ++g) ds[t][g] = __builtin_amdgcn_raw_buffer_load_b64(r_dx, xo[t] + 16 * g, 0, 0);
      }
      bf16x8 bq[2][NPT];
      int rowb, gs;
      rows_of(0, 0, rowb, gs);
#pragma unroll
      for (int t = 0; t < NPT; ++t) bq[0][t] = lds_frag(cur, (0 ^ gs) + rowb + t * 8192);
#ifndef PBX_ABL_NOMFMA
#pragma unroll
      for (int it = 0; it < 2 * KS; ++it) {        // tap-iterations: narrow taps 0..8, then wide 0..8
        const int c = it / KS;
        const unsigned char* as = cur + (c ? RN * 256 : 0);
        const int cn = it + 1 < 2 * KS ? (it + 1) / KS : 1, kn = it + 1 < 2 * KS ? (it + 1) % KS : KS - 1;
        const unsigned char* asn = cur + (cn ? RN * 256 : 0);
        int rowbn, gsn;
        rows_of(cn, kn, rowbn, gsn);
#pragma unroll
        for (int kb = 0; kb < 8; ++kb) {
          const int s = it * 8 + kb;
          fr[(s + RING - 1) % RING] = wfrag(min(s + RING - 1, 2 * NI - 1));
          const unsigned char* nb = kb < 7 ? as : asn;
          const int noff = kb < 7 ? ((32 * (kb + 1)) ^ gs) + rowb : (0 ^ gsn) + rowbn;
#pragma unroll
          for (int t = 0; t < NPT; ++t) bq[(kb + 1) & 1][t] = lds_frag(nb, noff + t * 8192);
          __builtin_amdgcn_sched_barrier(0);     // keep the prefetch distances (the scheduler would sink them)
#pragma unroll
          for (int t = 0; t < NPT; ++t) acc[t] = mfma32(fr[s % RING], bq[kb & 1][t], acc[t]);
        }
        rowb = rowbn;
        gs = gsn;
      }
#endif
      D5_STAMP(0);                                 // MFMA loop
      // dx = dS1 + conv^T dpre, 4 channels (8 B) per store
#pragma unroll
      for (int t = 0; t < NPT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float d4[4], o[4];
          unpack4(make_uint2(ds[t][g].x, ds[t][g].y), d4);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = d4[e] + acc[t][4 * g + e];
          const uint2 q = packq4(o);
          u32x2 v;
          v.x = q.x;
          v.y = q.y;
          __builtin_amdgcn_raw_buffer_store_b64(v, r_dx, xo[t] + 16 * g, 0, 0);
        }
      D5_STAMP(1);                                 // epilogue
      // P: MFMA reads of `cur` done (the dx stores need no completion: nobody in the workgroup reads them)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      D5_STAMP(2);
    }
    stamps_out();
    return;
  }

  // ===================== staging waves =====================
  const int p = tid - 256;
  const int c16 = p & 15, jt = p >> 4;
  const int joff = halo_w - halo_n;                 // wide row of narrow row 0
  const __amdgpu_buffer_rsrc_t r_dh = rsrc(fa.dh1, tbytes), r_s = rsrc(fa.s1, tbytes), r_gw = rsrc(gdw, tbytes),
                               r_gn = rsrc(gdn, tbytes), r_pw = rsrc(dpre_w, tbytes), r_pn = rsrc(dpre_n, tbytes),
                               r_g1 = rsrc(fa.g1, (unsigned)L * 512u),
                               r_dgb = rsrc(fa.dgb, (unsigned)(ntiles / T) * 512u);
  const int sink = 2 * BUF + p * 16;                // LDS slot for the stores of masked-out units
  auto row_of = [&](int u) {                        // wide-tile row of unit u (>= RW: no such row)
    if (u < NCU) return halo_w + jt + RS * u;
    const int hr = jt + RS * (u - NCU);
    return hr < 2 * halo_w ? (hr < halo_w ? hr : hr + BM) : RW;
  };
  auto unit_load = [&](int b, int pos0, bool valid, int u, UnitIn& in) {
    const int j = row_of(u);
    const int q = min(max(pos0 - halo_w + j, 0), L - 1);
    const bool ld = valid && j < RW;
    const unsigned off = ld ? ((unsigned)(b * L + q) * CH + c16 * 8) * 2u : OOB;
    const unsigned go = ld ? ((unsigned)q * CH + c16 * 8) * 4u : OOB;
    in.dh = ld16(r_dh, off);
    in.s = ld16(r_s, off);
    in.gw = ld16(r_gw, off);
    in.gn = ld16(r_gn, off);
    in.ga = ld16f(r_g1, go);
    in.gb = ld16f(r_g1, go + 16);
  };
  auto dpre_of = [&](const uint4& gq, const uint4& pq) {
    float g[8], pv[8], o[8];
    unpack8(gq, g);
    unpack8(pq, pv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = pv[e] * g[e];
    return packq8(o);
  };
  UnitIn ring[R];
  float csum[8];
  // unit u of tile (b, pos0): dS1 -> dx (central rows), dpre_w / dpre_n -> LDS tile + HBM (central rows)
  auto unit_compute = [&](int b, int pos0, const float4& lc, int u, const UnitIn& in, unsigned char* bb) {
    const int j = row_of(u);
    const int pos = pos0 - halo_w + j;
    const bool ok = j < RW && pos >= 0 && pos < L;
    float dv[8], sv[8], o[8];
    unpack8(in.dh, dv);
    unpack8(in.s, sv);
    const float g[8] = {in.ga.x, in.ga.y, in.ga.z, in.ga.w, in.gb.x, in.gb.y, in.gb.z, in.gb.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = lc.y * (dv[e] * g[e] - lc.z - (sv[e] - lc.x) * lc.y * lc.w);
    // masks, not `ok ? x : 0`: the compiler turns those into one exec-mask branch per element
    const unsigned mk = ok ? ~0u : 0u;
    auto msk = [&](uint4 q) { return make_uint4(q.x & mk, q.y & mk, q.z & mk, q.w & mk); };
    const uint4 dq = msk(packq8(o));                // dS1, rounded as ln1_finalize stores it
    const uint4 vw = msk(dpre_of(dq, in.gw)), vn = msk(dpre_of(dq, in.gn));
    const int jn = j - joff;
    *reinterpret_cast<uint4*>(smem + (j < RW ? (int)(bb - smem) + RN * 256 + swz256(j, c16) : sink)) = vw;
    *reinterpret_cast<uint4*>(smem + (jn >= 0 && jn < RN ? (int)(bb - smem) + swz256(jn, c16) : sink)) = vn;
    if (u < NCU) {                                  // central rows (compile-time): HBM outputs, dgb sums
#ifdef PBX_ABL_NOGST
      const unsigned go = OOB;
#else
      const unsigned go = pos < L ? ((unsigned)(b * L + pos) * CH + c16 * 8) * 2u : OOB;
#endif
      st16(r_dx, go, dq);                           // dx = dS1 + ...: the MFMA waves add the product
      st16(r_pw, go, vw);
      st16(r_pn, go, vn);
      float t8[8];
      unpack8(dq, t8);
#pragma unroll
      for (int e = 0; e < 8; ++e) csum[e] += t8[e];
    }
  };
  float4 lcn = fa.lnc[tile_of(0) / T];
  // tile i -> buf(i); the ring holds its units 0..R-2 on entry and the next tile's on exit (out-of-range
  // loads after the last tile)
  auto stage = [&](int i) {
    const int tile = tile_of(i);
    const int b = tile / T, pos0 = (tile - b * T) * BM;
    const bool more = i + 1 < n;
    const int tn = more ? tile_of(i + 1) : tile;
    const int bn = tn / T, pos0n = (tn - bn * T) * BM;
    const float4 lc = lcn;
    unsigned char* bb = buf(i);
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int un = u + R - 1;                     // the unit whose loads go out now
      if (un == NU) lcn = fa.lnc[bn];
      if (un < NU) unit_load(b, pos0, true, un, ring[un % R]);
      else unit_load(bn, pos0n, more, un - NU, ring[un % R]);
      unit_compute(b, pos0, lc, u, ring[u % R], bb);
      if (u == NCU - 1) {                           // dgb partial: lanes with the same chunk, then atomics
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          csum[e] += __shfl_xor(csum[e], 16, 64);
          csum[e] += __shfl_xor(csum[e], 32, 64);
          __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(csum[e], r_dgb,
                                                          lane < 16 ? (unsigned)(b * CH + lane * 8 + e) * 4u : OOB, 0, 0);
        }
        // the rest of the stage issues only LDS stores and the loads of unit NU-1 and the next tile's
        // units 0..R-2 (R-1 units x 6 loads after every global store of this tile: see the barrier)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // P: this tile's LDS stores done, and its global stores complete -- all but the next tile's prefetch
  // loads, the youngest 6 (R-1) vector-memory ops, which stay in flight across the barrier
  auto barrier_p = [&]() {
    static_assert(R == 4, "the wait count below is 6 * (R - 1)");
    asm volatile("s_waitcnt vmcnt(18) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  {
    const int t0 = tile_of(0);
    const int b = t0 / T, pos0 = (t0 - b * T) * BM;
#pragma unroll
    for (int u = 0; u < R - 1; ++u) unit_load(b, pos0, true, u, ring[u]);
  }
#ifndef PBX_ABL_NOSTAGE
  stage(0);
#endif
  D5_STAMP(6);
  barrier_p();                                      // P0
  D5_STAMP(7);
  for (int i = 0; i + 1 < n; ++i) {                 // iteration i: stage(i+1) | P
#ifndef PBX_ABL_NOSTAGE
    stage(i + 1);
#endif
    D5_STAMP(0);                                    // stage
    barrier_p();
    D5_STAMP(1);
  }
  __builtin_amdgcn_s_barrier();                     // the MFMA waves' last P
  stamps_out();
}

bool dgrad5_attr_set = false;
int dgrad5_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
  }
  return n;
}
}  // namespace

int conv_dgrad5_lds(int dil) {
  return 2 * ((BM + 8) + (BM + 8 * dil)) * 256 + NST * 16;   // + the masked-store sink
}

#ifdef PBX_STAMPS
PBX_EXPORT int pbx_dgrad5_stamps_read(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(pbx_dgrad5_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif

// Whole sequences (no CP halos), KS = 9, dil <= 5 (two LDS buffers); same arguments and outputs as
// pbx_conv_dgrad4f (conv4.hip), which stays the form for other shapes, plus lnc: [B] float4 scratch for the
// per-sample LN1 constants.
PBX_EXPORT int pbx_conv_dgrad5f(const void* dh1, const void* s1, const float* st1, int T1, int BM1, const float* sums1,
                                int TS1, const float* g1, const void* gdn, const void* gdw, const void* ftn,
                                const void* ftw, void* dx, void* dpre_n, void* dpre_w, float* dgb, float* lnc, int B,
                                int L, int KS_, int dil, float eps, hipStream_t st) {
  const int lds = conv_dgrad5_lds(dil);
  if (KS_ != KS || dil < 1 || dil > 5 || lds > 163840 || B < 1 || L < 1 || T1 < 1 || BM1 < 1 || TS1 < 1)
    return (int)hipErrorInvalidValue;
  if (8 * dil > NHU * RS || (size_t)B * L * 256 >= (size_t)OOB) return (int)hipErrorInvalidValue;
  if (!dgrad5_attr_set) {
    (void)hipFuncSetAttribute((const void*)conv_dgrad5_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    dgrad5_attr_set = true;
  }
  hipLaunchKernelGGL(ln1_consts_kernel, dim3((B + 3) / 4), dim3(256), 0, st, st1, T1, BM1, sums1, TS1, B, L, eps,
                     reinterpret_cast<float4*>(lnc));
  const int T = (L + BM - 1) / BM;
  const int ntiles = B * T;
  int grid = dgrad5_cus();
  grid = grid < ntiles ? grid : ntiles;
  Fin5 fa{(const bf16_t*)dh1, (const bf16_t*)s1, reinterpret_cast<const float4*>(lnc), g1, dgb};
  hipLaunchKernelGGL(conv_dgrad5_kernel, dim3(grid), dim3(NTH), lds, st, (const bf16_t*)gdn, (const bf16_t*)gdw,
                     (const bf16x8*)ftn, (const bf16x8*)ftw, (bf16_t*)dx, (bf16_t*)dpre_n, (bf16_t*)dpre_w, L, dil,
                     ntiles, fa);
  return pbx_launch_status();
}
