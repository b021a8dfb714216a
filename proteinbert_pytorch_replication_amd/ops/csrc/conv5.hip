// Dual-dilation residue convolution forward, persistent and software-pipelined with a hand-counted memory
// pipeline.
//
// Reference: ProteinBERT/modules.py:124-147 (Conv1d C->C, k=9, dilation 1 and 5, padding "same", each +
// GELU) and :205-212 (x + narrow + wide + broadcast(global->local), LayerNorm over (L, C)).
//
// Why (conv2.hip conv_fwd3): two 512-thread workgroups per CU run their three phases -- x staging (HBM),
// the MFMA loop, the GELU / GELU' epilogue (VALU + stores) -- in lockstep, so the matrix pipe idles for the
// staging and the epilogue (phase stamps 14K / 31K / 25K cycles per wave, profiles/r5/conv_phase_stamps.txt;
// MFMA busy 0.45).  Round 4's persistent conv_fwd4 pipelined the epilogue into the next tile's K loop and
// did not win: every vector-memory operation of the epilogue (its x loads, its stores) and the x-tile DMA
// sat in the same in-order vmcnt queue as the weight-fragment loads, so each fragment wait also waited for
// them (an HBM round trip behind a 3-step-deep fragment ring).
//
// Here ONE workgroup per CU (8 waves, two per SIMD) walks its tiles of 128 positions:
//   * wave w runs conv c = w >> 2 for output channels 32q..32q+31, q = w & 3, over all 128 positions (four
//     32x32 accumulators; one weight fragment per K-step feeds 4 MFMAs);
//   * at the end of a tile each wave parks its pre-activations + bias (bf16: the rounding conv_fwd3's LDS
//     staging applies) in LDS row images and every thread keeps the x values of its 4 epilogue units in
//     registers; in the NEXT tile's 72-step K loop each thread runs its units' epilogue (s1 = x + GELU(n) +
//     GELU(w) + gb, GELU' of both convs, LayerNorm partials) in 32 slices beside its MFMAs -- two waves per
//     SIMD, so a slice's VALU issues while the partner's MFMAs run; stores are row-contiguous 16-B lanes
//     (16 lanes per 256-B row, as conv_fwd3's epilogue: 8-B row-per-lane stores were the bound);
//   * every vector-memory operation of the loop is issued by this kernel in a FIXED per-step schedule --
//     weight fragments (inline-asm global loads, PD steps ahead), the next tile's x rows and gb (global->LDS
//     DMA), the epilogue's stores (buffer stores, out-of-range rows dropped) -- so the vmcnt each fragment
//     wait needs is a compile-time constant (vm_wait below): a fragment wait never waits for a younger DMA
//     or store.  The compiler sees none of the loads, so it inserts no wait of its own.
//   LDS: two x-tile buffers (168 rows x 256 B, swz256), the previous tile's pre-activations (2 x 32 KB row
//   images), gb, biases: 151 KB.
//
// s1 and the GELU' images equal conv_fwd3's bitwise (both keep the GELU product out of FMA contraction;
// tests/test_hip_conv_fwd5.py); the LayerNorm (mean, M2) tile partials sum the same stored values in another
// order.  The inline-asm loads' registers are checked against compiler copies by tools/asm_hazards.py
// (tests/test_asm_hazards.py).
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int CH = 128;
constexpr int BM = 128;               // positions per tile
constexpr int KS = 9;
constexpr int DIL = 5;                // the wide dilation this kernel is built for (paper config)
constexpr int HALO = (KS / 2) * DIL;  // 20
constexpr int XR = BM + 2 * HALO;     // x-tile rows (168 = 42 DMA blocks of 4 rows)
constexpr int XB = XR * 256;          // bytes of one x-tile buffer
constexpr int NS = KS * 8;            // K-steps per tile (taps x 16-channel blocks)
constexpr int NPT = BM / 32;          // 32-position MFMA tiles
constexpr int NW = 8;                 // waves
constexpr int PD = 8;                 // weight-fragment prefetch distance (K-steps): the DMA / store slack
constexpr int NDMA = 11;              // DMAs per wave per tile (narrow waves: 42 x blocks + gb + 1 repeat)
constexpr int DMA0 = 0;               // first K-step carrying a DMA (then every step)
constexpr int NUNIT = 4;              // epilogue units (row, 8-channel chunk) per thread: 128 x 16 / 512
constexpr int NSL = 8 * NUNIT;        // epilogue slices per wave (8 per unit), slice j at step 2 j
constexpr int PRE = 2 * XB;           // LDS: previous tile's pre-activations, [conv][128 rows][256 B] swz256
constexpr int GBUF = PRE + 2 * BM * 256;   // LDS: gb [parity][1 KB]
constexpr int SINK = GBUF + 2048;     // LDS: 1 KB the wide waves' DMAs land in
constexpr int BIAS = SINK + 1024;     // LDS: bn | bw
constexpr int SCR = BIAS + 2 * CH * 4;   // LDS: 8 waves x (sum, sum of squares)
constexpr int LDS5 = SCR + 64;
static_assert(LDS5 <= 163840, "LDS");

__device__ __attribute__((aligned(16))) unsigned int g_zero16_c5[4];   // zero-initialised device global

// ---- the per-step vector-memory schedule of every wave (identical in every round) ----------------------
// step j issues, in this order: the weight fragment of step j + PD, a DMA on steps DMA0 .. DMA0 + NDMA - 1,
// and the stores of epilogue slice j / 2 on even steps < 2 NSL (slice 8u+3: gdn; 8u+7: gdw, then s1).
constexpr bool dma_step(int j) { return j >= DMA0 && j < DMA0 + NDMA; }
template <bool STORE>
constexpr int vm_ops_after_frag(int j) {
  int st = 0;
  if (j % 2 == 0 && j < 2 * NSL) {
    const int part = (j / 2) % 8;
    if (part == 3 && STORE) st = 1;
    if (part == 7) st = STORE ? 2 : 1;
  }
  return (dma_step(j) ? 1 : 0) + st;
}
// vmcnt for the wait at the top of step s: the ops issued after the fragment of step s (issued in step
// s - PD; steps < 0 are the previous round's last steps, which issue fragments only -- and the prologue
// issues fragments 0 .. PD-1 the same way).  Counting only what this kernel issues is safe: an op the count
// misses (a compiler-issued load or store between rounds) only makes the wait stricter.
template <bool STORE>
constexpr int vm_wait(int s) {
  int n = 0;
  const int j0 = s - PD;
  if (j0 >= 0) n += vm_ops_after_frag<STORE>(j0);
  for (int j = j0 + 1; j < s; ++j) n += 1 + (j >= 0 ? vm_ops_after_frag<STORE>(j) : 0);
  return n;
}
constexpr bool vm_fits() {
  for (int s = 0; s < NS; ++s)
    if (vm_wait<true>(s) > 63) return false;
  return true;
}
static_assert(vm_fits(), "vmcnt range");

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// One 1-KiB global->LDS DMA wave instruction: lane i's 16 source bytes land at lds_base + 16 i.
__device__ __forceinline__ void glds16_c5(const void* src, unsigned char* lds_base) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}

// One weight fragment (16 B per lane, 1 KiB per wave) -- invisible to the compiler's vmcnt tracking.
__device__ __forceinline__ bf16x8 wload(const unsigned char* base, unsigned voff) {
  bf16x8 v;
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(v) : "v"(voff), "s"(base) : "memory");
  return v;
}

// two fp32 -> packed bf16 pair (RNE) in one v_cvt_pk_bf16_f32
__device__ __forceinline__ unsigned pk2(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){a, b}, bf16x2_t));
}

// Tile of workgroup j in round rd: the workgroups of one XCD (ids congruent mod 8) take a contiguous run
// of tiles per round, so neighbouring tiles of a sample -- whose halos overlap -- share an L2.
__device__ __forceinline__ long tile_of5(long rd, int G) {
  const int j = blockIdx.x;
  if ((G & 7) == 0) return rd * G + (long)(j & 7) * (G >> 3) + (j >> 3);
  return rd * G + j;
}

template <bool STORE>
__global__ void __launch_bounds__(512, 1) conv_fwd5_kernel(
    const bf16_t* __restrict__ x, const bf16x8* __restrict__ fwn, const bf16x8* __restrict__ fww,
    const float* __restrict__ bn, const float* __restrict__ bw, const float* __restrict__ gbv,
    bf16_t* __restrict__ gdn, bf16_t* __restrict__ gdw, bf16_t* __restrict__ s1, float* __restrict__ stats,
    int B, int L, int xlo, int xhi) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* bias = reinterpret_cast<float*>(smem + BIAS);
  float* scratch = reinterpret_cast<float*>(smem + SCR);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = w & 3, c = w >> 2;                             // channel block, conv (0 narrow, 1 wide)
  const int r = lane & 31, h = lane >> 5;
  const int T = (L + BM - 1) / BM;
  const long NT = (long)B * T;
  const int G = gridDim.x;
  const int XS = L + xlo + xhi;                                // rows per sample of x (CP halo rows around L)
  if (tid < 2 * CH) bias[tid] = tid < CH ? bn[tid] : bw[tid - CH];
  unsigned char* pre = smem + PRE;                             // [conv][128 rows][256 B] swz256

  // DMA i of a round.  The x rows come from HBM: a DMA retires microseconds after its issue, and every
  // fragment wait of the issuing wave behind it (in-order vmcnt) stalls until then -- so only the NARROW
  // waves (c = 0) carry real DMAs: block d = q + 4 i (d < 42: x-tile block d of the tile whose sample rows
  // start at `xrow`, window start position `xp0`, null: no such tile, into `buf`; d = 42: the gb row `grow`
  // (512 B, lanes 0-31) into `gbuf`; d = 43: x block 0 again), while their SIMD partner, a wide wave, keeps
  // the matrix pipe busy; the wide waves issue the same number of DMAs from an L2-hot zero block into a sink
  // (identical vmcnt schedules, one code path).  Branch-free: rows outside the sequence read a zero block.
  auto dma = [&](int i, const bf16_t* xrow, int xp0, unsigned char* buf, const float* grow, unsigned char* gbuf) {
    const int d = q + 4 * i;
    const void* src = (const void*)g_zero16_c5;
    unsigned char* dst = smem + SINK;
    if (d == 42) {
      if (grow != nullptr && lane < 32) src = (const void*)(grow + lane * 4);
      dst = gbuf;
    } else {
      const int blk = d < 42 ? d : d - 43;
      const int row = 4 * blk + (lane >> 4);
      const int chunk = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));   // swz256 image
      const int pos = xp0 + row;
      if (xrow != nullptr && pos >= -xlo && pos < L + xhi) src = (const void*)(xrow + (ptrdiff_t)pos * CH + chunk * 8);
      dst = buf + blk * 1024;
    }
    if (c != 0) {
      src = (const void*)g_zero16_c5;
      dst = smem + SINK;
    }
    glds16_c5(src, dst);
  };
  // sample-row base and window start of tile `tl` (null past the last tile)
  auto tile_src = [&](long tl, const bf16_t*& xrow, int& xp0, const float*& grow) {
    if (tl < NT) {
      const int b = (int)(tl / T), t = (int)(tl - (long)b * T);
      xrow = x + ((size_t)b * XS + xlo) * CH;
      xp0 = t * BM - HALO;
      grow = gbv + (size_t)b * CH;
    } else {
      xrow = nullptr;
      xp0 = 0;
      grow = nullptr;
    }
  };

  // weight fragments of this wave's conv and 32-co block: step it -> fragment (it * 4 + q), 4 KB apart; a
  // running offset (opaque each step: not folded into hoisted addresses) wraps at the tile boundary
  const unsigned char* wb = reinterpret_cast<const unsigned char*>((c ? fww : fwn) + q * 64);
  const unsigned voff = lane * 16;
  bf16x8 fr[PD];                                               // ring: step s uses slot s % PD

  // prologue: tile of round 0 staged synchronously (x blocks only), fragments 0 .. PD-1 in flight
  long tile = tile_of5(0, G);
  {
    const bf16_t* xrow;
    const float* grow;
    int xp0;
    tile_src(tile, xrow, xp0, grow);
    for (int i = 0; i < NDMA; ++i)
      if (q + 4 * i != 42) dma(i, xrow, xp0, smem, nullptr, nullptr);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
  for (int s = 0; s < PD; ++s) fr[s] = wload(wb + s * 4096, voff);
  long wstep = PD * 4096;                                      // byte offset of the next fragment to load

  // the previous tile (its epilogue runs in this round): x values of this thread's 4 units, LN sums
  uint4 pvx[NUNIT];
  long ptile = -1;
  int pvrows = 0;
  f32x2 lns = {0.f, 0.f};
  const float* pgb = reinterpret_cast<const float*>(smem + GBUF);   // read (unused) before tile 0
  // epilogue stores: buffer stores over the tensors; rows past the tile's valid rows (or no previous tile)
  // get an offset past num_records and are dropped
  const int bytes_all = (int)min((long)B * L * CH * 2, 0x7fffff00L);
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(s1, (short)0, bytes_all, 0x00020000);
  const __amdgpu_buffer_rsrc_t rgn = __builtin_amdgcn_make_buffer_rsrc(gdn, (short)0, bytes_all, 0x00020000);
  const __amdgpu_buffer_rsrc_t rgw = __builtin_amdgcn_make_buffer_rsrc(gdw, (short)0, bytes_all, 0x00020000);
  int vo = 0x7ffffff0;                                         // store voffset of unit 0 (unit u: + 32 u rows)
  // this thread's 8-channel chunk: the one whose swz256 slot in row tid / 16 (and tid / 16 + 32 u) is
  // 16 B-slot tid % 16, so the 16 lanes of every ds_read_b128 lane group hit 16 distinct bank quads (the
  // plain chunk tid % 16 puts two rows' 8 chunks on the same quads: 2-way conflicts in conv_fwd3's epilogue)
  const int chunk8 = (tid & 15) ^ ((((tid >> 4) & 3) << 2) | (((tid >> 4) >> 2) & 3));

  // epilogue slice j (0 .. NSL - 1) of the previous tile, in the row layout of conv_fwd3 (unit u: row
  // (tid + 512 u) >> 4 = tid / 16 + 32 u, channels 8 chunk8 .. +7; 16 lanes store one 256-B row): parts 0-3
  // narrow pairs (gdn stored after part 3), 4-7 wide pairs (gdw stored), then s1 = ((x + GELU(n)) +
  // GELU(w)) + gb and the LN sums
  f32x2 egn[4], egw[4], edn[4], edw[4];
  uint4 pn, pw;
  auto epi_slice = [&](auto jc) {
    constexpr int j = decltype(jc)::value;
    constexpr int u = j / 8, part = j % 8;
    const int row = (tid >> 4) + 32 * u;
    const int vou = vo == 0x7ffffff0 || row >= pvrows ? 0x7ffffff0 : vo + u * 32 * CH * 2;
    if constexpr (part == 0) {
      pn = *reinterpret_cast<const uint4*>(pre + swz256(row, chunk8));
      pw = *reinterpret_cast<const uint4*>(pre + BM * 256 + swz256(row, chunk8));
    }
    constexpr int k = part % 4;
    const uint4& src = part < 4 ? pn : pw;
    const unsigned word = k == 0 ? src.x : k == 1 ? src.y : k == 2 ? src.z : src.w;
    const f32x2 in = {__uint_as_float(word << 16), __uint_as_float(word & 0xffff0000u)};
    if constexpr (part < 4) {
      if constexpr (STORE) gelu_n<1, 2>(&in, &egn[k], &edn[k]);
      else gelu_n<1, 0>(&in, &egn[k], nullptr);
      if constexpr (part == 3 && STORE)
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){pk2(edn[0].x, edn[0].y), pk2(edn[1].x, edn[1].y),
                                                       pk2(edn[2].x, edn[2].y), pk2(edn[3].x, edn[3].y)},
                                               rgn, vou, 0, 0);
    } else {
      if constexpr (STORE) gelu_n<1, 2>(&in, &egw[k], &edw[k]);
      else gelu_n<1, 0>(&in, &egw[k], nullptr);
      if constexpr (part == 7) {
        if constexpr (STORE)
          __builtin_amdgcn_raw_buffer_store_b128((u32x4){pk2(edw[0].x, edw[0].y), pk2(edw[1].x, edw[1].y),
                                                         pk2(edw[2].x, edw[2].y), pk2(edw[3].x, edw[3].y)},
                                                 rgw, vou, 0, 0);
        const float4 ga = *reinterpret_cast<const float4*>(pgb + chunk8 * 8);
        const float4 gb4 = *reinterpret_cast<const float4*>(pgb + chunk8 * 8 + 4);
        const float gv[8] = {ga.x, ga.y, ga.z, ga.w, gb4.x, gb4.y, gb4.z, gb4.w};
        const unsigned xw[4] = {pvx[u].x, pvx[u].y, pvx[u].z, pvx[u].w};
        unsigned p[4];
        float sa = 0.f, sq = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // ((x + GELU(n)) + GELU(w)) + gb, the order and roundings of conv_fwd3 -- no FMA contraction of the
          // GELU product into the adds, in either kernel (scalar: packed f32 beside MFMAs costs more)
#pragma clang fp contract(off)
          const float o0 = ((__uint_as_float(xw[e] << 16) + egn[e].x) + egw[e].x) + gv[2 * e];
          const float o1 = ((__uint_as_float(xw[e] & 0xffff0000u) + egn[e].y) + egw[e].y) + gv[2 * e + 1];
          p[e] = pk2(o0, o1);
          const float r0 = __uint_as_float(p[e] << 16), r1 = __uint_as_float(p[e] & 0xffff0000u);   // stored
          sa += r0 + r1;
          sq = fmaf(r0, r0, fmaf(r1, r1, sq));
        }
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){p[0], p[1], p[2], p[3]}, rs1, vou, 0, 0);
        const bool okr = vou != 0x7ffffff0;
        lns.x += okr ? sa : 0.f;
        lns.y += okr ? sq : 0.f;
      }
    }
  };

  // LN partial of the previous tile: the 8 waves' sums through LDS (after the round's barrier)
  auto finish_stats = [&]() {
    if (tid == 0 && ptile >= 0) {
      float sa = 0.f, sq = 0.f;
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        sa += scratch[2 * i];
        sq += scratch[2 * i + 1];
      }
      const float n = (float)(pvrows * CH), mu = sa / n;
      stats[ptile * 2] = mu;
      stats[ptile * 2 + 1] = fmaxf(sq - sa * mu, 0.f);
    }
  };
  auto reduce_stats = [&]() {
    const float sa = wave_reduce_sum(lns.x), sq = wave_reduce_sum(lns.y);
    if (lane == 0) {
      scratch[2 * w] = sa;
      scratch[2 * w + 1] = sq;
    }
    lns = (f32x2){0.f, 0.f};
  };
  auto set_prev = [&](long pt_, int pbb, int pp0) {
    vo = pt_ >= 0 ? ((pbb * L + pp0 + (tid >> 4)) * CH + chunk8 * 8) * 2 : 0x7ffffff0;
  };
  const int dl = c ? DIL : 1;

  for (long rd = 0;; ++rd) {
    tile = tile_of5(rd, G);
    if (tile >= NT) break;
    unsigned char* xs = smem + (rd & 1) * XB;
    unsigned char* nxt = smem + ((rd + 1) & 1) * XB;
    unsigned char* gcur = smem + GBUF + (rd & 1) * 1024;       // this tile's gb (DMA'd this round)
    const int b = (int)(tile / T), t = (int)(tile - (long)b * T);
    const int pos0 = t * BM;
    const bf16_t* nxrow;
    const float* ngrow;
    int nxp0;
    tile_src(tile_of5(rd + 1, G), nxrow, nxp0, ngrow);        // the next tile's x rows (DMA'd this round)
    const float* cgrow = gbv + (size_t)b * CH;                 // this tile's gb row (DMA'd this round)
    // per-tap B-fragment rows: an opaque copy of r keeps the 9 row offsets from being hoisted out of the
    // round loop (they would stay live across it)
    int rr = r;
    asm volatile("" : "+v"(rr));
    f32x16_t acc[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) acc[i] = zero16();
    // B fragment of (tap k, block kb): row rb = HALO + r + (k - 4) d (+ 32 pt), chunk 2 kb + h of the
    // swz256 tile = ((32 kb) ^ gs) + (rb << 8), gs = (h ^ swz(rb)) << 4
    int rowb = 0, gsw = 0;
    auto tap_rows = [&](int k) {
      const int rb = HALO + rr + (k - KS / 2) * dl;
      rowb = rb << 8;
      gsw = (h ^ (((rb & 3) << 2) | ((rb >> 2) & 3))) << 4;
    };
    bf16x8 bq[2][NPT];
    tap_rows(0);
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) bq[0][pt] = lds_frag(xs, (0 ^ gsw) + rowb + pt * 8192);
    static_for<0, NS>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      constexpr int slot = s % PD;
      // the fragment of step s (issued PD steps ago) -- and nothing younger -- has landed
      // ("memory": no store of an earlier slice may sink below this wait -- it is counted as issued)
      asm volatile("s_waitcnt vmcnt(%1)" : "+v"(fr[slot]) : "n"(vm_wait<STORE>(s)) : "memory");
      const bf16x8 af = fr[slot];
      asm volatile("" : "+s"(wstep));                          // opaque: not folded into hoisted addresses
      fr[slot] = wload(wb + wstep, voff);                      // fragment of step s + PD (mod NS)
      wstep = (s + PD + 1) % NS == 0 ? 0 : wstep + 4096;
      if constexpr (dma_step(s)) dma(s - DMA0, nxrow, nxp0, nxt, cgrow, gcur);
      if constexpr (s % 2 == 0 && s / 2 < NSL) epi_slice(std::integral_constant<int, s / 2>{});
      if constexpr (s + 1 < NS) {
        constexpr int k1 = (s + 1) / 8, kb1 = (s + 1) % 8;
        if constexpr (kb1 == 0) tap_rows(k1);
        const int o = ((32 * kb1) ^ gsw) + rowb;
#pragma unroll
        for (int pt = 0; pt < NPT; ++pt) bq[(s + 1) & 1][pt] = lds_frag(xs, o + pt * 8192);
      }
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) acc[pt] = mfma32(af, bq[s & 1][pt], acc[pt]);
      // one MFMA, then a few VALU (the epilogue slice) and one LDS read in its shadow
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    // this tile becomes the previous one: x values of this wave's epilogue rows (the buffer is the next
    // round's DMA target), pre-activations + bias as bf16 into channel block q's LDS slots (this wave's
    // conv half of every 16-B unit) -- after a barrier: the partner wave of channel block q may still be
    // reading the previous tile's slots in its last epilogue slices; the LN sums of the tile that just
    // finished its epilogue go through LDS
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    reduce_stats();
#pragma unroll
    for (int u = 0; u < NUNIT; ++u)
      pvx[u] = *reinterpret_cast<const uint4*>(xs + swz256(HALO + (tid >> 4) + 32 * u, chunk8));
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int co = q * 32 + 8 * g + 4 * h;
        const float4 b4 = *reinterpret_cast<const float4*>(bias + c * CH + co);
        const uint2 v = make_uint2(pk2(acc[pt][4 * g] + b4.x, acc[pt][4 * g + 1] + b4.y),
                                   pk2(acc[pt][4 * g + 2] + b4.z, acc[pt][4 * g + 3] + b4.w));
        *reinterpret_cast<uint2*>(pre + c * BM * 256 + swz256e(pt * 32 + r, co)) = v;
      }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // x tile read, pre + scratch written, DMAs landed
    finish_stats();
    ptile = tile;
    pvrows = min(BM, L - pos0);
    set_prev(ptile, b, pos0);
    pgb = reinterpret_cast<const float*>(gcur);
  }
  // the last tile's epilogue
  if (ptile >= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");           // its gb (DMA) landed
    static_for<0, NSL>([&](auto jc) { epi_slice(jc); });
    reduce_stats();
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    finish_stats();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no fragment load outlives the kernel
}

bool conv5_attrs_set = false;
}  // namespace

// Whole-sequence (xlo = xhi = 0) or context-parallel (halo rows around each sample) conv forward, dilation 5
// only; same contract as pbx_conv_fwd3x (csrc/conv2.hip).  Grid: one workgroup per CU.
PBX_EXPORT int pbx_conv_fwd5x(const void* x, const void* fwn, const void* fww, const float* bn, const float* bw,
                              const float* gb, void* gdn, void* gdw, void* s1, float* stats, int B, int L, int KS_,
                              int dil, int xlo, int xhi, hipStream_t st) {
  if (KS_ != KS || dil != DIL || B < 1 || L < 1 || xlo < 0 || xhi < 0 || gb == nullptr) return (int)hipErrorInvalidValue;
  if ((gdn == nullptr) != (gdw == nullptr)) return (int)hipErrorInvalidValue;
  if ((long)B * L * CH * 2 > 0x7fffff00L) return (int)hipErrorInvalidValue;   // buffer-store offsets are 32-bit
  if (!conv5_attrs_set) {
    (void)hipFuncSetAttribute((const void*)conv_fwd5_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    (void)hipFuncSetAttribute((const void*)conv_fwd5_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    conv5_attrs_set = true;
  }
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const long NT = (long)B * ((L + BM - 1) / BM);
  const int grid = (int)(NT < ncu ? NT : ncu);
  const int lds = LDS5;
  const auto kern = gdn != nullptr ? conv_fwd5_kernel<true> : conv_fwd5_kernel<false>;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, st, (const bf16_t*)x, (const bf16x8*)fwn, (const bf16x8*)fww,
                     bn, bw, gb, (bf16_t*)gdn, (bf16_t*)gdw, (bf16_t*)s1, stats, B, L, xlo, xhi);
  return pbx_launch_status();
}
