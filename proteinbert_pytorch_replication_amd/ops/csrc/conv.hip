// Dual-dilation residue convolutions of the ProteinBERT local track (SURVEY K3/K4/K5, 61 % of FLOPs).
//
// Reference: ProteinBERT/modules.py:124-147 (two Conv1d C->C, k=9, dilation 1 and 5, padding
// "same", each followed by GELU) and :205-212 (x + narrow + wide + broadcast(global->local), then
// LayerNorm over (L, C)).  The reference runs each conv as a separate cuDNN/MIOpen call on
// [B, C, L] tensors plus ~6 elementwise kernels; here, channels-last [B*L, 128] bf16:
//
//   conv_fwd   : ONE implicit-GEMM launch for both convs.  A workgroup owns BM positions of one
//                sequence; the x tile (+/- 20-row halo, zero outside the sequence) is staged in LDS
//                once and read at the 9 narrow and 9 wide tap shifts; weights stream per half-tap
//                (both convs, 32 KB) through a double-buffered LDS ring.  Epilogue fuses bias,
//                GELU x2, residual, the broadcast global->local vector and per-tile LayerNorm
//                (mean, M2) partials; it writes s1 (LN input) and the two pre-activations.
//   conv_dgrad : dX = dS1 + sum_taps W_n^T dpre_n[.-s] + W_w^T dpre_w[.-s]; dpre = dS1 * GELU'(pre)
//                is formed while staging (and written once for the weight gradient).
//   wgrad      : dW[tap][co][ci] = sum_pos dpre[pos][co] x[pos+s][ci] with both operands read
//                transposed from LDS (ds_read_b64_tr_b16), all 9 taps per workgroup, split over
//                position chunks into fp32 slabs that wgrad_reduce sums (deterministic).
//                The same kernel (KS=1) is the Linear weight gradient of the local MLP.
//
// Every GEMM is v_mfma_f32_32x32x16_bf16 (wave64), fp32 accumulation.  Specialised for C = 128
// channels (the paper's local_dim); other widths run the eager path.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;

// ------------------------------------------------------------------------------------------------
// forward: 512 threads = 8 waves, wave (wm = w>>1, wn = w&1) owns positions wm*64..+64 and
// channels wn*64..+64 of BOTH convs (2 x 2 x 2 tiles of 32x32 -> 128 fp32 accumulators / lane).
// D[co][pos] = sum_ci W[co][ci] * x[pos + shift][ci]  (A = weight rows, B = shifted x rows).
template <int BM>
__global__ void __launch_bounds__(512) conv_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ wpn, const bf16_t* __restrict__ wpw,
    const float* __restrict__ bn, const float* __restrict__ bw, const float* __restrict__ gb,
    bf16_t* __restrict__ pre_n, bf16_t* __restrict__ pre_w, bf16_t* __restrict__ s1,
    float* __restrict__ stats, int L, int KS, int dil) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = (L + BM - 1) / BM;
  const int b = blockIdx.x / T, t = blockIdx.x - (blockIdx.x / T) * T;
  const int pos0 = t * BM;
  const int half = KS >> 1;
  const int halo = half * dil;
  const int XR = BM + 2 * halo;
  unsigned char* xs = smem;
  unsigned char* wb = smem + XR * 256;
  float* bsm = reinterpret_cast<float*>(wb + 65536);      // bn | bw | gb[b]  (3 x 128 fp32)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  constexpr int WM = BM / 64, WN = 8 / WM, CT = 4 / WN;   // BM=256: 4x2 waves, BM=128: 2x4 waves
  const int wm = w / WN, wn = w % WN;
  const bf16_t* xsmp = x + (size_t)b * L * CH;
  if (tid < 3 * CH) bsm[tid] = tid < CH ? bn[tid] : tid < 2 * CH ? bw[tid - CH] : gb[(size_t)b * CH + tid - 2 * CH];

  stage_chunks(
      XR * 16,
      [&](int idx) {
        const int pos = pos0 - halo + (idx >> 4);
        return (pos >= 0 && pos < L) ? *reinterpret_cast<const uint4*>(xsmp + (size_t)pos * CH + (idx & 15) * 8)
                                     : make_uint4(0u, 0u, 0u, 0u);
      },
      [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(xs + swz256(idx >> 4, idx & 15)) = v; });

  f32x16_t an[CT][2], aw[CT][2];
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) { an[i][j] = zero16(); aw[i][j] = zero16(); }

  const int NS = 2 * KS;
  // weight staging for step s = (tap s>>1, input-channel half s&1): 2 convs x 128 rows x 128 B.
  // thread -> 4 chunks; register staging written after the step's MFMAs (one barrier per step).
  int wsrc[4], wdst[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + 512 * i;
    const int cv = id >> 10, row = (id >> 3) & 127, ch = id & 7;
    wsrc[i] = cv * (1 << 30) + row * CH + ch * 8;
    wdst[i] = cv * 16384 + swz128(row, ch);
  }
  auto wptr = [&](int i, int s) -> const uint4* {
    const bf16_t* base = (wsrc[i] >= (1 << 30)) ? wpw : wpn;
    const int off = wsrc[i] & ((1 << 30) - 1);
    return reinterpret_cast<const uint4*>(base + (size_t)(s >> 1) * CH * CH + (s & 1) * 64 + off);
  };
  uint4 w0 = *wptr(0, 0), w1 = *wptr(1, 0), w2 = *wptr(2, 0), w3 = *wptr(3, 0);
  *reinterpret_cast<uint4*>(wb + wdst[0]) = w0;
  *reinterpret_cast<uint4*>(wb + wdst[1]) = w1;
  *reinterpret_cast<uint4*>(wb + wdst[2]) = w2;
  *reinterpret_cast<uint4*>(wb + wdst[3]) = w3;
  __syncthreads();
  for (int s = 0; s < NS; ++s) {
    const int sn = s + 1 < NS ? s + 1 : s;
    w0 = *wptr(0, sn); w1 = *wptr(1, sn); w2 = *wptr(2, sn); w3 = *wptr(3, sn);
    const int k = s >> 1, hh = s & 1;
    const int shn = k - half, shw = (k - half) * dil;
    const unsigned char* wbn = wb + (s & 1) * 32768;
    const unsigned char* wbw = wbn + 16384;
    const int rbase = halo + wm * 64 + r;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kc = hh * 8 + kk * 2 + h;
      bf16x8 fan[CT], faw[CT], fbn[2], fbw[2];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int off = swz128(wn * CT * 32 + ct * 32 + r, kk * 2 + h);
        fan[ct] = lds_frag(wbn, off);
        faw[ct] = lds_frag(wbw, off);
      }
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        fbn[pt] = lds_frag(xs, swz256(rbase + pt * 32 + shn, kc));
        fbw[pt] = lds_frag(xs, swz256(rbase + pt * 32 + shw, kc));
      }
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          an[ct][pt] = mfma32(fan[ct], fbn[pt], an[ct][pt]);
          aw[ct][pt] = mfma32(faw[ct], fbw[pt], aw[ct][pt]);
        }
    }
    if (s + 1 < NS) {
      unsigned char* dst = wb + ((s + 1) & 1) * 32768;
      *reinterpret_cast<uint4*>(dst + wdst[0]) = w0;
      *reinterpret_cast<uint4*>(dst + wdst[1]) = w1;
      *reinterpret_cast<uint4*>(dst + wdst[2]) = w2;
      *reinterpret_cast<uint4*>(dst + wdst[3]) = w3;
    }
    __syncthreads();
  }

  // ---- epilogue: bias, GELU x2, residual, broadcast, LN partials --------------------------------
  // Outputs are staged through the (now free) weight buffer as a swizzled [BM][128] bf16 tile and
  // written with 16-B-per-lane row-contiguous stores; biases / broadcast vector come from LDS.
  const int vrows = min(BM, L - pos0);
  unsigned char* ot = wb;                       // BM x 256 B output staging tile
  auto copy_out = [&](bf16_t* __restrict__ dst) {
    __syncthreads();                            // tile complete
    for (int idx = tid; idx < BM * 16; idx += 512) {
      const int row = idx >> 4, c = idx & 15;
      if (row < vrows)
        *reinterpret_cast<uint4*>(dst + ((size_t)b * L + pos0 + row) * CH + c * 8) =
            *reinterpret_cast<const uint4*>(ot + swz256(row, c));
    }
    __syncthreads();                            // tile drained before it is rewritten
  };
  // pre_n, pre_w = accumulators + bias (bf16)
#pragma unroll
  for (int cv = 0; cv < 2; ++cv) {
    const float* bias = bsm + cv * CH;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int ch0 = wn * CT * 32 + ct * 32 + 8 * g + 4 * h;
          const int p = wm * 64 + pt * 32 + r;
          const float4 bv = *reinterpret_cast<const float4*>(bias + ch0);
          const float ba[4] = {bv.x, bv.y, bv.z, bv.w};
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (cv == 0 ? an : aw)[ct][pt][4 * g + e] + ba[e];
          *reinterpret_cast<uint2*>(ot + swz256e(p, ch0)) = packq4(v);
        }
    copy_out(cv == 0 ? pre_n : pre_w);
  }
  // s1 = x + GELU(pre_n) + GELU(pre_w) + gb  (kept in an[] for the LN partials)
  float lsum = 0.f;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int ch0 = wn * CT * 32 + ct * 32 + 8 * g + 4 * h;
        const int p = wm * 64 + pt * 32 + r;
        const bool ok = p < vrows;
        float xv[4], o[4];
        unpack4(*reinterpret_cast<const uint2*>(xs + swz256e(halo + p, ch0)), xv);
        const float4 bnv = *reinterpret_cast<const float4*>(bsm + ch0);
        const float4 bwv = *reinterpret_cast<const float4*>(bsm + CH + ch0);
        const float4 gbv = *reinterpret_cast<const float4*>(bsm + 2 * CH + ch0);
        const float bna[4] = {bnv.x, bnv.y, bnv.z, bnv.w};
        const float bwa[4] = {bwv.x, bwv.y, bwv.z, bwv.w};
        const float gba[4] = {gbv.x, gbv.y, gbv.z, gbv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          o[e] = bfround(xv[e] + gelu_f(an[ct][pt][4 * g + e] + bna[e]) + gelu_f(aw[ct][pt][4 * g + e] + bwa[e]) +
                         gba[e]);
        *reinterpret_cast<uint2*>(ot + swz256e(p, ch0)) = packq4(o);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          an[ct][pt][4 * g + e] = ok ? o[e] : 0.f;
          lsum += ok ? o[e] : 0.f;
        }
      }
  copy_out(s1);
  // LN partial (mean, M2) of the tile: per-lane -> wave (Chan merge) -> 8 wave partials in LDS
  float n = 0.f, m = 0.f, M2 = 0.f;
  {
    int cnt = 0;
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) cnt += (wm * 64 + pt * 32 + r) < vrows ? CT * 16 : 0;
    n = (float)cnt;
    m = cnt > 0 ? lsum / n : 0.f;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        const bool ok = (wm * 64 + pt * 32 + r) < vrows;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float d = an[ct][pt][i] - m;
          M2 += ok ? d * d : 0.f;
        }
      }
  }
  wave_chan(n, m, M2);
  float* scratch = reinterpret_cast<float*>(wb);
  if (lane == 0) { scratch[3 * w] = n; scratch[3 * w + 1] = m; scratch[3 * w + 2] = M2; }
  __syncthreads();
  if (tid == 0) {
    float tn = 0.f, tm = 0.f, tM2 = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) chan_merge(tn, tm, tM2, scratch[3 * i], scratch[3 * i + 1], scratch[3 * i + 2]);
    stats[((size_t)b * T + t) * 2] = tm;
    stats[((size_t)b * T + t) * 2 + 1] = tM2;
  }
}

// ------------------------------------------------------------------------------------------------
// data gradient: D[ci][pos] = sum_taps sum_co WT[tap][ci][co] * dpre[pos - shift][co], both convs
// accumulated into one set of 2x2 tiles per wave (wm: 64 positions, wn: 64 input channels).
template <int BM>
__global__ void __launch_bounds__(512) conv_dgrad_kernel(
    const bf16_t* __restrict__ ds1, const bf16_t* __restrict__ pre_n, const bf16_t* __restrict__ pre_w,
    const bf16_t* __restrict__ wtn, const bf16_t* __restrict__ wtw, bf16_t* __restrict__ dx,
    bf16_t* __restrict__ dpre_n, bf16_t* __restrict__ dpre_w, int L, int KS, int dil) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int T = (L + BM - 1) / BM;
  const int b = blockIdx.x / T, t = blockIdx.x - (blockIdx.x / T) * T;
  const int pos0 = t * BM;
  const int half = KS >> 1;
  const int XR = BM + 2 * half * dil;
  unsigned char* as = smem;
  unsigned char* wb = smem + XR * 256;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  constexpr int WM = BM / 64, WN = 8 / WM, CT = 4 / WN;
  const int wm = w / WN, wn = w % WN;
  const size_t sbase = (size_t)b * L * CH;

  f32x16_t acc[CT][2];
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  for (int phase = 0; phase < 2; ++phase) {
    const int d = phase ? dil : 1;
    const int halo = half * d;
    const bf16_t* pre = phase ? pre_w : pre_n;
    bf16_t* dpo = phase ? dpre_w : dpre_n;
    const bf16_t* wt = phase ? wtw : wtn;
    // weight staging for tap k: 128 rows (ci) x 256 B (co); thread -> 4 chunks
    auto wptr = [&](int i, int k) -> const uint4* {
      const int id = tid + 512 * i;
      return reinterpret_cast<const uint4*>(wt + ((size_t)(k * CH + (id >> 4)) * CH + (id & 15) * 8));
    };
    auto wdst = [&](int i) -> int {
      const int id = tid + 512 * i;
      return swz256(id >> 4, id & 15);
    };
    uint4 w0 = *wptr(0, 0), w1 = *wptr(1, 0), w2 = *wptr(2, 0), w3 = *wptr(3, 0);
    // stage dpre = dS1 * GELU'(pre) with halo; central rows also go to global for the wgrad
    const int AR = BM + 2 * halo;
    const int nch = AR * 16;
    for (int base = tid; base < nch; base += 4 * 512) {   // 4 chunk pairs in flight per thread
      uint4 gq[4], pq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = base + i * 512;
        const int pos = pos0 - halo + (idx >> 4);
        const bool ok = idx < nch && pos >= 0 && pos < L;
        const size_t off = sbase + (size_t)pos * CH + (idx & 15) * 8;
        gq[i] = ok ? *reinterpret_cast<const uint4*>(ds1 + off) : make_uint4(0u, 0u, 0u, 0u);
        pq[i] = ok ? *reinterpret_cast<const uint4*>(pre + off) : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = base + i * 512;
        if (idx >= nch) break;
        const int j = idx >> 4, ch = idx & 15;
        const int pos = pos0 - halo + j;
        float g[8], pv[8], o[8];
        unpack8(gq[i], g);
        unpack8(pq[i], pv);
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 d = gelu_grad2((f32x2){pv[e], pv[e + 1]}) * (f32x2){g[e], g[e + 1]};
          o[e] = d.x;
          o[e + 1] = d.y;
        }
        const uint4 v = (pos >= 0 && pos < L) ? packq8(o) : make_uint4(0u, 0u, 0u, 0u);
        if (pos >= 0 && pos < L && j >= halo && j < halo + BM)
          *reinterpret_cast<uint4*>(dpo + sbase + (size_t)pos * CH + ch * 8) = v;
        *reinterpret_cast<uint4*>(as + swz256(j, ch)) = v;
      }
    }
    *reinterpret_cast<uint4*>(wb + wdst(0)) = w0;
    *reinterpret_cast<uint4*>(wb + wdst(1)) = w1;
    *reinterpret_cast<uint4*>(wb + wdst(2)) = w2;
    *reinterpret_cast<uint4*>(wb + wdst(3)) = w3;
    __syncthreads();
    for (int k = 0; k < KS; ++k) {
      const int kn = k + 1 < KS ? k + 1 : k;
      w0 = *wptr(0, kn); w1 = *wptr(1, kn); w2 = *wptr(2, kn); w3 = *wptr(3, kn);
      const int sh = (k - half) * d;
      const unsigned char* wk = wb + (k & 1) * 32768;
      const int rbase = halo + wm * 64 + r - sh;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        bf16x8 fa[CT], fb[2];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) fa[ct] = lds_frag(wk, swz256(wn * CT * 32 + ct * 32 + r, kk * 2 + h));
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) fb[pt] = lds_frag(as, swz256(rbase + pt * 32, kk * 2 + h));
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) acc[ct][pt] = mfma32(fa[ct], fb[pt], acc[ct][pt]);
      }
      if (k + 1 < KS) {
        unsigned char* dst = wb + ((k + 1) & 1) * 32768;
        *reinterpret_cast<uint4*>(dst + wdst(0)) = w0;
        *reinterpret_cast<uint4*>(dst + wdst(1)) = w1;
        *reinterpret_cast<uint4*>(dst + wdst(2)) = w2;
        *reinterpret_cast<uint4*>(dst + wdst(3)) = w3;
      }
      __syncthreads();
    }
  }

  // epilogue: dx = ds1 + D^T.  The fp32 accumulators are staged through LDS (the x / weight buffers
  // are free: [BM][128] fp32, 16-B chunks XOR-swizzled by row so the 32 rows a half-wave writes hit
  // distinct banks), then combined with row-contiguous 16-B loads of ds1 and 16-B stores of dx.
  const int vrows = min(BM, L - pos0);
  float* ft = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      const int p = wm * 64 + pt * 32 + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c4 = (wn * CT * 32 + ct * 32 + 8 * g + 4 * h) >> 2;
        *reinterpret_cast<float4*>(ft + p * CH + ((c4 ^ (p & 31)) << 2)) =
            make_float4(acc[ct][pt][4 * g], acc[ct][pt][4 * g + 1], acc[ct][pt][4 * g + 2], acc[ct][pt][4 * g + 3]);
      }
    }
  __syncthreads();
  for (int idx = tid; idx < BM * 16; idx += 512) {
    const int row = idx >> 4, c = idx & 15;
    if (row >= vrows) continue;
    const size_t off = sbase + (size_t)(pos0 + row) * CH + c * 8;
    float gv[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(ds1 + off), gv);
    const float4 f0 = *reinterpret_cast<const float4*>(ft + row * CH + (((2 * c) ^ (row & 31)) << 2));
    const float4 f1 = *reinterpret_cast<const float4*>(ft + row * CH + (((2 * c + 1) ^ (row & 31)) << 2));
    const float fa[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = gv[e] + fa[e];
    *reinterpret_cast<uint4*>(dx + off) = packq8(o);
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient. 1-D grid of nconv * 4 output-channel groups ("types") x R position chunks, 256
// threads.  Wave w owns input channels w*32..+32 for all KS taps (KS tiles of 32x32 -> 16*KS
// accumulators).  D[co][ci] += sum_pos dy[pos][co] * x[pos + shift][ci]  (A, B via transposed LDS
// reads).  XCD-aware mapping: workgroups are dealt to the 8 XCDs round-robin by id, so the types of
// one chunk (which all stage the same x rows) get ids congruent mod 8 and share one XCD's L2
// instead of fetching those rows from HBM once per XCD.
template <int KS, int BM>
__global__ void __launch_bounds__(256) wgrad_kernel(const bf16_t* __restrict__ dy0, const bf16_t* __restrict__ dy1,
                                                    const bf16_t* __restrict__ x, float* __restrict__ slab,
                                                    float* __restrict__ bslab, int B, int L, int dil1, int nconv,
                                                    int R) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ntypes = nconv * 4;
  int type, chunk;
  if ((R & 7) == 0) {
    const int id = blockIdx.x, j = id >> 3;
    chunk = (j / ntypes) * 8 + (id & 7);
    type = j - (j / ntypes) * ntypes;
  } else {
    chunk = blockIdx.x / ntypes;
    type = blockIdx.x - chunk * ntypes;
  }
  const int cv = type >> 2, cg = type & 3;
  const bf16_t* dy = cv ? dy1 : dy0;
  const int d = cv ? dil1 : 1;
  const int half = KS >> 1;
  const int halo = half * d;
  const int halo_max = half * (nconv > 1 ? max(dil1, 1) : 1);
  unsigned char* dys = smem;                  // BM rows x 64 B (32 output channels), unswizzled
  unsigned char* xs = smem + BM * 64;         // (BM + 2 halo_max) rows x 256 B, swz256
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int T = (L + BM - 1) / BM;
  const long NT = (long)B * T;
  const long t0 = NT * chunk / R, t1 = NT * (chunk + 1) / R;

  f32x16_t acc[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) acc[k] = zero16();
  float bsum = 0.f;

  for (long tile = t0; tile < t1; ++tile) {
    const int b = (int)(tile / T), t = (int)(tile - (long)(tile / T) * T);
    const int pos0 = t * BM;
    const size_t sbase = (size_t)b * L * CH;
    __syncthreads();
    const int XR = BM + 2 * halo;
    // one batched pass: chunks [0, BM*4) are the dy tile (64-B rows), the rest the x tile (with halo)
    stage_chunks(
        BM * 4 + XR * 16,
        [&](int idx) {
          if (idx < BM * 4) {
            const int pos = pos0 + (idx >> 2);
            return pos < L ? *reinterpret_cast<const uint4*>(dy + sbase + (size_t)pos * CH + cg * 32 + (idx & 3) * 8)
                           : make_uint4(0u, 0u, 0u, 0u);
          }
          const int i2 = idx - BM * 4;
          const int pos = pos0 - halo + (i2 >> 4);
          return (pos >= 0 && pos < L) ? *reinterpret_cast<const uint4*>(x + sbase + (size_t)pos * CH + (i2 & 15) * 8)
                                       : make_uint4(0u, 0u, 0u, 0u);
        },
        [&](int idx, uint4 v) {
          // one store site with a 16-B-aligned offset (two sites compile to 4 x ds_write_b32)
          const int i2 = idx - BM * 4;
          const int off = idx < BM * 4 ? (idx >> 2) * 64 + (idx & 3) * 16 : BM * 64 + swz256(i2 >> 4, i2 & 15);
          *reinterpret_cast<uint4*>(__builtin_assume_aligned(smem + off, 16)) = v;
        });
    __syncthreads();
#pragma unroll 2
    for (int kk = 0; kk < BM / 16; ++kk) {
      const int ra = kk * 16 + 8 * h + q;
      const bf16x8 fa = cat_tr(lds_tr(dys, ra * 64 + tc * 2), lds_tr(dys, (ra + 4) * 64 + tc * 2));
      if (w == 0) {
        typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
        const u16x8 u = __builtin_bit_cast(u16x8, fa);
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum += bf2f(u[e]);
      }
      const int colb = w * 32 + tc;
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int rb = halo + ra + (k - half) * d;
        const bf16x8 fb = cat_tr(lds_tr(xs, swz256e(rb, colb)), lds_tr(xs, swz256e(rb + 4, colb)));
        acc[k] = mfma32(fa, fb, acc[k]);
      }
    }
  }
  (void)halo_max;
  // slab in the torch weight layout [co][ci][KS] so the reduction streams it with 16-B accesses
  float* dst = slab + ((size_t)chunk * nconv + cv) * KS * CH * CH + (size_t)(w * 32 + r) * KS;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int co = cg * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
#pragma unroll
    for (int k = 0; k < KS; ++k) dst[(size_t)co * CH * KS + k] = acc[k][i];
  }
  if (w == 0) {
    bsum += __shfl_xor(bsum, 32, 64);
    if (h == 0) bslab[((size_t)chunk * nconv + cv) * CH + cg * 32 + r] = bsum;
  }
}

// sum the R slabs (fixed order: deterministic) and ADD the result into the torch layouts:
// weight [co][ci][KS] (KS == 1: [co][ci]) -- the slabs already use it, so both sides stream with
// 16-B accesses -- and bias [co]; the destinations are the flat-arena .grad views (or zero-initialised
// tensors); one thread owns each destination element (no atomics).
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float4* __restrict__ slab,
                                                           const float* __restrict__ bslab, float* __restrict__ dw0,
                                                           float* __restrict__ dw1, float* __restrict__ db0,
                                                           float* __restrict__ db1, int R, int nconv, int KS) {
  const int per4 = KS * CH * CH / 4;
  const int total4 = nconv * per4;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < total4) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int rr = 0;
    for (; rr + 4 <= R; rr += 4) {
      const float4 a = slab[(size_t)rr * total4 + idx], b = slab[(size_t)(rr + 1) * total4 + idx];
      const float4 c = slab[(size_t)(rr + 2) * total4 + idx], d = slab[(size_t)(rr + 3) * total4 + idx];
      s.x += (a.x + b.x) + (c.x + d.x); s.y += (a.y + b.y) + (c.y + d.y);
      s.z += (a.z + b.z) + (c.z + d.z); s.w += (a.w + b.w) + (c.w + d.w);
    }
    for (; rr < R; ++rr) {
      const float4 a = slab[(size_t)rr * total4 + idx];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
    const int cv = idx >= per4;
    float4* dw = reinterpret_cast<float4*>(cv ? dw1 : dw0) + (idx - cv * per4);
    float4 o = *dw;
    o.x += s.x; o.y += s.y; o.z += s.z; o.w += s.w;
    *dw = o;
  }
  if (idx < nconv * CH) {
    float s = 0.f;
    for (int rr = 0; rr < R; ++rr) s += bslab[(size_t)rr * nconv * CH + idx];
    float* db = idx >= CH ? db1 : db0;
    if (db != nullptr) db[idx % CH] += s;
  }
}

// torch conv weight [co][ci][KS] fp32 -> WP[KS][co][ci] and WT[KS][ci][co] bf16
__global__ void __launch_bounds__(256) pack_conv_kernel(const float* __restrict__ w, bf16_t* __restrict__ wp,
                                                        bf16_t* __restrict__ wt, int KS) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= KS * CH * CH) return;
  const int k = idx / (CH * CH), co = (idx / CH) % CH, ci = idx % CH;
  const bf16_t v = f2bf(w[((size_t)co * CH + ci) * KS + k]);
  wp[((size_t)k * CH + co) * CH + ci] = v;
  wt[((size_t)k * CH + ci) * CH + co] = v;
}

template <int BM>
int launch_fwd(const void* x, const void* wpn, const void* wpw, const float* bn, const float* bw,
               const float* gb, void* pre_n, void* pre_w, void* s1, float* stats, int B, int L, int KS, int dil,
               hipStream_t st) {
  const int T = (L + BM - 1) / BM;
  const int lds = (BM + 2 * (KS / 2) * dil) * 256 + 65536 + 3 * CH * 4;
  if (lds > 163840) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(conv_fwd_kernel<BM>, dim3(B * T), dim3(512), lds, st, (const bf16_t*)x, (const bf16_t*)wpn,
                     (const bf16_t*)wpw, bn, bw, gb, (bf16_t*)pre_n, (bf16_t*)pre_w, (bf16_t*)s1, stats, L, KS, dil);
  return pbx_launch_status();
}

template <int BM>
int launch_dgrad(const void* ds1, const void* pre_n, const void* pre_w, const void* wtn, const void* wtw, void* dx,
                 void* dpre_n, void* dpre_w, int B, int L, int KS, int dil, hipStream_t st) {
  const int T = (L + BM - 1) / BM;
  const int lds = (BM + 2 * (KS / 2) * dil) * 256 + 65536;
  if (lds > 163840) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(conv_dgrad_kernel<BM>, dim3(B * T), dim3(512), lds, st, (const bf16_t*)ds1,
                     (const bf16_t*)pre_n, (const bf16_t*)pre_w, (const bf16_t*)wtn, (const bf16_t*)wtw,
                     (bf16_t*)dx, (bf16_t*)dpre_n, (bf16_t*)dpre_w, L, KS, dil);
  return pbx_launch_status();
}
}  // namespace

static bool conv_attrs_set = false;
static void set_conv_attrs() {
  if (conv_attrs_set) return;
  (void)hipFuncSetAttribute((const void*)conv_fwd_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)conv_fwd_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)conv_dgrad_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)conv_dgrad_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)wgrad_kernel<9, 128>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)wgrad_kernel<1, 128>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  conv_attrs_set = true;
}

PBX_EXPORT int pbx_conv_fwd(const void* x, const void* wpn, const void* wpw, const float* bn, const float* bw,
                            const float* gb, void* pre_n, void* pre_w, void* s1, float* stats, int B, int L, int KS,
                            int dil, int BM, hipStream_t st) {
  set_conv_attrs();
  if (BM == 256) return launch_fwd<256>(x, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, stats, B, L, KS, dil, st);
  if (BM == 128) return launch_fwd<128>(x, wpn, wpw, bn, bw, gb, pre_n, pre_w, s1, stats, B, L, KS, dil, st);
  return (int)hipErrorInvalidValue;
}

PBX_EXPORT int pbx_conv_dgrad(const void* ds1, const void* pre_n, const void* pre_w, const void* wtn,
                              const void* wtw, void* dx, void* dpre_n, void* dpre_w, int B, int L, int KS, int dil,
                              int BM, hipStream_t st) {
  set_conv_attrs();
  if (BM == 256) return launch_dgrad<256>(ds1, pre_n, pre_w, wtn, wtw, dx, dpre_n, dpre_w, B, L, KS, dil, st);
  if (BM == 128) return launch_dgrad<128>(ds1, pre_n, pre_w, wtn, wtw, dx, dpre_n, dpre_w, B, L, KS, dil, st);
  return (int)hipErrorInvalidValue;
}

// slab: R * nconv * KS * 128 * 128 floats; bslab: R * nconv * 128 floats
PBX_EXPORT int pbx_wgrad(const void* dy0, const void* dy1, const void* x, float* slab, float* bslab, float* dw0,
                         float* dw1, float* db0, float* db1, int B, int L, int KS, int dil1, int nconv, int R,
                         int accumulate, hipStream_t st) {
  set_conv_attrs();
  constexpr int BM = 128;
  const int halo = (KS / 2) * (nconv > 1 ? dil1 : 1);
  const int lds = BM * 64 + (BM + 2 * halo) * 256;
  if (lds > 163840 || nconv < 1 || nconv > 2) return (int)hipErrorInvalidValue;
  dim3 grid(nconv * 4 * R);
  if (KS == 9)
    hipLaunchKernelGGL((wgrad_kernel<9, BM>), grid, dim3(256), lds, st, (const bf16_t*)dy0, (const bf16_t*)dy1,
                       (const bf16_t*)x, slab, bslab, B, L, dil1, nconv, R);
  else if (KS == 1)
    hipLaunchKernelGGL((wgrad_kernel<1, BM>), grid, dim3(256), lds, st, (const bf16_t*)dy0, (const bf16_t*)dy1,
                       (const bf16_t*)x, slab, bslab, B, L, dil1, nconv, R);
  else
    return (int)hipErrorInvalidValue;
  (void)accumulate;   // destinations are always accumulated into (zero-initialised when not arena views)
  const int total4 = nconv * KS * CH * CH / 4;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total4 + 255) / 256), dim3(256), 0, st, (const float4*)slab,
                     bslab, dw0, dw1, db0, db1, R, nconv, KS);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_pack_conv(const float* w, void* wp, void* wt, int KS, hipStream_t st) {
  const int n = KS * CH * CH;
  hipLaunchKernelGGL(pack_conv_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w, (bf16_t*)wp, (bf16_t*)wt, KS);
  return pbx_launch_status();
}
