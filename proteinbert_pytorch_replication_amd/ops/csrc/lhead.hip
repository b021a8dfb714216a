// Local (amino-acid) pretraining head + its loss, reference semantics, as coalesced multi-pass kernels
// (SURVEY K9/K10).
//
// Reference: ProteinBERT/modules.py:277-284,304 (Linear C -> V, then nn.Softmax() with the implicit
// dim, which for the [B, L, V] output is dim 0: a softmax over the BATCH for every (position, token))
// and ProteinBERT/utils.py:293 (CrossEntropyLoss over V applied to those probabilities, times the
// per-residue weight, mean over B * L):
//   Z[b,l,v]  = h[b,l,:] . Wo[v,:] + bo[v]
//   P[b,l,v]  = exp(Z - M[l,v]) / S[l,v],       M = max_b Z, S = sum_b exp(Z - M)
//   loss      = 1/(BL) sum_{b,l} w[b,l] (log sum_v exp(P[b,l,v]) - P[b,l,y])
//   G[b,l,v]  = w/(BL) (exp(P)/se - [v == y])                      (dloss/dP)
//   dZ        = P (G - T[l,v]),  T[l,v] = sum_b G P                 (softmax-over-batch backward)
//   dh = dZ Wo ;  dWo = dZ^T h ;  dbo = sum dZ
//
// The batch coupling needs two statistics per (l, v) over all B samples before any gradient exists,
// so the head runs as passes over row tiles of 16 samples x 32 positions (each sample's 32 rows are one
// contiguous 8 KB run of h): (1) logits + per-tile (max, sum exp) partials, (2) fold them to (M, 1/S),
// (3) CE loss + per-tile partials of G P, (4) fold them to T, (5) dZ, dh = dZ Wo (MFMA) and dZ rows for
// the dWo GEMM.  A workgroup per POSITION walking all B samples (the round-2 form) read rows L * 256
// bytes apart and ran at ~150 us for B = L = 512; every pass here streams contiguous rows.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int SB = 16;     // samples per tile
constexpr int PT = 32;     // positions per tile
constexpr int VP = 32;     // padded vocabulary

// Wo (fp32 [V][128]) -> bf16 LDS tile [32][128] (swz256, rows >= V zero); bias into bo_s[32]
__device__ __forceinline__ void stage_wo(unsigned char* wos, float* bo_s, const float* __restrict__ wo,
                                        const float* __restrict__ bo, int V) {
  for (int idx = threadIdx.x; idx < VP * 16; idx += blockDim.x) {
    const int v = idx >> 4, c8 = idx & 15;
    float e[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (v < V) {
      const float4 a = *reinterpret_cast<const float4*>(wo + v * CH + c8 * 8);
      const float4 b = *reinterpret_cast<const float4*>(wo + v * CH + c8 * 8 + 4);
      e[0] = a.x; e[1] = a.y; e[2] = a.z; e[3] = a.w; e[4] = b.x; e[5] = b.y; e[6] = b.z; e[7] = b.w;
    }
    *reinterpret_cast<uint4*>(wos + swz256(v, c8)) = packq8(e);
  }
  if (threadIdx.x < VP) bo_s[threadIdx.x] = threadIdx.x < V ? bo[threadIdx.x] : 0.f;
}

// tile id -> (first sample, first position); tiles ordered position-tile-major within a sample chunk
__device__ __forceinline__ void tile_of(int L, int& b0, int& p0, int& chunk) {
  const int TP = (L + PT - 1) / PT;
  chunk = blockIdx.x / TP;
  b0 = chunk * SB;
  p0 = (blockIdx.x - chunk * TP) * PT;
}

// ---- pass 1: Z = h Wo^T + bo (fp32, [B*L][32]) and per-tile (max, sum exp) over the tile's samples
__global__ void __launch_bounds__(512) lhead_logits_kernel(const bf16_t* __restrict__ h, const float* __restrict__ wo,
                                                           const float* __restrict__ bo, float* __restrict__ Z,
                                                           float2* __restrict__ part, int B, int L, int V) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* wos = smem;                                              // [32][128] bf16
  float* bo_s = reinterpret_cast<float*>(smem + VP * 256);                // [32]
  float (*zt)[PT][VP + 1] = reinterpret_cast<float (*)[PT][VP + 1]>(bo_s + VP);   // [SB][PT][VP + 1]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  int b0, p0, chunk;
  tile_of(L, b0, p0, chunk);
  stage_wo(wos, bo_s, wo, bo, V);
  __syncthreads();
  bf16x8 wf[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) wf[kk] = lds_frag(wos, swz256(r, kk * 2 + hh));
  const float bv = bo_s[r];
#pragma unroll
  for (int si = 0; si < 2; ++si) {
    const int sl = 2 * w + si, b = b0 + sl;
    const int pos = p0 + r;
    const bool okrow = b < B && pos < L;
    const size_t row = (size_t)min(b, B - 1) * L + min(pos, L - 1);        // clamped: loads in bounds
    bf16x8 hf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) hf[kk] = *reinterpret_cast<const bf16x8*>(h + row * CH + kk * 16 + 8 * hh);
    f32x16_t acc = zero16();
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) acc = mfma32(hf[kk], wf[kk], acc);
    // D[pos][v]: lane column v = r, rows (e & 3) + 8 (e >> 2) + 4 hh
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int pl = (e & 3) + 8 * (e >> 2) + 4 * hh;
      const int pp = p0 + pl;
      const float z = acc[e] + bv;
      zt[sl][pl][r] = z;
      if (b < B && pp < L) Z[((size_t)b * L + pp) * VP + r] = r < V ? z : 0.f;
    }
    (void)okrow;
  }
  __syncthreads();
  // (max, sum exp) over the tile's valid samples for each (position, v): thread -> (pl, v pair)
  {
    const int pl = tid >> 4, v0 = (tid & 15) * 2;
    const int pp = p0 + pl;
    const int nb = min(SB, B - b0);
    if (pp < L) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int v = v0 + j;
        float m = -3.0e38f;
        for (int s = 0; s < nb; ++s) m = fmaxf(m, zt[s][pl][v]);
        float se = 0.f;
        for (int s = 0; s < nb; ++s) se += __expf(zt[s][pl][v] - m);
        part[((size_t)chunk * L + pp) * VP + v] = make_float2(m, se);
      }
    }
  }
}

// ---- passes 2 / 4: fold the per-chunk partials of every (l, v)
//  mode 0: (max, sum exp) -> (M, 1/S);  mode 1: sum G P -> T (stored in .x)
// 64 (l, v) entries per workgroup, the chunks split over 4 thread groups (one pass with an online
// max / rescaled-sum merge, 4x the loads in flight of a thread walking all chunks twice), the four
// partials combined in a fixed order
__global__ void __launch_bounds__(256) lhead_fold_kernel(const float2* __restrict__ part, int nchunks, int L,
                                                         float2* __restrict__ out, int mode) {
  __shared__ float2 red[4][64];
  const int il = threadIdx.x & 63, cg = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + il;                 // l * 32 + v
  const bool ok = i < L * VP;
  float m = -3.0e38f, sum = 0.f;
  if (ok) {
    for (int c = cg; c < nchunks; c += 4) {
      const float2 p = part[(size_t)c * L * VP + i];
      if (mode != 1) {
        const float mn = fmaxf(m, p.x);
        sum = sum * __expf(m - mn) + p.y * __expf(p.x - mn);
        m = mn;
      } else {
        sum += p.x;
      }
    }
  }
  red[cg][il] = make_float2(m, sum);
  __syncthreads();
  if (cg != 0 || !ok) return;
  if (mode != 1) {
    float mm = red[0][il].x;
#pragma unroll
    for (int k = 1; k < 4; ++k) mm = fmaxf(mm, red[k][il].x);
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) ss += red[k][il].y * __expf(red[k][il].x - mm);
    out[i] = make_float2(mm, mode == 2 ? ss : ss > 0.f ? 1.0f / ss : 0.f);   // mode 2: raw (M, S)
  } else {
    out[i] = make_float2(red[0][il].y + red[1][il].y + red[2][il].y + red[3][il].y, 0.f);
  }
}

// Per-lane row math shared by passes 3 and 5: lane (r, hh) owns row (b, pos) and the 16 tokens
// v = 8 hh + j (j < 8) and 16 + 8 hh + j; the two lanes of a row (hh = 0, 1) exchange their halves
// of sum_v exp(P).  Returns P, G for the 16 tokens and the row's CE term (on hh = 0; 0 elsewhere).
struct RowTerms {
  float P[16], G[16];
  float loss;
};
__device__ __forceinline__ RowTerms row_terms(const float* __restrict__ Z, const float2* ms, size_t row, int pl,
                                              int hh, int V, bool ok, int yv, float coef) {
  RowTerms t;
  float zv[16];
  {
    const float4* zp0 = reinterpret_cast<const float4*>(Z + row * VP + 8 * hh);
    const float4* zp1 = reinterpret_cast<const float4*>(Z + row * VP + 16 + 8 * hh);
    const float4 a = zp0[0], b = zp0[1], c = zp1[0], d = zp1[1];
    const float tmp[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
#pragma unroll
    for (int j = 0; j < 16; ++j) zv[j] = tmp[j];
  }
  float e[16], se = 0.f, py = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int v = (j < 8 ? 0 : 16) + 8 * hh + (j & 7);
    const float2 s = ms[pl * VP + v];
    const bool inv = v < V;
    t.P[j] = inv ? __expf(zv[j] - s.x) * s.y : 0.f;
    e[j] = inv ? __expf(t.P[j]) : 0.f;
    se += e[j];
    py += v == yv ? t.P[j] : 0.f;
  }
  se += __shfl_xor(se, 32, 64);
  const float rse = 1.0f / se;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int v = (j < 8 ? 0 : 16) + 8 * hh + (j & 7);
    t.G[j] = ok ? coef * (e[j] * rse - (v == yv ? 1.f : 0.f)) : 0.f;
  }
  // this lane's share of w (log se - P[y]) (the coefficient w / (B L) is applied by the caller)
  t.loss = ok ? ((hh == 0 ? __logf(se) : 0.f) - py) : 0.f;
  return t;
}

// ---- pass 3: CE loss and per-tile partials of T = sum_b G P
__global__ void __launch_bounds__(512) lhead_ce_kernel(const float* __restrict__ Z, const float2* __restrict__ MS,
                                                       const long long* __restrict__ y, const float* __restrict__ wl,
                                                       float2* __restrict__ tpart, float* __restrict__ loss_part,
                                                       int B, int L, int V, float inv_bl) {
  __shared__ float2 ms[PT * VP];
  __shared__ float gp[8][PT][VP + 1];           // per wave: sum over its 2 samples
  __shared__ float red[8];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  int b0, p0, chunk;
  tile_of(L, b0, p0, chunk);
  for (int i = tid; i < PT * VP; i += 512) {
    const int pp = min(p0 + i / VP, L - 1);
    ms[i] = MS[(size_t)pp * VP + (i % VP)];
  }
  __syncthreads();
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  float lsum = 0.f;
#pragma unroll
  for (int si = 0; si < 2; ++si) {
    const int b = b0 + 2 * w + si, pos = p0 + r;
    const bool ok = b < B && pos < L;
    const size_t row = (size_t)min(b, B - 1) * L + min(pos, L - 1);
    const int yv = (int)y[row];
    const float wgt = ok ? wl[row] : 0.f;
    const RowTerms t = row_terms(Z, ms, row, r, hh, V, ok, yv, wgt * inv_bl);
    lsum += wgt * t.loss;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] += t.G[j] * t.P[j];
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) gp[w][r][(j < 8 ? 0 : 16) + 8 * hh + (j & 7)] = acc[j];
  lsum = wave_reduce_sum(lsum);
  if (lane == 0) red[w] = lsum;
  __syncthreads();
  for (int i = tid; i < PT * VP; i += 512) {
    const int pl = i / VP, v = i % VP;
    if (p0 + pl < L) {
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) s += gp[ww][pl][v];
      tpart[((size_t)chunk * L + p0 + pl) * VP + v] = make_float2(s, 0.f);
    }
  }
  if (tid == 0) {
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) s += red[ww];
    loss_part[blockIdx.x] = s * inv_bl;
  }
}

// ---- pass 5: dZ = P (G - T), dh = dZ Wo (MFMA), dZ rows (bf16 [B*L][32]) for the dWo GEMM and the
// per-workgroup dbo partials.  Wave w: samples 2w, 2w+1 of the tile.
__global__ void __launch_bounds__(512) lhead_grad_kernel(const float* __restrict__ Z, const float2* __restrict__ MS,
                                                         const float2* __restrict__ T, const long long* __restrict__ y,
                                                         const float* __restrict__ wl, const float* __restrict__ wo,
                                                         const float* __restrict__ bo, bf16_t* __restrict__ dh,
                                                         bf16_t* __restrict__ dz, float* __restrict__ dbo_part, int B,
                                                         int L, int V, float inv_bl) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ot = smem;                                               // [8 waves][32][128] bf16: dh staging
  unsigned char* wos = smem + 8 * PT * 256;                               // [32][128] bf16
  float2* ms = reinterpret_cast<float2*>(wos + VP * 256);                 // [PT * VP]
  float* ts = reinterpret_cast<float*>(ms + PT * VP);                     // [PT * VP]
  float* bo_s = ts + PT * VP;                                             // [VP]
  float (*dbr)[VP] = reinterpret_cast<float (*)[VP]>(bo_s + VP);          // [8][VP]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  int b0, p0, chunk;
  tile_of(L, b0, p0, chunk);
  stage_wo(wos, bo_s, wo, bo, V);
  for (int i = tid; i < PT * VP; i += 512) {
    const int pp = min(p0 + i / VP, L - 1);
    ms[i] = MS[(size_t)pp * VP + (i % VP)];
    ts[i] = T[(size_t)pp * VP + (i % VP)].x;
  }
  __syncthreads();
  float dba[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) dba[j] = 0.f;
  unsigned char* myot = ot + w * PT * 256;
#pragma unroll 1
  for (int si = 0; si < 2; ++si) {
    const int b = b0 + 2 * w + si, pos = p0 + r;
    const bool ok = b < B && pos < L;
    const size_t row = (size_t)min(b, B - 1) * L + min(pos, L - 1);
    const int yv = (int)y[row];
    const float wgt = ok ? wl[row] : 0.f;
    const RowTerms t = row_terms(Z, ms, row, r, hh, V, ok, yv, wgt * inv_bl);
    float d[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int v = (j < 8 ? 0 : 16) + 8 * hh + (j & 7);
      d[j] = ok && v < V ? t.P[j] * (t.G[j] - ts[r * VP + v]) : 0.f;
      dba[j] += d[j];
    }
    const bf16x8 f0 = pack8(d), f1 = pack8(d + 8);      // k-steps 0 / 1: v = 8 hh + j, 16 + 8 hh + j
    if (ok) {
      *reinterpret_cast<bf16x8*>(dz + row * VP + 8 * hh) = f0;
      *reinterpret_cast<bf16x8*>(dz + row * VP + 16 + 8 * hh) = f1;
    }
    // dh[pos][c] = sum_v dZ[pos][v] Wo[v][c]: A = dZ rows (this lane's fragments), B = Wo tile read
    // transposed (K = v along its rows)
    f32x16_t acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = zero16();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int rlo = kk * 16 + 8 * hh + q;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int col = ct * 32 + tc;
        const bf16x8 fb = cat_tr(lds_tr(wos, swz256e(rlo, col)), lds_tr(wos, swz256e(rlo + 4, col)));
        acc[ct] = mfma32(kk == 0 ? f0 : f1, fb, acc[ct]);
      }
    }
    // stage the 32 x 128 bf16 tile (rows (e & 3) + 8 (e >> 2) + 4 hh, column ct * 32 + r), then
    // 256-B row stores
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        *reinterpret_cast<bf16_t*>(myot + swz256e((e & 3) + 8 * (e >> 2) + 4 * hh, ct * 32 + r)) = f2bf(acc[ct][e]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (b < B) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int idx = lane + 64 * i;           // 512 16-B chunks = 32 rows x 16
        const int rr = idx >> 4, c8 = idx & 15;
        if (p0 + rr < L)
          *reinterpret_cast<uint4*>(dh + ((size_t)b * L + p0 + rr) * CH + c8 * 8) =
              *reinterpret_cast<const uint4*>(myot + swz256(rr, c8));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // dbo partial: sum over the wave's rows (lanes with the same hh) then over the 8 waves
#pragma unroll
  for (int j = 0; j < 16; ++j) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) dba[j] += __shfl_xor(dba[j], o, 64);
  }
  if (r == 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) dbr[w][(j < 8 ? 0 : 16) + 8 * hh + (j & 7)] = dba[j];
  }
  __syncthreads();
  if (tid < V) {
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) s += dbr[ww][tid];
    dbo_part[(size_t)blockIdx.x * V + tid] = s;
  }
}

// ---- one-launch form (B <= 512): a workgroup owns PP = 2 positions and ALL samples, so both batch
// reductions ((max, sum exp), then T = sum_b G P) are workgroup-local and the head is one pass over h:
// (1) Z = h Wo^T + bo for the 2B rows (MFMA) into an fp32 LDS table, (2) column (max, sum exp) ->
// (M, 1/S), (3) per row P, the CE term and G P (P kept in registers), (4) column sums -> T, (5) dZ =
// P (G - T) into the table and the bf16 dz rows for the dWo GEMM, (6) dbo partial and dh = dZ Wo (MFMA,
// staged through LDS for 256-B row stores).  h is read once (512-B runs per sample), Z never leaves
// the CU.
// PP = 1 (513 <= B <= 1024): a workgroup owns ONE position; the table holds PP * B <= 1024 rows either way.
constexpr int ROWSF = 1024;       // table rows = PP * max B
constexpr int ZS = VP + 1;        // fp32 row stride of the table (column walks hit distinct banks)
constexpr int FUSED_LDS = ROWSF * ZS * 4 + VP * 256 + VP * 4 + 8 * 64 * 8 + 64 * 8 + 64 * 4 + 8 * 4;

template <int PP>
__global__ void __launch_bounds__(512) lhead_fused_kernel(const bf16_t* __restrict__ h, const float* __restrict__ wo,
                                                          const float* __restrict__ bo,
                                                          const long long* __restrict__ y,
                                                          const float* __restrict__ wl, bf16_t* __restrict__ dh,
                                                          bf16_t* __restrict__ dz, float* __restrict__ dbo_part,
                                                          float* __restrict__ loss_part, int B, int L, int V,
                                                          float inv_bl) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NPAIR = PP * 32, PARTS = 512 / NPAIR;   // (position, v) columns; sample slices per column
  float* zt = reinterpret_cast<float*>(smem);                              // [PP * B][ZS]
  unsigned char* wos = smem + ROWSF * ZS * 4;                              // [32][128] bf16
  float* bo_s = reinterpret_cast<float*>(wos + VP * 256);                  // [32]
  float2* red = reinterpret_cast<float2*>(bo_s + VP);                      // [PARTS][NPAIR]
  float2* ms = red + 8 * 64;                                               // [NPAIR] (M, 1/S) per (p, v)
  float* tt = reinterpret_cast<float*>(ms + 64);                           // [NPAIR] T per (p, v)
  float* lred = tt + 64;                                                   // [8]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int l0 = blockIdx.x * PP;
  const int NR = PP * B, NT = (NR + 31) / 32;
  stage_wo(wos, bo_s, wo, bo, V);
  __syncthreads();
  // (1) logits
  {
    bf16x8 wf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) wf[kk] = lds_frag(wos, swz256(r, kk * 2 + hh));
    const float bv = bo_s[r];
#pragma unroll 2
    for (int t = w; t < NT; t += 8) {
      const int row = min(t * 32 + r, NR - 1);
      const int p = row / B, s = row - (row / B) * B;
      const bf16_t* src = h + ((size_t)s * L + min(l0 + p, L - 1)) * CH + 8 * hh;
      bf16x8 hf[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) hf[kk] = *reinterpret_cast<const bf16x8*>(src + kk * 16);
      f32x16_t acc = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) acc = mfma32(hf[kk], wf[kk], acc);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rr = t * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
        if (rr < NR) zt[rr * ZS + r] = acc[e] + bv;
      }
    }
  }
  __syncthreads();
  const int pair = tid % NPAIR, part = tid / NPAIR;  // column (p, v) and sample slice of the reductions
  const int pp = pair >> 5, pv = pair & 31;
  // (2) (max, sum exp) over the samples of every (p, v)
  {
    float m = -3.0e38f, se = 0.f;
    for (int s = part; s < B; s += PARTS) {
      const float z = zt[(pp * B + s) * ZS + pv];
      const float mn = fmaxf(m, z);
      se = se * __expf(m - mn) + __expf(z - mn);
      m = mn;
    }
    red[part * NPAIR + pair] = make_float2(m, se);
  }
  __syncthreads();
  if (tid < NPAIR) {
    float mm = red[tid].x;
#pragma unroll
    for (int k = 1; k < PARTS; ++k) mm = fmaxf(mm, red[k * NPAIR + tid].x);
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < PARTS; ++k) ss += red[k * NPAIR + tid].y * __expf(red[k * NPAIR + tid].x - mm);
    ms[tid] = make_float2(mm, ss > 0.f ? 1.0f / ss : 0.f);
  }
  __syncthreads();
  // (3) per row: P (registers), CE term, G P into the table
  constexpr int RPT = ROWSF / 512;                  // rows per thread
  float P[RPT][VP], rse[RPT], coef[RPT];
  int yv[RPT];
  float lsum = 0.f;
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int row = tid + 512 * k;
    // rows past NR (small B) give p = row / B up to 1023 / B: clamp the ms[] index into the PP positions
    const int p = min(row / B, PP - 1), s = row - (row / B) * B;
    const bool ok = row < NR && l0 + p < L;
    const size_t gi = (size_t)s * L + min(l0 + p, L - 1);
    yv[k] = ok ? (int)y[gi] : -1;
    const float wgt = ok ? wl[gi] : 0.f;
    coef[k] = wgt * inv_bl;
    float e[VP], se = 0.f, py = 0.f;
#pragma unroll
    for (int v = 0; v < VP; ++v) {
      const float2 mv = ms[p * 32 + v];
      const float z = row < NR ? zt[row * ZS + v] : 0.f;
      P[k][v] = ok && v < V ? __expf(z - mv.x) * mv.y : 0.f;
      e[v] = ok && v < V ? __expf(P[k][v]) : 0.f;
      se += e[v];
      py += v == yv[k] ? P[k][v] : 0.f;
    }
    rse[k] = se > 0.f ? 1.0f / se : 0.f;
    lsum += ok ? wgt * (__logf(se) - py) : 0.f;
    if (row < NR) {
#pragma unroll
      for (int v = 0; v < VP; ++v) zt[row * ZS + v] = coef[k] * (e[v] * rse[k] - (v == yv[k] ? 1.f : 0.f)) * P[k][v];
    }
  }
  __syncthreads();
  // (4) T = sum_b G P for every (p, v)
  {
    float a = 0.f;
    for (int s = part; s < B; s += PARTS) a += zt[(pp * B + s) * ZS + pv];
    red[part * NPAIR + pair] = make_float2(a, 0.f);
  }
  __syncthreads();
  if (tid < NPAIR) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < PARTS; ++k) a += red[k * NPAIR + tid].x;
    tt[tid] = a;
  }
  __syncthreads();
  // (5) dZ = P (G - T): fp32 into the table, bf16 rows for the dWo GEMM
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int row = tid + 512 * k;
    if (row >= NR) continue;
    const int p = row / B, s = row - (row / B) * B;
    const bool ok = l0 + p < L;
    float d[VP];
#pragma unroll
    for (int v = 0; v < VP; ++v) {
      const float G = coef[k] * (__expf(P[k][v]) * rse[k] - (v == yv[k] ? 1.f : 0.f));
      d[v] = ok && v < V ? P[k][v] * (G - tt[p * 32 + v]) : 0.f;
      zt[row * ZS + v] = d[v];
    }
    if (ok) {
      uint4* dst = reinterpret_cast<uint4*>(dz + ((size_t)s * L + l0 + p) * VP);
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[c] = packq8(d + 8 * c);
    }
  }
  lsum = wave_reduce_sum(lsum);
  if (lane == 0) lred[w] = lsum;
  __syncthreads();
  if (tid == 0) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) a += lred[k];
    loss_part[blockIdx.x] = a * inv_bl;
  }
  // (6a) dbo partial: column sums of dZ (16 row slices of the 32 columns)
  {
    const int v = tid & 31, sl = tid >> 5;
    float a = 0.f;
    for (int row = sl; row < NR; row += 16) a += zt[row * ZS + v];
    reinterpret_cast<float*>(red)[sl * 32 + v] = a;
  }
  // (6b) dh = dZ Wo: A fragments (bf16 of the fp32 table) of this wave's row tiles first
  constexpr int TPW = ROWSF / 32 / 8;               // row tiles per wave
  bf16x8 fa[TPW][2];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int row = (w + 8 * i) * 32 + r;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      float a8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) a8[j] = row < NR ? zt[row * ZS + kk * 16 + 8 * hh + j] : 0.f;
      fa[i][kk] = pack8(a8);
    }
  }
  __syncthreads();                                   // table and dbo slices read
  if (tid < V) {
    float a = 0.f;
#pragma unroll
    for (int sl = 0; sl < 16; ++sl) a += reinterpret_cast<float*>(red)[sl * 32 + tid];
    dbo_part[(size_t)blockIdx.x * V + tid] = a;
  }
  unsigned char* myot = smem + w * PT * 256;        // per-wave [32][128] bf16 staging over the table
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = w + 8 * i;
    if (t >= NT) break;
    f32x16_t acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = zero16();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int rlo = kk * 16 + 8 * hh + q;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int col = ct * 32 + tc;
        const bf16x8 fb = cat_tr(lds_tr(wos, swz256e(rlo, col)), lds_tr(wos, swz256e(rlo + 4, col)));
        acc[ct] = mfma32(fa[i][kk], fb, acc[ct]);
      }
    }
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        *reinterpret_cast<bf16_t*>(myot + swz256e((e & 3) + 8 * (e >> 2) + 4 * hh, ct * 32 + r)) = f2bf(acc[ct][e]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = lane + 64 * k;                 // 512 16-B chunks = 32 rows x 16
      const int rr = idx >> 4, c8 = idx & 15;
      const int row = t * 32 + rr;
      const int p = row / B, s = row - (row / B) * B;
      if (row < NR && l0 + p < L)
        *reinterpret_cast<uint4*>(dh + ((size_t)s * L + l0 + p) * CH + c8 * 8) =
            *reinterpret_cast<const uint4*>(myot + swz256(rr, c8));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}
}  // namespace

// Workspace sizes (floats) for pbx_local_head3: Z [B*L*32], part/tpart [ceil(B/16) * L * 32 * 2] each,
// MS/T [L * 32 * 2] each, loss_part / dbo_part [ntiles], [ntiles * V]; ntiles = ceil(B/16) ceil(L/32).
PBX_EXPORT int pbx_local_head3_tiles(int B, int L) { return ((B + SB - 1) / SB) * ((L + PT - 1) / PT); }

namespace {
constexpr int LDS1 = VP * 256 + VP * 4 + SB * PT * (VP + 1) * 4;
constexpr int LDS5 = 8 * PT * 256 + VP * 256 + PT * VP * 8 + PT * VP * 4 + VP * 4 + 8 * VP * 4;
void lhead3_attrs() {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lhead_logits_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS1);
    (void)hipFuncSetAttribute((const void*)lhead_grad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS5);
    attr = true;
  }
}
}  // namespace

// The five passes in three stages, so that a data-parallel group can share the batch axis of the softmax
// (parallel/batch_softmax.py): stage A = passes 1-2 -- with raw = 1 the fold leaves (M, S) for the caller
// to merge over ranks into (M, 1/S) --, stage B = passes 3-4 (T, which the caller sums over ranks),
// stage C = pass 5.
PBX_EXPORT int pbx_local_head3_a(const void* h, const float* wo, const float* bo, float* Z, float* part, float* MS,
                                 int raw, int B, int L, int V, hipStream_t st) {
  if (V > VP || V < 1 || B < 1 || L < 1) return (int)hipErrorInvalidValue;
  lhead3_attrs();
  const int nt = pbx_local_head3_tiles(B, L);
  const int nch = (B + SB - 1) / SB;
  hipLaunchKernelGGL(lhead_logits_kernel, dim3(nt), dim3(512), LDS1, st, (const bf16_t*)h, wo, bo, Z, (float2*)part,
                     B, L, V);
  hipLaunchKernelGGL(lhead_fold_kernel, dim3((L * VP + 63) / 64), dim3(256), 0, st, (const float2*)part, nch, L,
                     (float2*)MS, raw ? 2 : 0);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_local_head3_b(const float* Z, const float* MS, const void* y, const float* wl, float* tpart,
                                 float* loss_part, float* T, int B, int L, int V, hipStream_t st) {
  if (V > VP || V < 1 || B < 1 || L < 1) return (int)hipErrorInvalidValue;
  const int nt = pbx_local_head3_tiles(B, L);
  const int nch = (B + SB - 1) / SB;
  const float inv_bl = 1.0f / ((float)B * (float)L);
  hipLaunchKernelGGL(lhead_ce_kernel, dim3(nt), dim3(512), 0, st, Z, (const float2*)MS, (const long long*)y, wl,
                     (float2*)tpart, loss_part, B, L, V, inv_bl);
  hipLaunchKernelGGL(lhead_fold_kernel, dim3((L * VP + 63) / 64), dim3(256), 0, st, (const float2*)tpart, nch, L,
                     (float2*)T, 1);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_local_head3_c(const float* Z, const float* MS, const float* T, const void* y, const float* wl,
                                 const float* wo, const float* bo, void* dh, void* dz, float* dbo_part, int B, int L,
                                 int V, hipStream_t st) {
  if (V > VP || V < 1 || B < 1 || L < 1) return (int)hipErrorInvalidValue;
  lhead3_attrs();
  const int nt = pbx_local_head3_tiles(B, L);
  const float inv_bl = 1.0f / ((float)B * (float)L);
  hipLaunchKernelGGL(lhead_grad_kernel, dim3(nt), dim3(512), LDS5, st, Z, (const float2*)MS, (const float2*)T,
                     (const long long*)y, wl, wo, bo, (bf16_t*)dh, (bf16_t*)dz, dbo_part, B, L, V, inv_bl);
  return pbx_launch_status();
}

// Passes 1-5 (see header).  Outputs: dh [B][L][128] bf16, dz [B*L][32] bf16 (for dWo = dz^T h, a GEMM
// the caller issues), dbo_part [ntiles][V], loss_part [ntiles] (each already divided by B L).
PBX_EXPORT int pbx_local_head3(const void* h, const float* wo, const float* bo, const void* y, const float* wl,
                               void* dh, void* dz, float* dbo_part, float* loss_part, float* Z, float* part,
                               float* tpart, float* MS, float* T, int B, int L, int V, hipStream_t st) {
  int rc = pbx_local_head3_a(h, wo, bo, Z, part, MS, 0, B, L, V, st);
  if (rc == 0) rc = pbx_local_head3_b(Z, MS, y, wl, tpart, loss_part, T, B, L, V, st);
  if (rc == 0) rc = pbx_local_head3_c(Z, MS, T, y, wl, wo, bo, dh, dz, dbo_part, B, L, V, st);
  return rc;
}

// Positions per workgroup of pbx_local_head_fused: 2 for B <= 512, 1 for B <= 1024 (0: unsupported).
PBX_EXPORT int pbx_local_head_fused_pp(int B) { return B <= 512 ? 2 : B <= 1024 ? 1 : 0; }

// One-launch head (B <= 1024): dbo_part [ceil(L / pp)][V], loss_part [ceil(L / pp)] (each already / (B L)),
// pp = pbx_local_head_fused_pp(B)
PBX_EXPORT int pbx_local_head_fused(const void* h, const float* wo, const float* bo, const void* y, const float* wl,
                                    void* dh, void* dz, float* dbo_part, float* loss_part, int B, int L, int V,
                                    hipStream_t st) {
  const int pp = pbx_local_head_fused_pp(B);
  if (V > VP || V < 1 || B < 1 || pp == 0 || L < 1) return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lhead_fused_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, FUSED_LDS);
    (void)hipFuncSetAttribute((const void*)lhead_fused_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, FUSED_LDS);
    attr = true;
  }
  const float inv_bl = 1.0f / ((float)B * (float)L);
  hipLaunchKernelGGL(pp == 2 ? lhead_fused_kernel<2> : lhead_fused_kernel<1>, dim3((L + pp - 1) / pp), dim3(512),
                     FUSED_LDS, st, (const bf16_t*)h, wo, bo, (const long long*)y, wl, (bf16_t*)dh, (bf16_t*)dz,
                     dbo_part, loss_part, B, L, V, inv_bl);
  return pbx_launch_status();
}
