// Fused paper-semantics attention (local -> global, one query per head, softmax over positions):
// the K / V projections run on MFMA inside the attention kernels, so the [B*L, H*(K+VD)]
// pre-activation tensor of paper_attn.hip (400 MB per block at B=512, L=512, written once and read
// three times) never exists.  Published ProteinBERT attention; the reference's GlobalAttentionHead
// (modules.py:49-60) softmaxes over the key axis instead (reference semantics).
//
//   k = tanh(h2 Wk_h) [L, 64],  v = GELU(h2 Wv_h) [L, 128],  s = k . q_h (q pre-scaled by 1/sqrt(K)),
//   o_h = sum_l softmax_l(s) v_l   (pad-masked)
//
// Workgroup = 8 waves x 32 positions (one "chunk" of 256 positions of one sample) and one PAIR of
// heads whose [Wk | Wv] rows (2 x 192 rows x 256 B = 96 KB) stay in LDS for the workgroup's lifetime
// (blockIdx.y = head pair; persistent over (sample, chunk) items).
//   keys   D[k][pos] (A = Wk^T rows, B = h2 row fragments: lane = position) -> the score reduces over
//          k inside the lane;
//   values forward: D[pos][v] (A = the SAME h2 fragments, B = Wv^T rows: lane = value column) -> the
//          softmax-weighted sum over positions stays inside the lane; backward: D[v][pos] (lane =
//          position) so the dO . v reduction is in-lane and the dv / dk tiles are directly the B
//          operands of dh2 = Wv dv + Wk dk (A = transposed LDS reads of the same weight rows).
// Forward partials (m, l, acc[128]) per (sample, head, chunk) merge in a combine kernel (o, lse);
// the backward writes dh2 per head pair, the dpre = [dk | dv] rows for the weight-gradient GEMM and
// fixed-order dq partials.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int PK = 64;                 // key dim
constexpr int PV = 128;                // value dim per head
constexpr int HROWS = PK + PV;         // weight-image rows per head: 64 key rows, then 128 value rows
constexpr int HP = 2;                  // heads per workgroup
constexpr int NW = 8;                  // waves per workgroup
constexpr int CHUNK = 32 * NW;         // positions per work item
constexpr int WBYTES = HP * HROWS * 256;

__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __expf(2.0f * x);               // saturates correctly at +-inf
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}

__device__ __forceinline__ void stage_img(unsigned char* dst, const bf16_t* __restrict__ w) {
  stage_chunks(
      HP * HROWS * 16, [&](int idx) { return *reinterpret_cast<const uint4*>(w + (size_t)idx * 8); },
      [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(dst + swz256(idx >> 4, idx & 15)) = v; });
}

// h2 row fragments of position `pos` (lane = position r, half h: channels kk*16 + 8h .. +8)
__device__ __forceinline__ void load_hf(bf16x8* hf, const bf16_t* __restrict__ h2, int b, int pos, int L, int h) {
  const bool ok = pos < L;
  const bf16_t* src = h2 + ((size_t)b * L + min(pos, L - 1)) * CH;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const uint4 v = *reinterpret_cast<const uint4*>(src + kk * 16 + 8 * h);
    hf[kk] = __builtin_bit_cast(bf16x8, ok ? v : make_uint4(0u, 0u, 0u, 0u));
  }
}

// D[row][pos] for 32 weight rows starting at `row0`: A = weight rows, B = h2 fragments
__device__ __forceinline__ f32x16_t rows_x_h(const unsigned char* ws, int row0, const bf16x8* hf, int r, int h) {
  f32x16_t acc = zero16();
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) acc = mfma32(lds_frag(ws, swz256(row0 + r, kk * 2 + h)), hf[kk], acc);
  return acc;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Reduce-scatter over the 32 lanes of a half-wave: on entry every lane holds v[0..31]; on exit lane r
// (= lane & 31) returns sum over the 32 lanes of v[r].  31 exchanges instead of 32 x 5.  Each stage
// is a template instance so every register index is a compile-time constant (a runtime index into a
// register array becomes a compare/select chain per access).
template <int N>
__device__ __forceinline__ void rs_stage(float (&v)[32], int r) {
  const bool up = (r & N) != 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float send = up ? v[i] : v[i + N];
    const float keep = up ? v[i + N] : v[i];
    v[i] = keep + __shfl_xor(send, N, 64);
  }
}
__device__ __forceinline__ float reduce_scatter32(float (&v)[32], int r) {
  rs_stage<16>(v, r);
  rs_stage<8>(v, r);
  rs_stage<4>(v, r);
  rs_stage<2>(v, r);
  rs_stage<1>(v, r);
  return v[0];
}

// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(512) pa_fused_fwd_kernel(
    const bf16_t* __restrict__ h2, const bf16_t* __restrict__ wimg, const float* __restrict__ qs,
    const unsigned char* __restrict__ mask, float* __restrict__ part, int B, int L, int H) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;
  float* qsl = reinterpret_cast<float*>(smem + WBYTES);            // [HP][64]
  float* pb = qsl + HP * PK;                                         // [NW][32] softmax weights
  float* mrg = pb + NW * 32;                                         // [NW][HP][2 + PV]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int h0 = blockIdx.y * HP;
  const int nsplit = (L + CHUNK - 1) / CHUNK;
  const long items = (long)B * nsplit;
  stage_img(ws, wimg + (size_t)h0 * HROWS * CH);
  for (long item = blockIdx.x; item < items; item += gridDim.x) {
    const int b = (int)(item / nsplit), c = (int)(item - (item / nsplit) * nsplit);
    __syncthreads();                                               // previous item's LDS readers done
    if (tid < HP * PK) qsl[tid] = qs[((size_t)b * H + h0) * PK + tid];
    __syncthreads();
    const int pos = c * CHUNK + w * 32 + r;
    const bool okp = pos < L && (mask == nullptr || mask[(size_t)b * L + min(pos, L - 1)] != 0);
    bf16x8 hf[8];
    load_hf(hf, h2, b, pos, L, h);
#pragma unroll
    for (int j = 0; j < HP; ++j) {
      // ---- score of this lane's position: s = sum_k q_k tanh(key_k)
      float sp = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const f32x16_t ka = rows_x_h(ws, j * HROWS + kb * 32, hf, r, h);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 q4 = *reinterpret_cast<const float4*>(qsl + j * PK + kb * 32 + 8 * g + 4 * h);
          sp += q4.x * tanh_fast(ka[4 * g]) + q4.y * tanh_fast(ka[4 * g + 1]) + q4.z * tanh_fast(ka[4 * g + 2]) +
                q4.w * tanh_fast(ka[4 * g + 3]);
        }
      }
      const float s = okp ? sp + __shfl_xor(sp, 32, 64) : -INFINITY;
      const float m = wave_max(s);
      const float p = (okp && m > -INFINITY) ? __expf(s - m) : 0.f;
      const float l = wave_reduce_sum(h == 0 ? p : 0.f);
      if (h == 0) pb[w * 32 + r] = p;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // ---- values: D[pos][v] (lane = value column v), weighted by p over this tile's positions
      float av[4];
#pragma unroll
      for (int vb = 0; vb < 4; ++vb) {
        f32x16_t va = zero16();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
          va = mfma32(hf[kk], lds_frag(ws, swz256(j * HROWS + PK + vb * 32 + r, kk * 2 + h)), va);
        float a = 0.f;
#pragma unroll
        for (int hg = 0; hg < 2; ++hg) {
          const f32x2 xi[4] = {(f32x2){va[8 * hg], va[8 * hg + 1]}, (f32x2){va[8 * hg + 2], va[8 * hg + 3]},
                               (f32x2){va[8 * hg + 4], va[8 * hg + 5]}, (f32x2){va[8 * hg + 6], va[8 * hg + 7]}};
          f32x2 gv[4];
          gelu2_fast_n<4, false>(xi, gv);
#pragma unroll
          for (int gg = 0; gg < 2; ++gg) {
            const int g = 2 * hg + gg;
            const float4 p4 = *reinterpret_cast<const float4*>(pb + w * 32 + 8 * g + 4 * h);
            a += p4.x * gv[2 * gg].x + p4.y * gv[2 * gg].y + p4.z * gv[2 * gg + 1].x + p4.w * gv[2 * gg + 1].y;
          }
        }
        av[vb] = a + __shfl_xor(a, 32, 64);
      }
      float* mw = mrg + (w * HP + j) * (2 + PV);
      if (lane == 0) { mw[0] = m; mw[1] = l; }
      if (h == 0) {
#pragma unroll
        for (int vb = 0; vb < 4; ++vb) mw[2 + vb * 32 + r] = av[vb];
      }
    }
    __syncthreads();
    if (w < HP) {                                                  // wave j merges head j over the NW waves
      const int j = w;
      float M = -INFINITY;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) M = fmaxf(M, mrg[(ww * HP + j) * (2 + PV)]);
      float Ls = 0.f, A0 = 0.f, A1 = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) {
        const float* mw = mrg + (ww * HP + j) * (2 + PV);
        const float cw = (mw[0] == -INFINITY) ? 0.f : __expf(mw[0] - M);
        Ls = fmaf(mw[1], cw, Ls);
        A0 = fmaf(mw[2 + 2 * lane], cw, A0);
        A1 = fmaf(mw[3 + 2 * lane], cw, A1);
      }
      float* out = part + (((size_t)b * H + h0 + j) * nsplit + c) * (2 + PV);
      if (lane == 0) { out[0] = M; out[1] = Ls; }
      out[2 + 2 * lane] = A0;
      out[3 + 2 * lane] = A1;
    }
  }
}

// one wave per (b, h): merge the chunk partials -> o [B, H*VD] (fp32), lse [B*H]
__global__ __launch_bounds__(64) void pa_fused_combine_kernel(const float* __restrict__ part, float* __restrict__ o,
                                                             float* __restrict__ lse, int nsplit) {
  const int bh = blockIdx.x, lane = threadIdx.x;
  const float* p = part + (size_t)bh * nsplit * (2 + PV);
  float M = -INFINITY;
  for (int i = 0; i < nsplit; ++i) M = fmaxf(M, p[i * (2 + PV)]);
  float Ls = 0.f, A0 = 0.f, A1 = 0.f;
  for (int i = 0; i < nsplit; ++i) {
    const float* q = p + i * (2 + PV);
    const float c = (q[0] == -INFINITY) ? 0.f : __expf(q[0] - M);
    Ls = fmaf(q[1], c, Ls);
    A0 = fmaf(q[2 + 2 * lane], c, A0);
    A1 = fmaf(q[3 + 2 * lane], c, A1);
  }
  const float inv = Ls > 0.f ? 1.0f / Ls : 0.f;      // a fully padded row has no key: output 0
  o[(size_t)bh * PV + 2 * lane] = A0 * inv;
  o[(size_t)bh * PV + 2 * lane + 1] = A1 * inv;
  if (lane == 0) lse[bh] = Ls > 0.f ? M + __logf(Ls) : INFINITY;
}

// ------------------------------------------------------------------------------------------------
// backward: recompute keys / values per tile, p = exp(s - lse);
//   dv = p dO GELU'(v_pre) ; ds = p (dO . v - dO . o) ; dk = ds q (1 - tanh^2) ; dq = sum_l ds tanh(k)
//   dh2 (per head pair) = Wv dv + Wk dk ; dpre rows = [dk | dv] (for dW = h2^T dpre)
// 8 waves (two per SIMD) of 32 positions; the keys are recomputed after the value loop instead of
// keeping 32 tanh values live across it, which fits a wave in 256 registers
template <int NWB>
__global__ void __launch_bounds__(64 * NWB) pa_fused_bwd_kernel(
    const bf16_t* __restrict__ h2, const bf16_t* __restrict__ wimg, const float* __restrict__ qs,
    const unsigned char* __restrict__ mask, const float* __restrict__ lse, const float* __restrict__ o,
    const float* __restrict__ dO, bf16_t* __restrict__ dh2, bf16_t* __restrict__ dpre, float* __restrict__ dq_part,
    int B, int L, int H) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;
  float* qsl = reinterpret_cast<float*>(smem + WBYTES);            // [HP][64]
  float* dol = qsl + HP * PK;                                        // [HP][128]
  float* cst = dol + HP * PV;                                        // [HP][2]: lse, D = dO . o
  float* dqs = cst + HP * 2;                                         // [NWB][HP][64]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int h0 = blockIdx.y * HP;
  constexpr int CHUNKB = 32 * NWB;
  const int nsplit = (L + CHUNKB - 1) / CHUNKB;
  const long items = (long)B * nsplit;
  const int NC = H * (PK + PV);                                      // dpre row length
  bf16_t* dh2p = dh2 + (size_t)blockIdx.y * B * L * CH;              // this head pair's dh2 buffer
  stage_img(ws, wimg + (size_t)h0 * HROWS * CH);
  for (long item = blockIdx.x; item < items; item += gridDim.x) {
    const int b = (int)(item / nsplit), c = (int)(item - (item / nsplit) * nsplit);
    __syncthreads();
    if (tid < HP * PK) qsl[tid] = qs[((size_t)b * H + h0) * PK + tid];
    if (tid < HP * PV) dol[tid] = dO[((size_t)b * H + h0) * PV + tid];
    if (w < HP) {                                                  // D_j = dO_j . o_j, lse_j
      const size_t base = ((size_t)b * H + h0 + w) * PV;
      const float d = wave_reduce_sum(dO[base + 2 * lane] * o[base + 2 * lane] +
                                      dO[base + 2 * lane + 1] * o[base + 2 * lane + 1]);
      if (lane == 0) { cst[2 * w] = lse[(size_t)b * H + h0 + w]; cst[2 * w + 1] = d; }
    }
    __syncthreads();
    const int pos = c * CHUNKB + w * 32 + r;
    const bool inb = pos < L;
    const bool okp = inb && (mask == nullptr || mask[(size_t)b * L + min(pos, L - 1)] != 0);
    const size_t row = (size_t)b * L + min(pos, L - 1);
    bf16x8 hf[8];
    load_hf(hf, h2, b, pos, L, h);
    f32x16_t y[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) y[ct] = zero16();
#pragma unroll 1
    for (int j = 0; j < HP; ++j) {
      const int hd = h0 + j;
      // ---- keys (pass 1): score and p
      float sp = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const f32x16_t ka = rows_x_h(ws, j * HROWS + kb * 32, hf, r, h);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 q4 = *reinterpret_cast<const float4*>(qsl + j * PK + kb * 32 + 8 * g + 4 * h);
          sp += q4.x * tanh_fast(ka[4 * g]) + q4.y * tanh_fast(ka[4 * g + 1]) + q4.z * tanh_fast(ka[4 * g + 2]) +
                q4.w * tanh_fast(ka[4 * g + 3]);
        }
      }
      const float s = sp + __shfl_xor(sp, 32, 64);
      const float p = okp ? __expf(s - cst[2 * j]) : 0.f;
      // ---- values (lane = position): dv, dO . v, dh2 += Wv dv
      float dp = 0.f;
#pragma unroll 1
      for (int vb = 0; vb < 4; ++vb) {
        const f32x16_t va = rows_x_h(ws, j * HROWS + PK + vb * 32, hf, r, h);
        float dv[16];
#pragma unroll
        for (int hg = 0; hg < 2; ++hg) {
          const f32x2 xi[4] = {(f32x2){va[8 * hg], va[8 * hg + 1]}, (f32x2){va[8 * hg + 2], va[8 * hg + 3]},
                               (f32x2){va[8 * hg + 4], va[8 * hg + 5]}, (f32x2){va[8 * hg + 6], va[8 * hg + 7]}};
          f32x2 gv[4], gd[4];
          gelu2_both_n<4>(xi, gv, gd);
#pragma unroll
          for (int gg = 0; gg < 2; ++gg) {
            const int g = 2 * hg + gg;
            const float4 d4 = *reinterpret_cast<const float4*>(dol + j * PV + vb * 32 + 8 * g + 4 * h);
            dp += d4.x * gv[2 * gg].x + d4.y * gv[2 * gg].y + d4.z * gv[2 * gg + 1].x + d4.w * gv[2 * gg + 1].y;
            dv[4 * g] = p * d4.x * gd[2 * gg].x;
            dv[4 * g + 1] = p * d4.y * gd[2 * gg].y;
            dv[4 * g + 2] = p * d4.z * gd[2 * gg + 1].x;
            dv[4 * g + 3] = p * d4.w * gd[2 * gg + 1].y;
          }
        }
        if (inb) {
          bf16_t* drow = dpre + row * NC + H * PK + hd * PV + vb * 32;
#pragma unroll
          for (int g = 0; g < 4; ++g) *reinterpret_cast<uint2*>(drow + 8 * g + 4 * h) = packq4(dv + 4 * g);
        }
#pragma unroll
        for (int sh = 0; sh < 2; ++sh) {
          const bf16x8 fb = pack8(dv + 8 * sh);
          const int rlo = j * HROWS + PK + vb * 32 + 16 * sh + 4 * h + q;
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) {
            const int col = ct * 32 + tc;
            const bf16x8 fa = cat_tr(lds_tr(ws, swz256e(rlo, col)), lds_tr(ws, swz256e(rlo + 8, col)));
            y[ct] = mfma32(fa, fb, y[ct]);
          }
        }
      }
      dp += __shfl_xor(dp, 32, 64);
      const float ds = p * (dp - cst[2 * j + 1]);
      // ---- keys (pass 2, recomputed: cheaper than 32 live registers across the value loop):
      //      dk = ds q (1 - t^2) -> dpre, dh2 += Wk dk ; dq terms u = ds t
      float u[32];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const f32x16_t ka = rows_x_h(ws, j * HROWS + kb * 32, hf, r, h);
        float dk[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 q4 = *reinterpret_cast<const float4*>(qsl + j * PK + kb * 32 + 8 * g + 4 * h);
          const float qq[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float tv = tanh_fast(ka[4 * g + e]);
            dk[4 * g + e] = ds * qq[e] * fmaf(-tv, tv, 1.0f);
            u[kb * 16 + 4 * g + e] = ds * tv;
          }
        }
        if (inb) {
          bf16_t* drow = dpre + row * NC + hd * PK + kb * 32;
#pragma unroll
          for (int g = 0; g < 4; ++g) *reinterpret_cast<uint2*>(drow + 8 * g + 4 * h) = packq4(dk + 4 * g);
        }
#pragma unroll
        for (int sh = 0; sh < 2; ++sh) {
          const bf16x8 fb = pack8(dk + 8 * sh);
          const int rlo = j * HROWS + kb * 32 + 16 * sh + 4 * h + q;
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) {
            const int col = ct * 32 + tc;
            const bf16x8 fa = cat_tr(lds_tr(ws, swz256e(rlo, col)), lds_tr(ws, swz256e(rlo + 8, col)));
            y[ct] = mfma32(fa, fb, y[ct]);
          }
        }
      }
      // dq: lane (r, h) ends with k = (r >> 4) * 32 + 8 ((r & 15) >> 2) + 4 h + (r & 3)
      const float dqv = reduce_scatter32(u, r);
      dqs[(w * HP + j) * PK + (r >> 4) * 32 + 8 * ((r & 15) >> 2) + 4 * h + (r & 3)] = dqv;
    }
    // dh2 of this head pair: y[ct][4g + e] = D[c = ct*32 + 8g + 4h + e][pos]
    if (inb) {
      bf16_t* drow = dh2p + row * CH;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float v4[4] = {y[ct][4 * g], y[ct][4 * g + 1], y[ct][4 * g + 2], y[ct][4 * g + 3]};
          *reinterpret_cast<uint2*>(drow + ct * 32 + 8 * g + 4 * h) = packq4(v4);
        }
    }
    __syncthreads();
    if (w < HP) {                                                  // fixed-order sum over the waves
      const int j = w;
      float a = 0.f;
#pragma unroll
      for (int ww = 0; ww < NWB; ++ww) a += dqs[(ww * HP + j) * PK + lane];
      dq_part[(((size_t)b * H + h0 + j) * nsplit + c) * PK + lane] = a;
    }
  }
}

int g_pf_cus = -1;
int pf_num_cus() {
  if (g_pf_cus < 0) {
    int dev = 0;
    g_pf_cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, dev) == hipSuccess) g_pf_cus = p.multiProcessorCount;
    }
  }
  return g_pf_cus;
}
bool g_pf_attrs = false;
void pf_attrs() {
  if (g_pf_attrs) return;
  (void)hipFuncSetAttribute((const void*)pa_fused_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)pa_fused_bwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  (void)hipFuncSetAttribute((const void*)pa_fused_bwd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
  g_pf_attrs = true;
}
dim3 pf_grid(long items, int H) {
  const int pairs = H / HP;
  long per = (pf_num_cus() + pairs - 1) / pairs;       // one workgroup per CU over all head pairs
  if (per > items) per = items;
  if (per < 1) per = 1;
  return dim3((unsigned)per, (unsigned)pairs);
}
}  // namespace

// h2 [B, L, 128] bf16; wimg [H][192][128] bf16 (rows: Wk_h^T (64), Wv_h^T (128)); qs [B, H, 64] fp32
// (tanh(g Wq) / sqrt(K)); mask [B, L] u8 or null; part [B*H][ceil(L/256)][130] fp32 workspace;
// o [B, H*128] fp32; lse [B*H] fp32.  H even.
PBX_EXPORT int pbx_pa_fused_fwd(const void* h2, const void* wimg, const float* qs, const void* mask, float* part,
                                float* o, float* lse, int B, int L, int H, hipStream_t st) {
  if (B <= 0 || L <= 0 || H <= 0 || (H % HP) != 0) return (int)hipErrorInvalidValue;
  pf_attrs();
  const int nsplit = (L + CHUNK - 1) / CHUNK;
  const int lds = WBYTES + (HP * PK + NW * 32 + NW * HP * (2 + PV)) * 4;
  hipLaunchKernelGGL(pa_fused_fwd_kernel, pf_grid((long)B * nsplit, H), dim3(64 * NW), lds, st, (const bf16_t*)h2,
                     (const bf16_t*)wimg, qs, (const unsigned char*)mask, part, B, L, H);
  hipLaunchKernelGGL(pa_fused_combine_kernel, dim3(B * H), dim3(64), 0, st, (const float*)part, o, lse, nsplit);
  return pbx_launch_status();
}

// dh2 [H/2][B, L, 128] bf16 (one buffer per head pair, every in-range row written); dpre [B, L, H*(64+128)]
// bf16 ([dk heads | dv heads], in-range rows written); dq_part [B*H][ceil(L/(32 nwb))][64] fp32 (written)
PBX_EXPORT int pbx_pa_fused_bwd(const void* h2, const void* wimg, const float* qs, const void* mask, const float* lse,
                                const float* o, const float* dO, void* dh2, void* dpre, float* dq_part, int B, int L,
                                int H, int nwb, hipStream_t st) {
  if (B <= 0 || L <= 0 || H <= 0 || (H % HP) != 0 || (nwb != 4 && nwb != 8)) return (int)hipErrorInvalidValue;
  pf_attrs();
  const int nsplit = (L + 32 * nwb - 1) / (32 * nwb);
  const int lds = WBYTES + (HP * PK + HP * PV + HP * 2 + nwb * HP * PK) * 4;
  hipLaunchKernelGGL(nwb == 8 ? pa_fused_bwd_kernel<8> : pa_fused_bwd_kernel<4>, pf_grid((long)B * nsplit, H),
                     dim3(64 * nwb), lds, st, (const bf16_t*)h2, (const bf16_t*)wimg, qs, (const unsigned char*)mask,
                     lse, o, dO, (bf16_t*)dh2, (bf16_t*)dpre, dq_part, B, L, H);
  return pbx_launch_status();
}
