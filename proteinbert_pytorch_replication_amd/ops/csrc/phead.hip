// Local (amino-acid) pretraining head + loss, PAPER semantics, one launch (SURVEY K9/K10 paper mode).
//
// Reference: ProteinBERT/modules.py:277-284 (Linear C -> V + softmax) with the softmax over the
// vocabulary (the published model; the reference's implicit dim 0 softmax over the batch is
// semantics="reference", csrc/lhead.hip) and utils.py:293 (per-residue weighted CE, mean over B L):
//   Z = h Wo^T + bo ;  loss = 1/(BL) sum_rows w (logsumexp_v Z - Z[y])
//   dZ = w/(BL) (softmax_v(Z) - onehot(y)) ;  dh = dZ Wo ;  dbo = sum_rows dZ ;  dWo = dZ^T h
//
// One wave per 32-row tile (grid-stride).  Z^T = Wo h^T on MFMA (A = Wo rows from LDS, B = the tile's h
// rows straight from global), so a lane holds 16 of the 32 (padded) vocabulary logits of ONE row and
// the row softmax is an in-lane reduction plus one cross-half shuffle.  dh^T = Wo^T dZ^T reuses the
// logits' register layout as the B operand with its K (vocabulary) order permuted to
// {4h + 0..3, 8 + 4h + 0..3} per 16-step, and the transposed Wo reads deliver exactly that order
// (the attn_bwd2 pattern, ln.hip): no data movement between the two products.  dbo accumulates per lane
// across tiles and is reduced once per wave; dZ rows (bf16, 32 padded columns) go out for the dWo
// GEMM (K = B L, csrc/gemm.hip).  Replaces addmm + logsumexp + gather + softmax + scatter_add + mm +
// the bias sum (library GEMMs and seven elementwise launches).
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int VP = 32;    // padded vocabulary

__global__ void __launch_bounds__(256) phead_kernel(const bf16_t* __restrict__ h, const float* __restrict__ wo,
                                                    const float* __restrict__ bo, const long long* __restrict__ y,
                                                    const float* __restrict__ wl, bf16_t* __restrict__ dh,
                                                    bf16_t* __restrict__ dz, float* __restrict__ dbo_part,
                                                    float* __restrict__ loss_part, long R, int V, float inv_bl) {
  __shared__ __attribute__((aligned(16))) unsigned char wos[VP * 256];   // Wo bf16 [32][128] swz256
  __shared__ float bo_s[VP];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  for (int idx = tid; idx < VP * 16; idx += 256) {
    const int v = idx >> 4, c8 = idx & 15;
    float e[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (v < V) {
      const float4 a = *reinterpret_cast<const float4*>(wo + v * CH + c8 * 8);
      const float4 b = *reinterpret_cast<const float4*>(wo + v * CH + c8 * 8 + 4);
      e[0] = a.x; e[1] = a.y; e[2] = a.z; e[3] = a.w; e[4] = b.x; e[5] = b.y; e[6] = b.z; e[7] = b.w;
    }
    *reinterpret_cast<uint4*>(wos + swz256(v, c8)) = packq8(e);
  }
  if (tid < VP) bo_s[tid] = tid < V ? bo[tid] : 0.f;
  __syncthreads();
  bf16x8 wf[8];                                     // A = Wo rows (v = r), k = channels
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) wf[kk] = lds_frag(wos, swz256(r, kk * 2 + hh));
  bf16x8 wt[2][4];                                  // A = Wo^T (rows c), k = vocabulary (permuted order)
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
      wt[ks][ct] = cat_tr(lds_tr(wos + 4096 * ks, swz256e(4 * hh + q, ct * 32 + tc)),
                          lds_tr(wos + 4096 * ks, swz256e(4 * hh + q + 8, ct * 32 + tc)));
  float bov[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) bov[e] = bo_s[(e & 3) + 8 * (e >> 2) + 4 * hh];
  float dbo[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) dbo[e] = 0.f;
  float lsum = 0.f;
  const long ntile = (R + 31) / 32;
  for (long t = (long)blockIdx.x * 4 + w; t < ntile; t += (long)gridDim.x * 4) {
    const long row = t * 32 + r;
    const bool ok = row < R;
    const long rc = ok ? row : R - 1;
    const bf16_t* src = h + rc * CH + 8 * hh;
    bf16x8 hf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) hf[kk] = *reinterpret_cast<const bf16x8*>(src + kk * 16);
    const int yv = ok ? (int)y[rc] : -1;
    const float wgt = ok ? wl[rc] * inv_bl : 0.f;
    f32x16_t z = zero16();
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) z = mfma32(wf[kk], hf[kk], z);   // z[e]: v = (e&3) + 8(e>>2) + 4 hh, row r
    float m = -3.0e38f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int v = (e & 3) + 8 * (e >> 2) + 4 * hh;
      z[e] = v < V ? z[e] + bov[e] : -3.0e38f;
      m = fmaxf(m, z[e]);
    }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float se = 0.f, zy = 0.f;
    float p[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int v = (e & 3) + 8 * (e >> 2) + 4 * hh;
      p[e] = v < V ? __expf(z[e] - m) : 0.f;
      se += p[e];
      zy += v == yv ? z[e] : 0.f;
    }
    se += __shfl_xor(se, 32, 64);
    zy += __shfl_xor(zy, 32, 64);
    const float inv = 1.0f / se;
    if (hh == 0) lsum += ok ? wgt * (m + __logf(se) - zy) : 0.f;
    float g[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int v = (e & 3) + 8 * (e >> 2) + 4 * hh;
      g[e] = wgt * (p[e] * inv - (v == yv ? 1.f : 0.f));
    }
    // dZ rows (bf16) for the dWo GEMM: lane holds v = 4hh + {0..3} + 8 j, stored as 4 x 8-byte runs
    const uint2 q0 = packq4(g), q1 = packq4(g + 4), q2 = packq4(g + 8), q3 = packq4(g + 12);
    if (ok) {
      bf16_t* zr = dz + row * VP + 4 * hh;
      *reinterpret_cast<uint2*>(zr) = q0;
      *reinterpret_cast<uint2*>(zr + 8) = q1;
      *reinterpret_cast<uint2*>(zr + 16) = q2;
      *reinterpret_cast<uint2*>(zr + 24) = q3;
    }
    // the bias gradient and dh use the stored (bf16-rounded) dZ, as the dWo GEMM does
    float gr[16];
    unpack4(q0, gr);
    unpack4(q1, gr + 4);
    unpack4(q2, gr + 8);
    unpack4(q3, gr + 12);
#pragma unroll
    for (int e = 0; e < 16; ++e) dbo[e] += gr[e];
    const bf16x8 b0 = pack8(gr), b1 = pack8(gr + 8);     // B = dZ^T, k-steps v 0..15 / 16..31
    f32x16_t d[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      d[ct] = mfma32(wt[0][ct], b0, zero16());
      d[ct] = mfma32(wt[1][ct], b1, d[ct]);
    }
    if (ok) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const float o[4] = {d[ct][4 * gq], d[ct][4 * gq + 1], d[ct][4 * gq + 2], d[ct][4 * gq + 3]};
          *reinterpret_cast<uint2*>(dh + row * CH + ct * 32 + 8 * gq + 4 * hh) = packq4(o);
        }
    }
  }
  // per-wave partials: dbo over the 32 rows of every lane group, the loss over the wave
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    float s = dbo[e];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) s += __shfl_xor(s, o, 64);
    dbo[e] = s;
  }
  const long wid = (long)blockIdx.x * 4 + w;
  if (r == 0) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int v = (e & 3) + 8 * (e >> 2) + 4 * hh;
      if (v < V) dbo_part[wid * V + v] = dbo[e];
    }
  }
  lsum = wave_reduce_sum(lsum);
  if (lane == 0) loss_part[wid] = lsum;
}
}  // namespace

// Number of per-wave partial rows written by pbx_paper_head (dbo_part [n][V], loss_part [n]).
PBX_EXPORT int pbx_paper_head_parts(long R) {
  long ntile = (R + 31) / 32;
  long wg = (ntile + 3) / 4;
  if (wg > 1024) wg = 1024;
  return (int)(wg * 4);
}

// h [R][128] bf16, wo [V][128] fp32, bo [V], y [R] int64, wl [R] fp32 -> dh [R][128] bf16, dz [R][32] bf16
// (columns >= V zero), dbo_part [parts][V], loss_part [parts] (each already divided by B L = 1 / inv_bl).
PBX_EXPORT int pbx_paper_head(const void* h, const float* wo, const float* bo, const void* y, const float* wl, void* dh,
                              void* dz, float* dbo_part, float* loss_part, long R, int V, float inv_bl, hipStream_t st) {
  if (V < 1 || V > VP || R < 1) return (int)hipErrorInvalidValue;
  const int parts = pbx_paper_head_parts(R);
  hipLaunchKernelGGL(phead_kernel, dim3(parts / 4), dim3(256), 0, st, (const bf16_t*)h, wo, bo, (const long long*)y, wl,
                     (bf16_t*)dh, (bf16_t*)dz, dbo_part, loss_part, R, V, inv_bl);
  return pbx_launch_status();
}
