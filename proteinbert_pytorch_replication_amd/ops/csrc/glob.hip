// Global (per-protein) track, pretraining heads and losses.
//
// Reference: ProteinBERT/modules.py:175-199,221-229 (two Linear G->G + GELU + residual + LayerNorm(G)
// per block), :21-92 (attention output scaled by sum(W)/K in reference semantics), :277-293 (local
// head Linear C->V + nn.Softmax() over the BATCH axis, GO head Linear G->A + Sigmoid) and
// ProteinBERT/utils.py:293-294 (CE applied to the local probabilities, BCE with log clamp -100,
// weighted means over B*L and B*A).
//
// The [B, G] GEMMs run on hipBLASLt (bf16 in, fp32 out); everything around them is fused here:
//   row_ln_fwd  : z = res + GELU(u + b) [+ scale * sum_t vpart] -> LayerNorm(G)  (one row / workgroup)
//   row_ln_bwd  : LayerNorm + GELU backward, affine/bias gradients (accumulated in place), the
//                 attention-scale gradient and the gradient of the attention partial sums
//   local_head  : logits, softmax over the batch, CE on the probabilities, and the whole backward
//                 (the loss is terminal, so gradients are produced in the forward pass)
//   go_head     : sigmoid + BCE + weighted mean + dlogits in one pass over [B, A]
#include "mfma.h"

typedef unsigned short bf16_t;
using namespace pbx;

namespace {
constexpr int MAXG = 1024;   // global_dim supported by the row kernels (<= 4 values per thread)

__device__ __forceinline__ float block_reduce(float v, float* red) {
  v = wave_reduce_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// grid (B), block 256.  u: [B, G] GEMM output (no bias); out = LN(z)
__global__ void __launch_bounds__(256) row_ln_fwd_kernel(
    const float* __restrict__ u, const float* __restrict__ bias, const float* __restrict__ res,
    const float* __restrict__ vpart, int TV, const float* __restrict__ wp, int K, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ out, bf16_t* __restrict__ out_bf, float* __restrict__ xhat,
    float* __restrict__ rstd_out, float* __restrict__ vsum, int G, float eps) {
  __shared__ float red[8];
  const int b = blockIdx.x, tid = threadIdx.x;
  float scale = 0.f;
  if (vpart != nullptr) {
    float s = 0.f;
    for (int i = 0; i < K; ++i) s += wp[i];
    scale = s / (float)K;
  }
  float z[4];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    z[i] = 0.f;
    if (c < G) {
      float v = res[(size_t)b * G + c] + gelu_f(u[(size_t)b * G + c] + bias[c]);
      if (vpart != nullptr) {
        float vs = 0.f;
        for (int t = 0; t < TV; ++t) vs += vpart[((size_t)b * TV + t) * G + c];
        vsum[(size_t)b * G + c] = vs;
        v += scale * vs;
      }
      z[i] = v;
      sum += v;
    }
  }
  const float mean = block_reduce(sum, red) / (float)G;
  float var = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    if (c < G) var += (z[i] - mean) * (z[i] - mean);
  }
  var = block_reduce(var, red) / (float)G;
  const float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    if (c < G) {
      const float xh = (z[i] - mean) * rstd;
      const float o = xh * gamma[c] + beta[c];
      xhat[(size_t)b * G + c] = xh;
      out[(size_t)b * G + c] = o;
      out_bf[(size_t)b * G + c] = f2bf(o);
    }
  }
  if (tid == 0) rstd_out[b] = rstd;
}

// grid (B), block 256.  dout: [B, G] gradient of the LN output.
//   dz = rstd (dout g - mean(dout g) - xhat mean(dout g xhat))
//   dgamma += dout xhat ; dbeta += dout ; du = dz GELU'(u + b) (bf16, GEMM operand) ; dbias += du
//   dres = dz (fp32) ; with vpart: dvs = scale dz, dWp[i] += sum(dz vsum) / K
__global__ void __launch_bounds__(256) row_ln_bwd_kernel(
    const float* __restrict__ dout, const float* __restrict__ xhat, const float* __restrict__ rstd_in,
    const float* __restrict__ gamma, const float* __restrict__ u, const float* __restrict__ bias,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dbias, bf16_t* __restrict__ du,
    float* __restrict__ dres, const float* __restrict__ vsum, const float* __restrict__ wp, int K,
    float* __restrict__ dwp, float* __restrict__ dvs, int G) {
  __shared__ float red[8];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float rstd = rstd_in[b];
  float dxh[4], xh[4];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    dxh[i] = 0.f;
    xh[i] = 0.f;
    if (c < G) {
      const float d = dout[(size_t)b * G + c];
      xh[i] = xhat[(size_t)b * G + c];
      dxh[i] = d * gamma[c];
      s1 += dxh[i];
      s2 += dxh[i] * xh[i];
      atomicAdd(dgamma + c, d * xh[i]);
      atomicAdd(dbeta + c, d);
    }
  }
  const float m1 = block_reduce(s1, red) / (float)G;
  const float m2 = block_reduce(s2, red) / (float)G;
  float scale = 0.f;
  if (vsum != nullptr) {
    float s = 0.f;
    for (int i = 0; i < K; ++i) s += wp[i];
    scale = s / (float)K;
  }
  float ds = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    if (c < G) {
      const float dz = rstd * (dxh[i] - m1 - xh[i] * m2);
      dres[(size_t)b * G + c] = dz;
      const float g = dz * gelu_grad_f(u[(size_t)b * G + c] + bias[c]);
      du[(size_t)b * G + c] = f2bf(g);
      atomicAdd(dbias + c, g);
      if (vsum != nullptr) {
        dvs[(size_t)b * G + c] = scale * dz;
        ds += dz * vsum[(size_t)b * G + c];
      }
    }
  }
  if (vsum != nullptr) {
    ds = block_reduce(ds, red);
    if (tid < K) atomicAdd(dwp + tid, ds / (float)K);
  }
}

// out = GELU(u + b) (fp32 and bf16 copies); used for the global input layer and gb = global->local
__global__ void __launch_bounds__(256) bias_gelu_kernel(const float* __restrict__ u, const float* __restrict__ bias,
                                                        float* __restrict__ out, bf16_t* __restrict__ out_bf,
                                                        int n, int N) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float v = gelu_f(u[i] + bias[i % N]);
  if (out != nullptr) out[i] = v;
  if (out_bf != nullptr) out_bf[i] = f2bf(v);
}

// du = dout * GELU'(u + b) (bf16) ; dbias += column sums
__global__ void __launch_bounds__(256) bias_gelu_bwd_kernel(const float* __restrict__ dout,
                                                            const float* __restrict__ u,
                                                            const float* __restrict__ bias, bf16_t* __restrict__ du,
                                                            float* __restrict__ dbias, int M, int N) {
  // grid (ceil(N/256), ceil(M/rows_per_block)); each thread owns one column for a run of rows
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= N) return;
  const int rpb = (M + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rpb, r1 = min(M, r0 + rpb);
  float acc = 0.f;
  const float bc = bias[c];
  for (int r = r0; r < r1; ++r) {
    const float g = dout[(size_t)r * N + c] * gelu_grad_f(u[(size_t)r * N + c] + bc);
    du[(size_t)r * N + c] = f2bf(g);
    acc += g;
  }
  atomicAdd(dbias + c, acc);
}

// ------------------------------------------------------------------------------------------------
// Local head + loss, reference semantics (modules.py:277-284, utils.py:293):
//   z[b,l,v] = h[b,l] . Wo[v] + bo[v] ; P = softmax over b of z[., l, v]
//   loss_bl = logsumexp_v P[b,l,:] - P[b,l,y]          (CrossEntropyLoss applied to probabilities)
//   L_loc = sum_bl w_bl loss_bl / (B L)
// backward (in the same pass): G = w/(BL) (softmax_v(P) - onehot(y)); dz = P (G - sum_b G P);
//   dh = dz Wo (bf16) ; dWo += dz^T h ; dbo += sum dz.
// grid (L), block 256: one position l per workgroup, all B samples (B <= 1024).
__global__ void __launch_bounds__(256) local_head_kernel(
    const bf16_t* __restrict__ h, const float* __restrict__ wo, const float* __restrict__ bo,
    const long long* __restrict__ y, const float* __restrict__ wl, bf16_t* __restrict__ dh, float* __restrict__ dwo_part,
    float* __restrict__ dbo_part, float* __restrict__ loss, int B, int L, int V, float inv_bl) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* W = sm;                       // [V][128]
  float* zs = W + V * 128;             // [B][V]  logits -> probabilities -> dz
  float* red = zs + B * V;             // [8][V]  per-wave reductions
  float* colv = red + 8 * V;           // [V]
  const int tid = threadIdx.x, l = blockIdx.x;
  const int lane = tid & 63;
  for (int i = tid; i < V * 128; i += 256) W[i] = wo[i];
  __syncthreads();
  // logits: thread per sample row (the h row is read once; Wo reads are LDS broadcasts)
  for (int b = tid; b < B; b += 256) {
    const bf16_t* hr = h + ((size_t)b * L + l) * 128;
    float acc[32];
#pragma unroll
    for (int v = 0; v < 32; ++v) acc[v] = 0.f;
    for (int c8 = 0; c8 < 16; ++c8) {
      const uint4 q = *reinterpret_cast<const uint4*>(hr + c8 * 8);
      const float hv[8] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                           __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u),
                           __uint_as_float(q.z << 16), __uint_as_float(q.z & 0xffff0000u),
                           __uint_as_float(q.w << 16), __uint_as_float(q.w & 0xffff0000u)};
#pragma unroll
      for (int v = 0; v < 32; ++v) {
        if (v < V) {
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[v] = fmaf(hv[e], W[v * 128 + c8 * 8 + e], acc[v]);
        }
      }
    }
#pragma unroll
    for (int v = 0; v < 32; ++v)
      if (v < V) zs[b * V + v] = acc[v] + bo[v];
  }
  __syncthreads();
  // softmax over b for each v: 8 partial columns per v (8 threads), then combine
  {
    float* pm = colv + V;                // [8][V] partial max, then partial sum (reuses tail space)
    const int v = tid % 32, part = tid / 32;
    float m = -3.4e38f;
    if (v < V)
      for (int b = part; b < B; b += 8) m = fmaxf(m, zs[b * V + v]);
    if (v < V) red[part * V + v] = m;
    __syncthreads();
    if (tid < V) {
      float mm = -3.4e38f;
      for (int k = 0; k < 8; ++k) mm = fmaxf(mm, red[k * V + tid]);
      pm[tid] = mm;
    }
    __syncthreads();
    float sacc = 0.f;
    if (v < V)
      for (int b = part; b < B; b += 8) sacc += __expf(zs[b * V + v] - pm[v]);
    if (v < V) red[part * V + v] = sacc;
    __syncthreads();
    if (tid < V) {
      float ss = 0.f;
      for (int k = 0; k < 8; ++k) ss += red[k * V + tid];
      pm[V + tid] = 1.0f / ss;
    }
    __syncthreads();
    if (tid < V) { red[tid] = pm[tid]; red[V + tid] = pm[V + tid]; }
    __syncthreads();
  }
  for (int i = tid; i < B * V; i += 256) {
    const int v = i - (i / V) * V;
    zs[i] = __expf(zs[i] - red[v]) * red[V + v];
  }
  __syncthreads();
  // per (b, l): CE over v on the probabilities; G stored in place of P? keep P, accumulate colv = sum_b G P
  float lsum = 0.f;
  if (tid < V) colv[tid] = 0.f;
  __syncthreads();
  for (int b = tid; b < B; b += 256) {
    const float* p = zs + b * V;
    float mx = -3.4e38f;
    for (int v = 0; v < V; ++v) mx = fmaxf(mx, p[v]);
    float se = 0.f;
    for (int v = 0; v < V; ++v) se += __expf(p[v] - mx);
    const int yv = (int)y[(size_t)b * L + l];
    const float wgt = wl[(size_t)b * L + l];
    lsum += wgt * (mx + __logf(se) - p[yv]);
    const float coef = wgt * inv_bl;
    const float inv_se = 1.0f / se;
    for (int v = 0; v < V; ++v) {
      const float g = coef * (__expf(p[v] - mx) * inv_se - (v == yv ? 1.f : 0.f));
      atomicAdd(&colv[v], g * p[v]);
    }
  }
  __syncthreads();
  // dz = P (G - colv), recomputing G per element
  for (int b = tid; b < B; b += 256) {
    float* p = zs + b * V;
    float mx = -3.4e38f;
    for (int v = 0; v < V; ++v) mx = fmaxf(mx, p[v]);
    float se = 0.f;
    for (int v = 0; v < V; ++v) se += __expf(p[v] - mx);
    const int yv = (int)y[(size_t)b * L + l];
    const float coef = wl[(size_t)b * L + l] * inv_bl;
    const float inv_se = 1.0f / se;
    for (int v = 0; v < V; ++v) {
      const float g = coef * (__expf(p[v] - mx) * inv_se - (v == yv ? 1.f : 0.f));
      p[v] = p[v] * (g - colv[v]);
    }
  }
  __syncthreads();
  // dh[b,l,:] = sum_v dz[b,v] Wo[v,:]  (thread per (b, 8-channel chunk)); dWo += dz^T h
  for (int i = tid; i < B * 16; i += 256) {
    const int b = i >> 4, c8 = i & 15;
    const float* dz = zs + b * V;
    float o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int v = 0; v < V; ++v) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(dz[v], W[v * 128 + c8 * 8 + e], o[e]);
    }
    uint4 q;
    q.x = (unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16);
    q.y = (unsigned)f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16);
    q.z = (unsigned)f2bf(o[4]) | ((unsigned)f2bf(o[5]) << 16);
    q.w = (unsigned)f2bf(o[6]) | ((unsigned)f2bf(o[7]) << 16);
    *reinterpret_cast<uint4*>(dh + ((size_t)b * L + l) * 128 + c8 * 8) = q;
  }
  // per-position partials of dWo = sum_b dz[b,:]^T h[b,l,:] and dbo (summed over l by the caller):
  // thread (v pair vp = tid>>4, channel chunk c8 = tid&15) walks the batch
  {
    const int vp = tid >> 4, c8 = tid & 15;
    const int v0 = 2 * vp, v1 = 2 * vp + 1;
    float a0[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (v0 < V) {
      for (int b = 0; b < B; ++b) {
        const uint4 q = *reinterpret_cast<const uint4*>(h + ((size_t)b * L + l) * 128 + c8 * 8);
        const float hv[8] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                             __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u),
                             __uint_as_float(q.z << 16), __uint_as_float(q.z & 0xffff0000u),
                             __uint_as_float(q.w << 16), __uint_as_float(q.w & 0xffff0000u)};
        const float d0 = zs[b * V + v0], d1 = v1 < V ? zs[b * V + v1] : 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a0[e] = fmaf(d0, hv[e], a0[e]);
          a1[e] = fmaf(d1, hv[e], a1[e]);
        }
      }
      float* dst = dwo_part + (size_t)l * V * 128;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dst[v0 * 128 + c8 * 8 + e] = a0[e];
        if (v1 < V) dst[v1 * 128 + c8 * 8 + e] = a1[e];
      }
    }
  }
  if (tid < V) {
    float a = 0.f;
    for (int b = 0; b < B; ++b) a += zs[b * V + tid];
    dbo_part[(size_t)l * V + tid] = a;
  }
  lsum = wave_reduce_sum(lsum);
  if (lane == 0) atomicAdd(loss, lsum * inv_bl);
}

// MFMA version of the local head (B <= 608): one workgroup (8 waves; the MFMA phases use waves 0-3,
// the softmax / CE phases all 8) per position l; h_l is held in registers and passes through LDS in
// chunks of HC = 128 rows (twice: logits, then dWo), so the LDS holds only the [B][32] logit / dz
// tiles at full batch size.
//   logits  Z[b][v]   = h_l[b] . Wo[v] + bo[v]       (MFMA: A = h_l rows, B = Wo rows)
//   softmax over b, CE on the probabilities, dz      (VALU on the [B][32] logit tile, as above)
//   dWo_l[v][c]       = sum_b dz[b][v] h_l[b][c]     (MFMA: both operands transposed LDS reads)
//   dh[b][c]          = sum_v dz[b][v] Wo[v][c]      (MFMA, staged through LDS for 256-B row stores)
__global__ void __launch_bounds__(512) local_head_mfma_kernel(
    const bf16_t* __restrict__ h, const float* __restrict__ wo, const float* __restrict__ bo,
    const long long* __restrict__ y, const float* __restrict__ wl, bf16_t* __restrict__ dh, float* __restrict__ dwo_part,
    float* __restrict__ dbo_part, float* __restrict__ loss, int B, int L, int V, float inv_bl) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int HC = 128;
  const int Bp = (B + 31) & ~31;
  unsigned char* hs = smem;                                   // [HC][128] bf16 swz256 (h_l / dh chunk)
  unsigned char* wos = hs + HC * 256;                         // [32][128] bf16 swz256
  unsigned char* dzb = wos + 32 * 256;                        // [Bp][32] bf16, 64-B rows
  float* zs = reinterpret_cast<float*>(dzb + Bp * 64);        // [Bp][32] fp32
  float* red = zs + Bp * 32;                                  // [16][32]
  float* colv = red + 16 * 32;                                // [32] + [2][32]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  // Wo (bf16, zero rows beyond V)
  for (int idx = tid; idx < 32 * 16; idx += 512) {
    const int v = idx >> 4, c8 = idx & 15;
    float e[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (v < V) {
      const float4 a = *reinterpret_cast<const float4*>(wo + v * 128 + c8 * 8);
      const float4 b2 = *reinterpret_cast<const float4*>(wo + v * 128 + c8 * 8 + 4);
      e[0] = a.x; e[1] = a.y; e[2] = a.z; e[3] = a.w; e[4] = b2.x; e[5] = b2.y; e[6] = b2.z; e[7] = b2.w;
    }
    *reinterpret_cast<uint4*>(wos + swz256(v, c8)) = packq8(e);
  }
  const float bov = r < V ? bo[r] : 0.f;
  // a workgroup walks positions l = blockIdx.x, + gridDim.x, ...: its dWo / dbo partials sum over them
  // and are written once (row blockIdx.x of dwo_part / dbo_part)
  float lsum = 0.f, dbo_acc = 0.f;
  f32x16_t dwo_acc = zero16();
  for (int l = blockIdx.x; l < L; l += gridDim.x) {
    __syncthreads();                              // the previous position's dh stores read hs
    // h_l rows c0 .. c0 + HC - 1 -> hs (zero beyond B)
    // All of h_l (B <= 608 rows x 256 B) is loaded into registers once, up front (<= 5 chunks x 4 x 16 B
    // per thread): one HBM round trip instead of one per chunk and pass, and no second read for dWo.
    constexpr int MAXC = 5;
    uint4 hreg[MAXC][4];
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = tid + 512 * i;
        const int b = c * HC + (idx >> 4);
        hreg[c][i] = b < B ? *reinterpret_cast<const uint4*>(h + ((size_t)b * L + l) * 128 + (idx & 15) * 8)
                           : make_uint4(0u, 0u, 0u, 0u);
      }
    // chunk c (compile-time index after unrolling) -> hs
    auto stage_h = [&](const uint4 (&hc)[4]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = tid + 512 * i;
        *reinterpret_cast<uint4*>(hs + swz256(idx >> 4, idx & 15)) = hc[i];
      }
    };
    // logits, one h chunk at a time (wave w -> row tile w of the chunk)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int c0 = c * HC;
      if (c0 >= Bp) break;
      __syncthreads();                            // previous chunk consumed
      stage_h(hreg[c]);
      __syncthreads();
      const int rt = c0 / 32 + w;
      if (w < HC / 32 && rt < Bp / 32) {
        f32x16_t acc = zero16();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
          acc = mfma32(lds_frag(hs, swz256(w * 32 + r, kk * 2 + hh)), lds_frag(wos, swz256(r, kk * 2 + hh)), acc);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int b = rt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
          zs[b * 32 + r] = acc[i] + bov;
        }
      }
    }
    __syncthreads();
    // softmax over b for each v (16 partial columns per v)
    {
      const int v = tid & 31, part = tid >> 5;
      float m = -3.4e38f;
      if (v < V)
        for (int b = part; b < B; b += 16) m = fmaxf(m, zs[b * 32 + v]);
      red[part * 32 + v] = m;
      __syncthreads();
      if (tid < 32) {
        float mm = -3.4e38f;
        for (int k = 0; k < 16; ++k) mm = fmaxf(mm, red[k * 32 + tid]);
        colv[32 + tid] = mm;
      }
      __syncthreads();
      float sacc = 0.f;
      if (v < V)
        for (int b = part; b < B; b += 16) sacc += __expf(zs[b * 32 + v] - colv[32 + v]);
      red[part * 32 + v] = sacc;
      __syncthreads();
      if (tid < 32) {
        float ss = 0.f;
        for (int k = 0; k < 16; ++k) ss += red[k * 32 + tid];
        colv[64 + tid] = ss > 0.f ? 1.0f / ss : 0.f;
        colv[tid] = 0.f;
      }
      __syncthreads();
    }
    for (int i = tid; i < B * 32; i += 512) {
      const int v = i & 31;
      zs[i] = v < V ? __expf(zs[i] - colv[32 + v]) * colv[64 + v] : 0.f;
    }
    __syncthreads();
    // CE over v on the probabilities, one thread per sample: se_b = sum_v exp(P[b][v]) (P is a
    // probability in [0, 1]: no max shift needed), loss_b = log se_b - P[b][y_b]; the per-row scalars
    // (1/se_b, w_b/(BL), y_b) go to the free h staging tile.  G[b][v] = coef_b (exp(P)/se_b - [v==y_b]).
    float* rsv = reinterpret_cast<float*>(hs);                  // [Bp] 1/se_b
    float* cfv = rsv + Bp;                                      // [Bp] w_b / (B L)
    int* ybv = reinterpret_cast<int*>(cfv + Bp);                // [Bp] y_b
    for (int b = tid; b < B; b += 512) {
      const float* p = zs + b * 32;
      float se = 0.f;
#pragma unroll
      for (int v4 = 0; v4 < 8; ++v4) {
        const float4 q4 = *reinterpret_cast<const float4*>(p + 4 * v4);
        const float pv[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) se += (4 * v4 + e) < V ? __expf(pv[e]) : 0.f;
      }
      const int yv = (int)y[(size_t)b * L + l];
      const float wgt = wl[(size_t)b * L + l];
      lsum += wgt * (__logf(se) - p[yv]);
      rsv[b] = 1.0f / se;
      cfv[b] = wgt * inv_bl;
      ybv[b] = yv;
    }
    __syncthreads();
    // colv[v] = sum_b G[b][v] P[b][v]: thread (v, part) over rows part, part + 16, ...; 16 partial
    // columns combined in a fixed order
    const int cv_v = tid & 31, cv_part = tid >> 5;
    {
      float acc = 0.f;
      if (cv_v < V)
        for (int b = cv_part; b < B; b += 16) {
          const float pv = zs[b * 32 + cv_v];
          const float g = cfv[b] * (__expf(pv) * rsv[b] - (cv_v == ybv[b] ? 1.f : 0.f));
          acc += g * pv;
        }
      red[cv_part * 32 + cv_v] = acc;
      __syncthreads();
      if (tid < 32) {
        float t = 0.f;
        for (int k = 0; k < 16; ++k) t += red[k * 32 + tid];
        colv[tid] = t;
      }
      __syncthreads();
    }
    // dz = P (G - colv) -> bf16 dzb for the MFMAs (zero beyond B and V) and dbo_l[v] = sum_b dz
    {
      float acc = 0.f;
      const float cvv = colv[cv_v];
      for (int b = cv_part; b < Bp; b += 16) {
        float dz = 0.f;
        if (b < B && cv_v < V) {
          const float pv = zs[b * 32 + cv_v];
          const float g = cfv[b] * (__expf(pv) * rsv[b] - (cv_v == ybv[b] ? 1.f : 0.f));
          dz = pv * (g - cvv);
        }
        acc += dz;
        *reinterpret_cast<bf16_t*>(dzb + b * 64 + cv_v * 2) = f2bf(dz);
      }
      __syncthreads();                            // every colv / rsv read done before red is reused
      red[cv_part * 32 + cv_v] = acc;
      __syncthreads();
      if (tid < V) {
        float t = 0.f;
        for (int k = 0; k < 16; ++k) t += red[k * 32 + tid];
        dbo_acc += t;
      }
    }
    // dWo_l: wave w -> channel tile w & 3, row half w >> 2 of each chunk (the two halves summed
    // through LDS);  D[v][c] = sum_b dz^T[v][b] h[b][c]  (h chunks re-staged)
    {
      f32x16_t& acc = dwo_acc;
      const int colb = (w & 3) * 32 + tc;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        const int c0 = c * HC;
        if (c0 >= Bp) break;
        __syncthreads();
        stage_h(hreg[c]);
        __syncthreads();
        const int nkb = min(HC, Bp - c0) / 16;
        for (int kb = (w >> 2); kb < nkb; kb += 2) {
          const int ra = kb * 16 + 8 * hh + q;
          const bf16x8 fa =
              cat_tr(lds_tr(dzb, (c0 + ra) * 64 + tc * 2), lds_tr(dzb, (c0 + ra + 4) * 64 + tc * 2));
          const bf16x8 fb = cat_tr(lds_tr(hs, swz256e(ra, colb)), lds_tr(hs, swz256e(ra + 4, colb)));
          acc = mfma32(fa, fb, acc);
        }
      }
    }
    // dh: D[b][c] = sum_v dz[b][v] Wo[v][c]; per chunk: wave -> row tile, all 4 channel tiles, staged
    // in hs for 256-B row stores
    for (int c0 = 0; c0 < Bp; c0 += HC) {
      __syncthreads();                            // hs free (previous chunk stored / dWo done)
      const int rt = c0 / 32 + w;
      if (w < HC / 32 && rt < Bp / 32) {
      f32x16_t acc[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) acc[ct] = zero16();
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(dzb + (rt * 32 + r) * 64 + (kk * 16 + 8 * hh) * 2);
        const int rlo = kk * 16 + 8 * hh + q;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const int col = ct * 32 + tc;
          const bf16x8 fb = cat_tr(lds_tr(wos, swz256e(rlo, col)), lds_tr(wos, swz256e(rlo + 4, col)));
          acc[ct] = mfma32(fa, fb, acc[ct]);
        }
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int b = w * 32 + 8 * g + 4 * hh;    // chunk rows b .. b+3 (reg = 4g + e), column ct*32 + r
#pragma unroll
          for (int e = 0; e < 4; ++e)
            *reinterpret_cast<bf16_t*>(hs + swz256e(b + e, ct * 32 + r)) = f2bf(acc[ct][4 * g + e]);
        }
      }
      __syncthreads();
      for (int idx = tid; idx < HC * 16; idx += 512) {
        const int b = c0 + (idx >> 4), c8 = idx & 15;
        if (b < B)
          *reinterpret_cast<uint4*>(dh + ((size_t)b * L + l) * 128 + c8 * 8) =
              *reinterpret_cast<const uint4*>(hs + swz256(idx >> 4, c8));
      }
    }
  }  // positions
  // dWo: waves 4-7 hand their half to waves 0-3 through the (free) dh staging tile
  __syncthreads();
  float* xch = reinterpret_cast<float*>(hs);                  // [4 waves][16][64 lanes] fp32 = 16 KB
  if (w >= 4) {
#pragma unroll
    for (int i = 0; i < 16; ++i) xch[((w - 4) * 16 + i) * 64 + lane] = dwo_acc[i];
  }
  __syncthreads();
  if (w < 4) {
    float* dst = dwo_part + (size_t)blockIdx.x * V * 128;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int v = (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (v < V) dst[v * 128 + w * 32 + r] = dwo_acc[i] + xch[(w * 16 + i) * 64 + lane];
    }
  }
  if (tid < V) dbo_part[(size_t)blockIdx.x * V + tid] = dbo_acc;
  lsum = wave_reduce_sum(lsum);
  if (lane == 0) atomicAdd(loss, lsum * inv_bl);
}

// GO head: P = sigmoid(z), BCE(P, y) with PyTorch's log clamp (>= -100) and backward
// dz = w/(BA) (P - y) P(1-P) / max(P(1-P), 1e-12)   (BCELoss backward x sigmoid backward).
// z: [B, A] fp32 (GEMM output without bias); weights w[r * wsr + c * wsc] (wsc = 0: one per row)
__global__ void __launch_bounds__(256) go_head_kernel(const float* __restrict__ z, const float* __restrict__ bias,
                                                      const float* __restrict__ y, const float* __restrict__ wgt_p,
                                                      long wsr, long wsc, bf16_t* __restrict__ dz,
                                                      float* __restrict__ dbias, float* __restrict__ loss, int B,
                                                      int A, float inv_ba) {
  // thread owns column c for a run of rows (column bias gradient in registers)
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int rpb = (B + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rpb, r1 = min(B, r0 + rpb);
  float lsum = 0.f, dsum = 0.f;
  if (c < A) {
    const float bc = bias[c];
    for (int r = r0; r < r1; ++r) {
      const size_t i = (size_t)r * A + c;
      const float zz = z[i] + bc;
      const float p = 1.0f / (1.0f + __expf(-zz));
      const float yy = y[i];
      const float lp = fmaxf(__logf(p), -100.f), l1p = fmaxf(__logf(1.0f - p), -100.f);
      const float wgt = wgt_p[r * wsr + c * wsc];
      lsum += wgt * -(yy * lp + (1.0f - yy) * l1p);
      const float pq = p * (1.0f - p);
      const float g = wgt * inv_ba * (p - yy) * pq / fmaxf(pq, 1e-12f);
      dz[i] = f2bf(g);
      dsum += g;
    }
    atomicAdd(dbias + c, dsum);
  }
  __shared__ float red[8];
  lsum = block_reduce(lsum, red);
  if (threadIdx.x == 0) atomicAdd(loss, lsum * inv_ba);
}
}  // namespace

PBX_EXPORT int pbx_row_ln_fwd(const float* u, const float* bias, const float* res, const float* vpart, int TV,
                              const float* wp, int K, const float* gamma, const float* beta, float* out, void* out_bf,
                              float* xhat, float* rstd, float* vsum, int B, int G, float eps, hipStream_t st) {
  if (G > MAXG) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(row_ln_fwd_kernel, dim3(B), dim3(256), 0, st, u, bias, res, vpart, TV, wp, K, gamma, beta, out,
                     (bf16_t*)out_bf, xhat, rstd, vsum, G, eps);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_row_ln_bwd(const float* dout, const float* xhat, const float* rstd, const float* gamma,
                              const float* u, const float* bias, float* dgamma, float* dbeta, float* dbias, void* du,
                              float* dres, const float* vsum, const float* wp, int K, float* dwp, float* dvs, int B,
                              int G, hipStream_t st) {
  if (G > MAXG || (vsum != nullptr && K > 256)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(row_ln_bwd_kernel, dim3(B), dim3(256), 0, st, dout, xhat, rstd, gamma, u, bias, dgamma, dbeta,
                     dbias, (bf16_t*)du, dres, vsum, wp, K, dwp, dvs, G);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_bias_gelu(const float* u, const float* bias, float* out, void* out_bf, int M, int N,
                             hipStream_t st) {
  const int n = M * N;
  hipLaunchKernelGGL(bias_gelu_kernel, dim3((n + 255) / 256), dim3(256), 0, st, u, bias, out, (bf16_t*)out_bf, n, N);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_bias_gelu_bwd(const float* dout, const float* u, const float* bias, void* du, float* dbias, int M,
                                 int N, hipStream_t st) {
  const int gy = M < 32 ? M : 32;
  hipLaunchKernelGGL(bias_gelu_bwd_kernel, dim3((N + 255) / 256, gy), dim3(256), 0, st, dout, u, bias, (bf16_t*)du,
                     dbias, M, N);
  return pbx_launch_status();
}

// dwo_part: [P][V][128], dbo_part: [P][V] partial gradients (summed over P rows by the caller): with
// B <= 608 (MFMA form) P workgroups walk the positions (P <= L); the general form needs P == L
PBX_EXPORT int pbx_local_head2(const void* h, const float* wo, const float* bo, const void* y, const float* wl,
                               void* dh, float* dwo_part, float* dbo_part, float* loss, int B, int L, int V, int P,
                               hipStream_t st) {
  if (V > 32) return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)local_head_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    (void)hipFuncSetAttribute((const void*)local_head_mfma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              163840);
    attr = true;
  }
  const int Bp = (B + 31) & ~31;
  const int lds_m = 128 * 256 + 32 * 256 + Bp * 64 + Bp * 128 + (16 * 32 + 96) * 4;
  if (lds_m <= 163840) {
    if (P < 1 || P > L) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(local_head_mfma_kernel, dim3(P), dim3(512), lds_m, st, (const bf16_t*)h, wo, bo,
                       (const long long*)y, wl, (bf16_t*)dh, dwo_part, dbo_part, loss, B, L, V,
                       1.0f / ((float)B * (float)L));
    return pbx_launch_status();
  }
  const int lds = (V * 128 + B * V + 12 * V) * 4;
  if (lds > 163840 || P != L) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(local_head_kernel, dim3(L), dim3(256), lds, st, (const bf16_t*)h, wo, bo, (const long long*)y,
                     wl, (bf16_t*)dh, dwo_part, dbo_part, loss, B, L, V, 1.0f / ((float)B * (float)L));
  return pbx_launch_status();
}

PBX_EXPORT int pbx_local_head(const void* h, const float* wo, const float* bo, const void* y, const float* wl,
                              void* dh, float* dwo_part, float* dbo_part, float* loss, int B, int L, int V,
                              hipStream_t st) {
  return pbx_local_head2(h, wo, bo, y, wl, dh, dwo_part, dbo_part, loss, B, L, V, L, st);
}

PBX_EXPORT int pbx_go_head(const float* z, const float* bias, const float* y, const float* w, long wsr, long wsc,
                           void* dz, float* dbias, float* loss, int B, int A, hipStream_t st) {
  const int gy = B < 16 ? B : 16;
  hipLaunchKernelGGL(go_head_kernel, dim3((A + 255) / 256, gy), dim3(256), 0, st, z, bias, y, w, wsr, wsc,
                     (bf16_t*)dz, dbias, loss, B, A, 1.0f / ((float)B * (float)A));
  return pbx_launch_status();
}


// dst[c] += scale * sum_r src[r][c]   (scale: optional device scalar).  A block covers 32 columns with
// 8 row-lanes (row r -> lane r % 8), the 8 partials are combined in LDS in fixed order
// (deterministic); used to fold per-position partial gradients into the arena.
__global__ void __launch_bounds__(256) colsum_add_kernel(const float* __restrict__ src, int rows, int cols,
                                                         float* __restrict__ dst, const float* __restrict__ scale) {
  __shared__ float part[8][33];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float a0 = 0.f, a1 = 0.f;
  if (c < cols) {
    int r = rl;
    for (; r + 8 < rows; r += 16) {
      a0 += src[(size_t)r * cols + c];
      a1 += src[(size_t)(r + 8) * cols + c];
    }
    for (; r < rows; r += 8) a0 += src[(size_t)r * cols + c];
  }
  part[rl][cl] = a0 + a1;
  __syncthreads();
  if (rl == 0 && c < cols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += part[k][cl];
    dst[c] += scale != nullptr ? s * scale[0] : s;
  }
}

PBX_EXPORT int pbx_colsum_add(const float* src, int rows, int cols, float* dst, const float* scale, hipStream_t st) {
  if (cols <= 0 || rows <= 0) return 0;
  hipLaunchKernelGGL(colsum_add_kernel, dim3((cols + 31) / 32), dim3(256), 0, st, src, rows, cols, dst, scale);
  return pbx_launch_status();
}
