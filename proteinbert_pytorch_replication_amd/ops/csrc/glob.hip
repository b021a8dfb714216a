// Global (per-protein) track, pretraining heads and losses.
//
// Reference: ProteinBERT/modules.py:175-199,221-229 (two Linear G->G + GELU + residual + LayerNorm(G)
// per block), :21-92 (attention output scaled by sum(W)/K in reference semantics), :277-293 (local
// head Linear C->V + nn.Softmax() over the BATCH axis, GO head Linear G->A + Sigmoid) and
// ProteinBERT/utils.py:293-294 (CE applied to the local probabilities, BCE with log clamp -100,
// weighted means over B*L and B*A).
//
// General-shape path (global dims the one-launch kernels of glob2/glob3.hip are not built for): the [B, G]
// GEMMs run on the in-tree MFMA GEMM (csrc/gemm.hip, bf16 in, fp32 out); everything around them is fused here:
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
                                                            float* __restrict__ dbias, int M, int N,
                                                            float* __restrict__ slab) {
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
  if (slab != nullptr) slab[(size_t)blockIdx.y * N + c] = acc;    // deterministic: folded by the caller
  else atomicAdd(dbias + c, acc);
}

}  // namespace

extern "C" int pbx_colsum_add(const float* src, int rows, int cols, float* dst, const float* scale, hipStream_t st);

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

// slab (nullable): [min(M, 256)][N] fp32 -> the bias gradient is folded in a fixed order (deterministic)
PBX_EXPORT int pbx_bias_gelu_bwd(const float* dout, const float* u, const float* bias, void* du, float* dbias, int M,
                                 int N, float* slab, hipStream_t st) {
  const int gy = M < 256 ? M : 256;      // (ops/global_track.py BGB_ROWS)
  hipLaunchKernelGGL(bias_gelu_bwd_kernel, dim3((N + 255) / 256, gy), dim3(256), 0, st, dout, u, bias, (bf16_t*)du,
                     dbias, M, N, slab);
  if (slab != nullptr) {
    const int rc = pbx_launch_status();
    if (rc != 0) return rc;
    return pbx_colsum_add(slab, gy, N, dbias, nullptr, st);
  }
  return pbx_launch_status();
}

// dst[c] += scale * sum_r src[r][c]   (scale: optional device scalar).  A block covers 32 columns with
// 8 row-lanes (row r -> lane r % 8), the 8 partials are combined in LDS in fixed order
// (deterministic); used to fold per-position partial gradients into the arena.
template <bool SET>
__global__ void __launch_bounds__(256) colsum_add_kernel(const float* __restrict__ src, int rows, int cols, int ld,
                                                         float* __restrict__ dst, const float* __restrict__ scale) {
  __shared__ float part[8][33];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float a0 = 0.f, a1 = 0.f;
  if (c < cols) {
    int r = rl;
    for (; r + 8 < rows; r += 16) {
      a0 += src[(size_t)r * ld + c];
      a1 += src[(size_t)(r + 8) * ld + c];
    }
    for (; r < rows; r += 8) a0 += src[(size_t)r * ld + c];
  }
  part[rl][cl] = a0 + a1;
  __syncthreads();
  if (rl == 0 && c < cols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += part[k][cl];
    const float v = scale != nullptr ? s * scale[0] : s;
    if constexpr (SET) dst[c] = v;
    else dst[c] += v;
  }
}

// The same fold over 4 adjacent columns per thread (16-B loads, 128 columns per workgroup) with 8 rows in
// flight per thread; per column the additions are exactly colsum_add_kernel's (a0: rows rl + 16 i, a1: rows
// rl + 8 + 16 i, then the 8 row-lane partials in order), so the two give bitwise-equal results.
__device__ __forceinline__ void add4(float4& a, const float4& v) { a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w; }

// this thread's partial (row lane rl of 8) of column quad c, in colsum_add_kernel's order
__device__ __forceinline__ float4 fold4_partial(const float4* __restrict__ src, int rows, int cols4, int c, int rl) {
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
  int r = rl;
  for (; r + 56 < rows; r += 64) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(r + 8 * u) * cols4 + c];
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      add4(a0, v[u]);
      add4(a1, v[u + 1]);
    }
  }
  for (; r + 8 < rows; r += 16) {
    add4(a0, src[(size_t)r * cols4 + c]);
    add4(a1, src[(size_t)(r + 8) * cols4 + c]);
  }
  for (; r < rows; r += 8) add4(a0, src[(size_t)r * cols4 + c]);
  return make_float4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w);
}

template <bool SET>
__global__ void __launch_bounds__(256) colsum_add4_kernel(const float4* __restrict__ src, int rows, int cols4,
                                                          float4* __restrict__ dst, const float* __restrict__ scale) {
  __shared__ float4 part[8][32];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  part[rl][cl] = c < cols4 ? fold4_partial(src, rows, cols4, c, rl) : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (rl == 0 && c < cols4) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 8; ++k) add4(s, part[k][cl]);
    if (scale != nullptr) {
      const float f = scale[0];
      s = make_float4(s.x * f, s.y * f, s.z * f, s.w * f);
    }
    if constexpr (SET) {
      dst[c] = s;
    } else {
      float4 d = dst[c];
      add4(d, s);
      dst[c] = d;
    }
  }
}

template <bool SET>
int colsum_launch(const float* src, int rows, int cols, float* dst, const float* scale, hipStream_t st) {
  if ((cols & 3) == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
    const int cols4 = cols >> 2;
    hipLaunchKernelGGL(colsum_add4_kernel<SET>, dim3((cols4 + 31) / 32), dim3(256), 0, st, (const float4*)src, rows,
                       cols4, (float4*)dst, scale);
  } else {
    hipLaunchKernelGGL(colsum_add_kernel<SET>, dim3((cols + 31) / 32), dim3(256), 0, st, src, rows, cols, cols, dst,
                       scale);
  }
  return pbx_launch_status();
}

PBX_EXPORT int pbx_colsum_add(const float* src, int rows, int cols, float* dst, const float* scale, hipStream_t st) {
  if (cols <= 0 || rows <= 0) return 0;
  return colsum_launch<false>(src, rows, cols, dst, scale, st);
}

// dst[c] = scale * sum_r src[r][c] (no zero-fill of dst needed: the loss slots of the fused heads)
PBX_EXPORT int pbx_colsum_set(const float* src, int rows, int cols, float* dst, const float* scale, hipStream_t st) {
  if (cols <= 0 || rows <= 0) return (int)hipErrorInvalidValue;
  return colsum_launch<true>(src, rows, cols, dst, scale, st);
}

// dst[g][c] = sum_r src[g][r][c] over r = 0 .. R-1 in order (one thread per (g, c); loads coalesced over c):
// the per-group partial folds of paper semantics (dgb over position tiles, dq over split-L chunks)
__global__ void __launch_bounds__(256) group_colsum_kernel(const float* __restrict__ src, int G, int R, int C,
                                                           float* __restrict__ dst) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)G * C) return;
  const long g = i / C;
  const int c = (int)(i - g * C);
  const float* p = src + (size_t)g * R * C + c;
  float a = 0.f;
  for (int r = 0; r < R; ++r) a += p[(size_t)r * C];
  dst[i] = a;
}

PBX_EXPORT int pbx_group_colsum(const float* src, int G, int R, int C, float* dst, hipStream_t st) {
  if (G < 1 || R < 1 || C < 1) return (int)hipErrorInvalidValue;
  const long n = (long)G * C;
  hipLaunchKernelGGL(group_colsum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, G, R, C, dst);
  return pbx_launch_status();
}

// two folds with the same row count in one launch (a weight slab and its bias slab): blocks < ceil(cols0 / 32)
// fold (src0, cols0) into dst0, the rest (src1, cols1) into dst1; same fixed order as colsum_add_kernel
__global__ void __launch_bounds__(256) colsum_add2_kernel(const float* __restrict__ src0, int cols0,
                                                          float* __restrict__ dst0, const float* __restrict__ src1,
                                                          int cols1, float* __restrict__ dst1, int rows) {
  __shared__ float part[8][33];
  const int nb0 = (cols0 + 31) / 32;
  const bool second = (int)blockIdx.x >= nb0;
  const float* src = second ? src1 : src0;
  float* dst = second ? dst1 : dst0;
  const int cols = second ? cols1 : cols0;
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = ((int)blockIdx.x - (second ? nb0 : 0)) * 32 + cl;
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
    dst[c] += s;
  }
}

PBX_EXPORT int pbx_colsum_add2(const float* src0, int cols0, float* dst0, const float* src1, int cols1, float* dst1,
                               int rows, hipStream_t st) {
  if (cols0 <= 0 || cols1 <= 0 || rows <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(colsum_add2_kernel, dim3((cols0 + 31) / 32 + (cols1 + 31) / 32), dim3(256), 0, st, src0, cols0,
                     dst0, src1, cols1, dst1, rows);
  return pbx_launch_status();
}

// the same over column block [0, cols) of rows `ld` floats apart
PBX_EXPORT int pbx_colsum_add_ld(const float* src, int rows, int cols, int ld, float* dst, const float* scale,
                                 hipStream_t st) {
  if (cols <= 0 || rows <= 0 || ld < cols) return cols <= 0 || rows <= 0 ? 0 : (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(colsum_add_kernel<false>, dim3((cols + 31) / 32), dim3(256), 0, st, src, rows, cols, ld, dst, scale);
  return pbx_launch_status();
}
