// Per-residue fine-tuning head weight gradient (BASELINE cfg 5: frozen encoder + token classifier).
//
//   dW[k][c] = sum_rows g[row][k] h[row][c]        h: [M, 128] bf16 (encoder output), g: [M, K] fp32
//
// M = B * L = 262,144 rows and K = 8 classes: a hipBLASLt GEMM with the 262,144-long reduction axis
// ran 230 us (bf16) / 410 us (fp32) per step, a third of the whole fine-tune step; this kernel streams
// h once (64 MB) with fp32 accumulation.  Workgroup = 16 row lanes x 16 channel chunks of 8; each
// thread keeps its [KT][8] partial in registers over the workgroup's rows, the 4 row lanes of a wave
// are summed by shuffles and the 4 waves through LDS; every workgroup writes one partial row of a
// [P][K * 128] slab that pbx_colsum_add folds (deterministic, no atomics).
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;

template <int KT>
__global__ void __launch_bounds__(256) token_head_wgrad_kernel(const bf16_t* __restrict__ h,
                                                               const float* __restrict__ g, float* __restrict__ slab,
                                                               long M, int K) {
  __shared__ float red[4][KT * CH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rl = tid >> 4, cc = tid & 15;
  float acc[KT][8];
#pragma unroll
  for (int k = 0; k < KT; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
  for (long row = (long)blockIdx.x * 16 + rl; row < M; row += (long)gridDim.x * 16) {
    const uint4 q = *reinterpret_cast<const uint4*>(h + row * CH + cc * 8);
    float hv[8];
    unpack8(q, hv);
    float gv[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) gv[k] = k < K ? g[row * K + k] : 0.f;
#pragma unroll
    for (int k = 0; k < KT; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[k][e] = fmaf(gv[k], hv[e], acc[k][e]);
  }
  // lanes l, l^16, l^32, l^48 of a wave share the channel chunk
#pragma unroll
  for (int k = 0; k < KT; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      acc[k][e] += __shfl_xor(acc[k][e], 16, 64);
      acc[k][e] += __shfl_xor(acc[k][e], 32, 64);
    }
  if (lane < 16) {
#pragma unroll
    for (int k = 0; k < KT; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[w][k * CH + cc * 8 + e] = acc[k][e];
  }
  __syncthreads();
  float* dst = slab + (size_t)blockIdx.x * K * CH;
  for (int i = tid; i < K * CH; i += 256) dst[i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}
// Token-head logits (reference finetuning head, nn.Linear(128, K) on every residue):
//   out[m][k] = b[k] + sum_c h[m][c] W[k][c]
// A workgroup stages 256 rows (64 KiB) into LDS with coalesced 16-B loads (swz256 rows, so the
// row-per-thread reads below are conflict-free), then each thread owns one row: fp32 FMAs over the
// exact bf16 inputs and the fp32 weights (broadcast from LDS).  The library path needed two bf16 GEMMs
// on a hi / lo weight split for the same accuracy.
template <int K>
__global__ void __launch_bounds__(256) token_head_fwd_kernel(const bf16_t* __restrict__ h, const float* __restrict__ W,
                                                             const float* __restrict__ b, float* __restrict__ out,
                                                             long M) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];   // 256 rows x 256 B
  __shared__ float ws[K * CH];
  for (int i = threadIdx.x; i < K * CH; i += 256) ws[i] = W[i];
  const long m0 = (long)blockIdx.x * 256;
  const int n = (int)min((long)256, M - m0);
  stage_chunks(
      256 * 16,
      [&](int idx) {
        return (idx >> 4) < n ? *reinterpret_cast<const uint4*>(h + (m0 + (idx >> 4)) * CH + (idx & 15) * 8)
                              : make_uint4(0u, 0u, 0u, 0u);
      },
      [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(smem + swz256(idx >> 4, idx & 15)) = v; });
  __syncthreads();
  const int row = threadIdx.x;
  if (row >= n) return;
  float acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = b[k];
#pragma unroll 4
  for (int c = 0; c < 16; ++c) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(smem + swz256(row, c)), v);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float* wr = ws + k * CH + c * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[k] = fmaf(v[e], wr[e], acc[k]);
    }
  }
  float* o = out + (m0 + row) * K;
#pragma unroll
  for (int k = 0; k < K; ++k) o[k] = acc[k];
}

template <int K>
int token_head_fwd_launch(const void* h, const float* W, const float* b, float* out, long M, hipStream_t st) {
  static bool attr = false;                  // 64 KiB dynamic + the static weight copy exceed the default
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)token_head_fwd_kernel<K>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              256 * 256);
    attr = true;
  }
  hipLaunchKernelGGL(token_head_fwd_kernel<K>, dim3((unsigned)((M + 255) / 256)), dim3(256), 256 * 256, st,
                     (const bf16_t*)h, W, b, out, M);
  return pbx_launch_status();
}
}  // namespace

// out [M][K] fp32 = h [M][128] bf16 . W^T ([K][128] fp32) + b (K <= 16)
PBX_EXPORT int pbx_token_head_fwd(const void* h, const float* W, const float* b, float* out, long M, int K,
                                  hipStream_t st) {
  if (M < 1) return (int)hipErrorInvalidValue;
  switch (K) {
    case 1: return token_head_fwd_launch<1>(h, W, b, out, M, st);
    case 2: return token_head_fwd_launch<2>(h, W, b, out, M, st);
    case 3: return token_head_fwd_launch<3>(h, W, b, out, M, st);
    case 4: return token_head_fwd_launch<4>(h, W, b, out, M, st);
    case 5: return token_head_fwd_launch<5>(h, W, b, out, M, st);
    case 6: return token_head_fwd_launch<6>(h, W, b, out, M, st);
    case 7: return token_head_fwd_launch<7>(h, W, b, out, M, st);
    case 8: return token_head_fwd_launch<8>(h, W, b, out, M, st);
    case 9: return token_head_fwd_launch<9>(h, W, b, out, M, st);
    case 10: return token_head_fwd_launch<10>(h, W, b, out, M, st);
    case 11: return token_head_fwd_launch<11>(h, W, b, out, M, st);
    case 12: return token_head_fwd_launch<12>(h, W, b, out, M, st);
    case 13: return token_head_fwd_launch<13>(h, W, b, out, M, st);
    case 14: return token_head_fwd_launch<14>(h, W, b, out, M, st);
    case 15: return token_head_fwd_launch<15>(h, W, b, out, M, st);
    case 16: return token_head_fwd_launch<16>(h, W, b, out, M, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// slab: [P][K][128] fp32 partials (P = number of workgroups, chosen by the caller); K <= 16
PBX_EXPORT int pbx_token_head_wgrad(const void* h, const float* g, float* slab, long M, int K, int P,
                                    hipStream_t st) {
  if (K < 1 || K > 16 || P < 1) return (int)hipErrorInvalidValue;
  if (K <= 8)
    hipLaunchKernelGGL(token_head_wgrad_kernel<8>, dim3(P), dim3(256), 0, st, (const bf16_t*)h, g, slab, M, K);
  else
    hipLaunchKernelGGL(token_head_wgrad_kernel<16>, dim3(P), dim3(256), 0, st, (const bf16_t*)h, g, slab, M, K);
  return pbx_launch_status();
}
