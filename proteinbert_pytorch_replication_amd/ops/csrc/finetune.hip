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
}  // namespace

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
