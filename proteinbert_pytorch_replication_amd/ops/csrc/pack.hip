// All per-step weight images in ONE launch.
//
// The fused kernels read bf16 weights in MFMA-fragment-native layouts (conv2.hip: the dual
// dilated convs' A fragments for the forward and the data gradient; glob2.hip: the global-track
// Linear weights' B fragments for X W^T and dU W).  The fp32 masters change every optimizer step,
// so the images are rebuilt once per forward: one 2-D launch over every matrix of the model
// (grid.y = matrix) instead of ~30 small launches of ~5 us each.
#include "common.h"

namespace {
typedef unsigned short bf16_t;
constexpr int MAXM = 40;
constexpr int CH = 128;

struct PackBatch {
  const float* w[MAXM];
  bf16_t* o1[MAXM];
  bf16_t* o2[MAXM];
  int n[MAXM];        // rows N (glob) / kernel taps KS (conv)
  int k[MAXM];        // columns K (glob) / 0 (conv)
  int kind[MAXM];     // 0: conv [128][128][KS] -> fwd/dgrad A fragments; 1: Linear [N][K] -> fwd/bwd B fragments
};

__global__ void __launch_bounds__(256) pack_batch_kernel(PackBatch pb) {
  const int m = blockIdx.y;
  const float* __restrict__ w = pb.w[m];
  bf16_t* __restrict__ o1 = pb.o1[m];
  bf16_t* __restrict__ o2 = pb.o2[m];
  if (pb.kind[m] == 0) {
    const int KS = pb.n[m];
    const int total = KS * CH * CH;
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
      // [k][kb][mb][lane][8]: M = 32 mb + (lane & 31), K = 16 kb + 8 (lane >> 5) + j  (conv2.hip)
      const int j = idx & 7, lane = (idx >> 3) & 63, fi = idx >> 9;
      const int mb = fi & 3, kb = (fi >> 2) & 7, kk = fi >> 5;
      const int mm = mb * 32 + (lane & 31), ki = kb * 16 + 8 * (lane >> 5) + j;
      o1[idx] = f2bf(w[((size_t)mm * CH + ki) * KS + kk]);     // forward: M = co, K = ci
      o2[idx] = f2bf(w[((size_t)ki * CH + mm) * KS + kk]);     // dgrad:   M = ci, K = co
    }
  } else {
    const int N = pb.n[m], K = pb.k[m];
    const int total = N * K;
    for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
      // [tile][step][lane][8]  (glob2.hip pack_glob_frags_kernel)
      const int j = idx & 7, l = (idx >> 3) & 63, f = idx >> 9;
      {
        const int S = K / 32, t = f / S, s = f % S;
        o1[idx] = f2bf(w[(size_t)(t * 16 + (l & 15)) * K + s * 32 + 8 * (l >> 4) + j]);
      }
      {
        const int S = N / 32, t = f / S, s = f % S;
        o2[idx] = f2bf(w[(size_t)(s * 32 + 8 * (l >> 4) + j) * K + t * 16 + (l & 15)]);
      }
    }
  }
}
}  // namespace

// ptrs: 3 * count pointers (w, out1, out2 per matrix); meta: 3 * count ints (n, k, kind)
PBX_EXPORT int pbx_pack_batch(const void* const* ptrs, const int* meta, int count, hipStream_t st) {
  if (count < 1 || count > MAXM) return (int)hipErrorInvalidValue;
  PackBatch pb;
  int maxel = 0;
  for (int i = 0; i < count; ++i) {
    pb.w[i] = (const float*)ptrs[3 * i];
    pb.o1[i] = (bf16_t*)ptrs[3 * i + 1];
    pb.o2[i] = (bf16_t*)ptrs[3 * i + 2];
    pb.n[i] = meta[3 * i];
    pb.k[i] = meta[3 * i + 1];
    pb.kind[i] = meta[3 * i + 2];
    const int el = pb.kind[i] == 0 ? pb.n[i] * CH * CH : pb.n[i] * pb.k[i];
    if (pb.kind[i] == 1 && (pb.n[i] % 32 || pb.k[i] % 32)) return (int)hipErrorInvalidValue;
    maxel = el > maxel ? el : maxel;
  }
  const int gx = (maxel + 256 * 4 - 1) / (256 * 4);   // 4 elements per thread
  hipLaunchKernelGGL(pack_batch_kernel, dim3(gx, count), dim3(256), 0, st, pb);
  return pbx_launch_status();
}

// An empty one-wave kernel: the graph-capture ordering marker of ops/streams.py (a main-stream node
// captured between a fork point and the aux-stream body, so the main chain stays the fork point's
// first child and hipGraph's stream assignment keeps it on one queue).
__global__ void __launch_bounds__(64) noop_kernel() {}

PBX_EXPORT int pbx_noop(hipStream_t st) {
  hipLaunchKernelGGL(noop_kernel, dim3(1), dim3(64), 0, st);
  return pbx_launch_status();
}
