// On-device synthetic batch generation and pretraining corruption.
//
// Reference semantics (ProteinBERT/data_processing.py:86-180, dummy_tests.py:23-38), applied to a
// whole padded batch in two launches instead of per-sample Python:
//   tokens : <sos> aa... <eos>, random crop start ~ U[0, n+2-L) (exclusive, reference quirk), <pad>
//   token corruption : Bernoulli(p) on ids > <eos>, replacement U{3..V-1}
//   annotation corruption : blank row with prob blank_p, else (ann + Bern(neg)) * Bern(1 - pos)
//   weights : w_local = (token != <pad>), w_global[b] = any(ann[b, :])
// RNG is counter-based (seed, stream, element) so a step is reproducible and graph-replayable.
#include "common.h"

namespace {
constexpr int PAD = 0, SOS = 1, EOS = 2;

enum Stream : unsigned long long {
  S_LEN = 1, S_CROP = 2, S_AA = 3, S_ANN = 4, S_TOKMASK = 5, S_TOKRND = 6, S_BLANK = 7, S_KEEP = 8, S_ADD = 9
};

__device__ __forceinline__ unsigned long long stream_id(unsigned long long step, Stream s) {
  return step * 16ull + (unsigned long long)s;
}
}  // namespace

// grid: (B), block 256. tokens int64 [B, L]; ann f32 [B, A]
__global__ void __launch_bounds__(256) synth_batch_kernel(long long* __restrict__ tokens, float* __restrict__ ann,
                                                          int L, int A, int min_len, int max_len, float density,
                                                          int vocab, unsigned long long seed,
                                                          unsigned long long step,
                                                          const long long* __restrict__ step_dev) {
  if (step_dev != nullptr) step += (unsigned long long)*step_dev;
  const int b = blockIdx.x;
  const float u_len = pbx_uniform(seed, stream_id(step, S_LEN), b);
  const int n = min_len + min((int)(u_len * (float)(max_len - min_len + 1)), max_len - min_len);
  const int total = n + 2;
  int start = 0;
  if (total > L) {
    const float u = pbx_uniform(seed, stream_id(step, S_CROP), b);
    start = min((int)(u * (float)(total - L)), total - L - 1);
  }
  const int n_aa = vocab - 4;
  for (int j = threadIdx.x; j < L; j += blockDim.x) {
    const int s = start + j;
    int t;
    if (s == 0) t = SOS;
    else if (s == total - 1) t = EOS;
    else if (s >= total) t = PAD;
    else {
      const float u = pbx_uniform(seed, stream_id(step, S_AA), (unsigned long long)b * L + j);
      t = 4 + min((int)(u * (float)n_aa), n_aa - 1);
    }
    tokens[(long long)b * L + j] = t;
  }
  for (int a = threadIdx.x; a < A; a += blockDim.x) {
    const float u = pbx_uniform(seed, stream_id(step, S_ANN), (unsigned long long)b * A + a);
    ann[(long long)b * A + a] = u < density ? 1.0f : 0.0f;
  }
}

// grid: (B), block 256.
__global__ void __launch_bounds__(256) corrupt_batch_kernel(const long long* __restrict__ tokens,
                                                            const float* __restrict__ ann,
                                                            long long* __restrict__ x_local,
                                                            float* __restrict__ x_global,
                                                            float* __restrict__ w_local,
                                                            float* __restrict__ w_sample,
                                                            int L, int A, int vocab, float token_p,
                                                            float positive_p, float negative_p, float blank_p,
                                                            unsigned long long seed, unsigned long long step,
                                                            const long long* __restrict__ step_dev) {
  if (step_dev != nullptr) step += (unsigned long long)*step_dev;
  __shared__ int any_s[4];
  const int b = blockIdx.x;
  for (int j = threadIdx.x; j < L; j += blockDim.x) {
    const long long idx = (long long)b * L + j;
    const long long t = tokens[idx];
    long long x = t;
    if (t > EOS) {
      const float u = pbx_uniform(seed, stream_id(step, S_TOKMASK), idx);
      if (u < token_p) {
        const float r = pbx_uniform(seed, stream_id(step, S_TOKRND), idx);
        x = 3 + min((int)(r * (float)(vocab - 3)), vocab - 4);
      }
    }
    x_local[idx] = x;
    w_local[idx] = t != PAD ? 1.0f : 0.0f;
  }
  const bool blank = pbx_uniform(seed, stream_id(step, S_BLANK), b) <= blank_p;
  int any = 0;
  for (int a = threadIdx.x; a < A; a += blockDim.x) {
    const long long idx = (long long)b * A + a;
    const float v = ann[idx];
    any |= (v != 0.0f);
    float out = 0.0f;
    if (!blank) {
      const float keep = pbx_uniform(seed, stream_id(step, S_KEEP), idx) >= positive_p ? 1.0f : 0.0f;
      const float add = pbx_uniform(seed, stream_id(step, S_ADD), idx) < negative_p ? 1.0f : 0.0f;
      out = (v + add) * keep;
    }
    x_global[idx] = out;
  }
  // block-wide any()
  unsigned long long bal = __ballot(any);
  if ((threadIdx.x & 63) == 0) any_s[threadIdx.x >> 6] = bal != 0ull;
  __syncthreads();
  if (threadIdx.x == 0) w_sample[b] = (any_s[0] | any_s[1] | any_s[2] | any_s[3]) ? 1.0f : 0.0f;
}

// step_dev (optional, device int64): added to `step`, so a captured launch draws new data per replay
PBX_EXPORT int pbx_synth_batch(void* tokens, void* ann, int B, int L, int A, int min_len, int max_len,
                               float density, int vocab, unsigned long long seed, unsigned long long step,
                               const void* step_dev, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(synth_batch_kernel, dim3(B), dim3(256), 0, stream, (long long*)tokens, (float*)ann, L, A,
                     min_len, max_len, density, vocab, seed, step, (const long long*)step_dev);
  return pbx_launch_status();
}

PBX_EXPORT int pbx_corrupt_batch(const void* tokens, const void* ann, void* x_local, void* x_global,
                                 void* w_local, void* w_sample, int B, int L, int A, int vocab, float token_p,
                                 float positive_p, float negative_p, float blank_p, unsigned long long seed,
                                 unsigned long long step, const void* step_dev, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(corrupt_batch_kernel, dim3(B), dim3(256), 0, stream, (const long long*)tokens,
                     (const float*)ann, (long long*)x_local, (float*)x_global, (float*)w_local,
                     (float*)w_sample, L, A, vocab, token_p, positive_p, negative_p, blank_p, seed, step,
                     (const long long*)step_dev);
  return pbx_launch_status();
}

// ---- expansion of a compact host batch (ops/csrc/pbx_loader.cpp) -----------------------------
// tokens_u8 [B, L] -> int64 [B, L]; bits [B, nbytes] (little-endian per byte) -> f32 [B, A].
// grid (B), block 256; each thread expands one byte (8 annotations) per iteration.
__global__ void __launch_bounds__(256) unpack_batch_kernel(const unsigned char* __restrict__ tok_u8,
                                                           const unsigned char* __restrict__ bits,
                                                           long long* __restrict__ tokens,
                                                           float* __restrict__ ann, int L, int A, int nbytes) {
  const int b = blockIdx.x;
  const unsigned char* tb = tok_u8 + (size_t)b * L;
  long long* to = tokens + (size_t)b * L;
  for (int j = threadIdx.x; j < L; j += blockDim.x) to[j] = (long long)tb[j];
  const unsigned char* bb = bits + (size_t)b * nbytes;
  float* ao = ann + (size_t)b * A;
  for (int k = threadIdx.x; k < nbytes; k += blockDim.x) {
    const unsigned v = bb[k];
    const int a0 = k * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (a0 + i < A) ao[a0 + i] = (float)((v >> i) & 1u);
  }
}

PBX_EXPORT int pbx_unpack_batch(const void* tok_u8, const void* bits, void* tokens, void* ann, int B, int L, int A,
                                int nbytes, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(unpack_batch_kernel, dim3(B), dim3(256), 0, stream, (const unsigned char*)tok_u8,
                     (const unsigned char*)bits, (long long*)tokens, (float*)ann, L, A, nbytes);
  return pbx_launch_status();
}
