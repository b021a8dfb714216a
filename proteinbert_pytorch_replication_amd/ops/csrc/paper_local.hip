// Paper-semantics local track: per-position LayerNorm over the channels (published ProteinBERT;
// the reference's LayerNorm((L, C)) normalises the whole sequence, SURVEY A.2 Q5, and lives in ln.hip).
//
//   h1 = LN_C(s1; g1, b1) ; pre = h1 Wl^T + bl ; s2 = h1 + GELU(pre) ; h2 = LN_C(s2; g2, b2)
//
// (reference ProteinBERT/modules.py:148-164,212-217 with LayerNorm(C) instead of LayerNorm((L, C))).
// Rows are independent, so statistics never leave the workgroup: a work item is 32 positions of one
// sequence (the last tile of a sequence is masked), thread t of 512 owns row j = t >> 4 and channel
// chunk ch = t & 15, per-row sums are 16-lane shuffles, and the [C]-shaped affine gradients
// accumulate in registers for every row the workgroup visits.  The 128x128 GEMMs run on
// v_mfma_f32_32x32x16_bf16 through swz256 LDS tiles (mfma.h), as in ln.hip.
//
// Forward writes h2 (bf16) and per-row (mean1, rstd1, mean2, rstd2); the backward recomputes h1, the
// MLP pre-activation and s2 from s1 (one extra 32-MFMA GEMM per tile instead of storing two more
// [B, L, 128] activations) and produces ds1 (the conv-track gradient), per-(sample, tile) partial sums
// of ds1 (gradient of the broadcast global->local vector) and every parameter gradient.
#include "mfma.h"

using namespace pbx;
typedef unsigned short bf16_t;

namespace {
constexpr int CH = 128;
constexpr int TR = 32;        // rows (positions) per work item
constexpr int YS = CH + 4;    // padded row stride of the fp32 D^T tile

__device__ __forceinline__ void ld8f(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 c = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
}
__device__ __forceinline__ uint4 ldq(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u);
}
// sum over the 16 lanes of one row (lanes 16k .. 16k+15 of the wave)
__device__ __forceinline__ float row_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}
__device__ __forceinline__ void row_sum2(float& a, float& b) {
#pragma unroll
  for (int m = 1; m <= 8; m <<= 1) {
    a += __shfl_xor(a, m, 64);
    b += __shfl_xor(b, m, 64);
  }
}

// GELU and GELU' of 8 values sharing one erf/exp evaluation (common.h gelu_core2 arithmetic)
__device__ __forceinline__ void gelu_both8(const float* x, float* gv, float* gdv) {
  f32x2 xi[4], ax[4], t[4], e[4], pl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xi[i] = (f32x2){x[2 * i], x[2 * i + 1]};
    ax[i] = __builtin_elementwise_abs(xi[i]);
    t[i] = __builtin_elementwise_fma(ax[i], (f32x2){0.23164190f, 0.23164190f}, (f32x2){1.0f, 1.0f});
    e[i] = (xi[i] * -0.72134752044448170f) * xi[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    t[i] = (f32x2){__builtin_amdgcn_rcpf(t[i].x), __builtin_amdgcn_rcpf(t[i].y)};
    e[i] = (f32x2){__builtin_amdgcn_exp2f(e[i].x), __builtin_amdgcn_exp2f(e[i].y)};
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pl[i] = __builtin_elementwise_fma(t[i], (f32x2){-0.5307027145f, -0.5307027145f},
                                      (f32x2){0.7265760135f, 0.7265760135f});
    pl[i] = __builtin_elementwise_fma(t[i], pl[i], (f32x2){-0.7107068705f, -0.7107068705f});
    pl[i] = __builtin_elementwise_fma(t[i], pl[i], (f32x2){0.142248368f, 0.142248368f});
    pl[i] = __builtin_elementwise_fma(t[i], pl[i], (f32x2){-0.127414796f, -0.127414796f});
    pl[i] = __builtin_elementwise_fma(pl[i] * t[i], e[i], (f32x2){0.5f, 0.5f});   // h = 0.5 erf(|x|/sqrt2)
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 g = __builtin_elementwise_fma(ax[i], pl[i], xi[i] * 0.5f);
    const f32x2 sh = {copysignf(pl[i].x, xi[i].x), copysignf(pl[i].y, xi[i].y)};
    const f32x2 gd = __builtin_elementwise_fma(xi[i] * 0.3989422804014327f, e[i], sh + 0.5f);
    gv[2 * i] = g.x; gv[2 * i + 1] = g.y;
    gdv[2 * i] = gd.x; gdv[2 * i + 1] = gd.y;
  }
}
__device__ __forceinline__ void gelu8(const float* x, float* gv) {
  const f32x2 xi[4] = {(f32x2){x[0], x[1]}, (f32x2){x[2], x[3]}, (f32x2){x[4], x[5]}, (f32x2){x[6], x[7]}};
  f32x2 go[4];
  gelu2_fast_n<4, false>(xi, go);
#pragma unroll
  for (int i = 0; i < 4; ++i) { gv[2 * i] = go[i].x; gv[2 * i + 1] = go[i].y; }
}

__device__ __forceinline__ void stage_wl(unsigned char* dst, const bf16_t* __restrict__ w) {
  stage_chunks(
      CH * 16, [&](int idx) { return *reinterpret_cast<const uint4*>(w + (size_t)idx * 8); },
      [&](int idx, uint4 v) { *reinterpret_cast<uint4*>(dst + swz256(idx >> 4, idx & 15)) = v; });
}

// waves 0-3: yt[pos][w*32 + co'] = sum_ci Wl[w*32 + co'][ci] h1[pos][ci]   (D[co][pos], A = Wl rows)
__device__ __forceinline__ void gemm_fwd(const unsigned char* ws, const unsigned char* ht, float* yt, int w, int r,
                                         int h) {
  f32x16_t acc = zero16();
#pragma unroll
  for (int kk = 0; kk < 8; ++kk)
    acc = mfma32(lds_frag(ws, swz256(w * 32 + r, kk * 2 + h)), lds_frag(ht, swz256(r, kk * 2 + h)), acc);
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<float4*>(yt + r * YS + w * 32 + 8 * g + 4 * h) =
        make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
}

// h1 = LN_C(s1) ; s2 = h1 + GELU(h1 Wl^T + bl) ; h2 = LN_C(s2)
// grid: persistent over items (b, t), 512 threads; LDS: Wl 32 KB + h1 tile 8 KB + D^T tile 16.5 KB
__global__ void __launch_bounds__(512) pc_ln_linear_fwd_kernel(
    const bf16_t* __restrict__ s1, const float* __restrict__ g1, const float* __restrict__ be1,
    const bf16_t* __restrict__ wl, const float* __restrict__ bl, const float* __restrict__ g2,
    const float* __restrict__ be2, bf16_t* __restrict__ h2, float4* __restrict__ stats, int B, int L, float eps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;
  unsigned char* ht = smem + 32768;
  float* yt = reinterpret_cast<float*>(smem + 32768 + TR * 256);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int j = tid >> 4, ch = tid & 15;
  const int T = (L + TR - 1) / TR;
  const long items = (long)B * T;
  stage_wl(ws, wl);
  float ga1[8], bt1[8], ga2[8], bt2[8], bb[8];
  ld8f(g1 + ch * 8, ga1);
  ld8f(be1 + ch * 8, bt1);
  ld8f(g2 + ch * 8, ga2);
  ld8f(be2 + ch * 8, bt2);
  ld8f(bl + ch * 8, bb);
  const float inv_c = 1.0f / (float)CH;
  long item = blockIdx.x;
  auto row_of = [&](long it, bool& ok) -> size_t {
    const int b = (int)(it / T), t = (int)(it - (it / T) * T);
    const int l = t * TR + j;
    ok = it < items && l < L;
    return ((size_t)b * L + (ok ? l : 0)) * CH + ch * 8;
  };
  bool okn;
  size_t offn = row_of(item, okn);
  uint4 nxt = ldq(s1 + offn, okn);
  __syncthreads();
  for (; item < items; item += gridDim.x) {
    const bool ok = okn;
    const size_t off = offn;
    float x[8], d[8], hv[8];
    unpack8(nxt, x);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += x[e];
    const float mean1 = row_sum(s) * inv_c;
    float v = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { d[e] = x[e] - mean1; v += d[e] * d[e]; }
    const float rstd1 = rsqrtf(row_sum(v) * inv_c + eps);
#pragma unroll
    for (int e = 0; e < 8; ++e) hv[e] = ok ? bfround(d[e] * rstd1 * ga1[e] + bt1[e]) : 0.f;
    *reinterpret_cast<uint4*>(ht + swz256(j, ch)) = packq8(hv);
    __syncthreads();
    offn = row_of(item + gridDim.x, okn);
    nxt = ldq(s1 + offn, okn);
    if (w < 4) gemm_fwd(ws, ht, yt, w, r, h);
    __syncthreads();
    float pre[8], gv[8], s2[8];
    {
      const float4 ya = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8);
      const float4 yb = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8 + 4);
      pre[0] = ya.x + bb[0]; pre[1] = ya.y + bb[1]; pre[2] = ya.z + bb[2]; pre[3] = ya.w + bb[3];
      pre[4] = yb.x + bb[4]; pre[5] = yb.y + bb[5]; pre[6] = yb.z + bb[6]; pre[7] = yb.w + bb[7];
    }
    gelu8(pre, gv);
    s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { s2[e] = ok ? hv[e] + gv[e] : 0.f; s += s2[e]; }
    const float mean2 = row_sum(s) * inv_c;
    v = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { d[e] = s2[e] - mean2; v += d[e] * d[e]; }
    const float rstd2 = rsqrtf(row_sum(v) * inv_c + eps);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = d[e] * rstd2 * ga2[e] + bt2[e];
    if (ok) {
      *reinterpret_cast<uint4*>(h2 + off) = packq8(o);
      if (ch == 0) stats[off / CH] = make_float4(mean1, rstd1, mean2, rstd2);
    }
  }
}

// Backward of the above.  dh2 = dh2a + dh2b + dh2c (any may be null: the next block's gradient and
// the attention's, one buffer per head pair):
//   xh2 = (s2 - mean2) rstd2 ; ds2 = rstd2 (dh2 g2 - <dh2 g2> - xh2 <dh2 g2 xh2>)    (<.> = mean over C)
//   dpre = ds2 GELU'(pre) ; dh1 = ds2 + dpre Wl ; ds1 = rstd1 (dh1 g1 - <dh1 g1> - xh1 <dh1 g1 xh1>)
//   dWl += dpre^T h1 ; dbl += sum dpre ; dg2 += sum dh2 xh2 ; db2 += sum dh2 ; dg1 += sum dh1 xh1 ;
//   db1 += sum dh1 ; dgbp[b][t][c] = sum_{rows of item} ds1
// LDS: Wl 32 KB + h1 tile 8 KB + dpre tile 8 KB (reused for ds1) + D^T tile 16.5 KB -> 2 workgroups/CU.
__global__ void __launch_bounds__(512) pc_ln_linear_bwd_kernel(
    const bf16_t* __restrict__ dh2a, const bf16_t* __restrict__ dh2b, const bf16_t* __restrict__ dh2c,
    const bf16_t* __restrict__ s1,
    const float4* __restrict__ stats, const float* __restrict__ g1, const float* __restrict__ be1,
    const bf16_t* __restrict__ wl, const float* __restrict__ bl, const float* __restrict__ g2,
    bf16_t* __restrict__ ds1, float* __restrict__ dgbp, float* __restrict__ dg2, float* __restrict__ db2,
    float* __restrict__ dg1, float* __restrict__ db1, float* __restrict__ dwl, float* __restrict__ dbl,
    float* __restrict__ dwl_slab, int B, int L) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ws = smem;
  unsigned char* ht = smem + 32768;
  unsigned char* dt = ht + TR * 256;
  float* yt = reinterpret_cast<float*>(dt + TR * 256);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int q = tr_q(lane), tc = tr_c(lane);
  const int j = tid >> 4, ch = tid & 15;
  const int T = (L + TR - 1) / TR;
  const long items = (long)B * T;
  stage_wl(ws, wl);
  float ga1[8], bt1[8], ga2[8], bb[8];
  ld8f(g1 + ch * 8, ga1);
  ld8f(be1 + ch * 8, bt1);
  ld8f(g2 + ch * 8, ga2);
  ld8f(bl + ch * 8, bb);
  float adg2[8], adb2[8], adg1[8], adb1[8], adbl[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { adg2[e] = 0.f; adb2[e] = 0.f; adg1[e] = 0.f; adb1[e] = 0.f; adbl[e] = 0.f; }
  f32x16_t aw0 = zero16(), aw1 = zero16();
  const int wco = (w >> 1) * 32, wci = (w & 1) * 64;
  const float inv_c = 1.0f / (float)CH;
  long item = blockIdx.x;
  auto row_of = [&](long it, bool& ok) -> size_t {
    const int b = (int)(it / T), t = (int)(it - (it / T) * T);
    const int l = t * TR + j;
    ok = it < items && l < L;
    return ((size_t)b * L + (ok ? l : 0)) * CH + ch * 8;
  };
  bool okn;
  size_t offn = row_of(item, okn);
  uint4 n_s = ldq(s1 + offn, okn), n_a = ldq(dh2a + offn, okn && dh2a), n_b = ldq(dh2b + offn, okn && dh2b);
  uint4 n_c = ldq(dh2c + offn, okn && dh2c);
  float4 n_st = okn ? stats[offn / CH] : make_float4(0.f, 1.f, 0.f, 1.f);
  __syncthreads();
  for (; item < items; item += gridDim.x) {
    const bool ok = okn;
    const size_t off = offn;
    const float mean1 = n_st.x, rstd1 = n_st.y, mean2 = n_st.z, rstd2 = n_st.w;
    float x[8], xh1[8], hv[8], dh[8], tmp[8], tmc[8];
    unpack8(n_s, x);
    unpack8(n_a, dh);
    unpack8(n_b, tmp);
    unpack8(n_c, tmc);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dh[e] += tmp[e] + tmc[e];
      xh1[e] = (x[e] - mean1) * rstd1;
      hv[e] = ok ? bfround(xh1[e] * ga1[e] + bt1[e]) : 0.f;
    }
    *reinterpret_cast<uint4*>(ht + swz256(j, ch)) = packq8(hv);
    __syncthreads();                                                       // A: h1 tile ready
    offn = row_of(item + gridDim.x, okn);
    n_s = ldq(s1 + offn, okn);
    n_a = ldq(dh2a + offn, okn && dh2a);
    n_b = ldq(dh2b + offn, okn && dh2b);
    n_c = ldq(dh2c + offn, okn && dh2c);
    n_st = okn ? stats[offn / CH] : make_float4(0.f, 1.f, 0.f, 1.f);
    if (w < 4) gemm_fwd(ws, ht, yt, w, r, h);
    __syncthreads();                                                       // B: pre tile ready
    float pre[8], gv[8], gd[8], xh2[8], ds2[8], dp[8];
    {
      const float4 ya = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8);
      const float4 yb = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8 + 4);
      pre[0] = ya.x + bb[0]; pre[1] = ya.y + bb[1]; pre[2] = ya.z + bb[2]; pre[3] = ya.w + bb[3];
      pre[4] = yb.x + bb[4]; pre[5] = yb.y + bb[5]; pre[6] = yb.z + bb[6]; pre[7] = yb.w + bb[7];
    }
    gelu_both8(pre, gv, gd);
    float sa = 0.f, sc = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xh2[e] = ((hv[e] + gv[e]) - mean2) * rstd2;
      if (!ok) dh[e] = 0.f;
      adg2[e] += dh[e] * xh2[e];
      adb2[e] += dh[e];
      const float gg = dh[e] * ga2[e];
      sa += gg;
      sc += gg * xh2[e];
    }
    row_sum2(sa, sc);
    sa *= inv_c;
    sc *= inv_c;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ds2[e] = ok ? rstd2 * (dh[e] * ga2[e] - sa - xh2[e] * sc) : 0.f;
      dp[e] = bfround(ds2[e] * gd[e]);
      adbl[e] += dp[e];
    }
    *reinterpret_cast<uint4*>(dt + swz256(j, ch)) = packq8(dp);
    __syncthreads();                                                       // C: dpre tile ready, yt free
    if (w < 4) {
      // D[ci][pos] = sum_co Wl[co][ci] dpre[pos][co]: A = Wl^T (transposed LDS read), B = dpre rows
      f32x16_t acc = zero16();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const int rlo = kk * 16 + 8 * h + q;
        const int col = w * 32 + tc;
        const bf16x8 fa = cat_tr(lds_tr(ws, swz256e(rlo, col)), lds_tr(ws, swz256e(rlo + 4, col)));
        acc = mfma32(fa, lds_frag(dt, swz256(r, kk * 2 + h)), acc);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(yt + r * YS + w * 32 + 8 * g + 4 * h) =
            make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
    }
    // dWl[co][ci] += sum_pos dpre[pos][co] h1[pos][ci]   (both operands transposed LDS reads)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int rlo = ks * 16 + 8 * h + q;
      const bf16x8 fa = cat_tr(lds_tr(dt, swz256e(rlo, wco + tc)), lds_tr(dt, swz256e(rlo + 4, wco + tc)));
      const bf16x8 fb0 = cat_tr(lds_tr(ht, swz256e(rlo, wci + tc)), lds_tr(ht, swz256e(rlo + 4, wci + tc)));
      const bf16x8 fb1 =
          cat_tr(lds_tr(ht, swz256e(rlo, wci + 32 + tc)), lds_tr(ht, swz256e(rlo + 4, wci + 32 + tc)));
      aw0 = mfma32(fa, fb0, aw0);
      aw1 = mfma32(fa, fb1, aw1);
    }
    __syncthreads();                                                       // D: dh1 GEMM done, dt/ht free
    float dh1[8];
    {
      const float4 ya = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8);
      const float4 yb = *reinterpret_cast<const float4*>(yt + j * YS + ch * 8 + 4);
      const float yv[8] = {ya.x, ya.y, ya.z, ya.w, yb.x, yb.y, yb.z, yb.w};
      sa = 0.f;
      sc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dh1[e] = ok ? ds2[e] + yv[e] : 0.f;
        adg1[e] += dh1[e] * xh1[e];
        adb1[e] += dh1[e];
        const float gg = dh1[e] * ga1[e];
        sa += gg;
        sc += gg * xh1[e];
      }
    }
    row_sum2(sa, sc);
    sa *= inv_c;
    sc *= inv_c;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = ok ? rstd1 * (dh1[e] * ga1[e] - sa - xh1[e] * sc) : 0.f;
    const uint4 oq = packq8(o);
    if (ok) *reinterpret_cast<uint4*>(ds1 + off) = oq;
    // per-item column sums of ds1 (the broadcast global->local vector's gradient), plain layout in dt
    *reinterpret_cast<uint4*>(dt + j * 256 + ch * 16) = oq;
    __syncthreads();                                                       // E
    if (tid < CH) {
      float a = 0.f;
#pragma unroll 8
      for (int k = 0; k < TR; ++k) a += bf2f(*reinterpret_cast<const bf16_t*>(dt + k * 256 + tid * 2));
      dgbp[(size_t)item * CH + tid] = a;
    }
  }
  // [C] vector gradients: sum the 32 row-threads of each chunk through LDS, one atomic per channel
  float* accs[5] = {adg2, adb2, adg1, adb1, adbl};
  float* dsts[5] = {dg2, db2, dg1, db1, dbl};
#pragma unroll
  for (int a = 0; a < 5; ++a) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) yt[j * CH + ch * 8 + e] = accs[a][e];
    __syncthreads();
    if (tid < CH) {
      float v = 0.f;
#pragma unroll 8
      for (int k = 0; k < TR; ++k) v += yt[k * CH + tid];
      atomicAdd(dsts[a] + tid, v);
    }
  }
  // dwl_slab: one slab row per workgroup (folded by a column-sum pass), not 16 K contended atomics
  float* dw = dwl_slab != nullptr ? dwl_slab + (size_t)blockIdx.x * CH * CH : dwl;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int co = wco + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (dwl_slab != nullptr) {
      dw[(size_t)co * CH + wci + r] = aw0[i];
      dw[(size_t)co * CH + wci + 32 + r] = aw1[i];
    } else {
      atomicAdd(dw + (size_t)co * CH + wci + r, aw0[i]);
      atomicAdd(dw + (size_t)co * CH + wci + 32 + r, aw1[i]);
    }
  }
}

int g_pc_cus = -1;
int pc_num_cus() {
  if (g_pc_cus < 0) {
    int dev = 0;
    g_pc_cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, dev) == hipSuccess) g_pc_cus = p.multiProcessorCount;
    }
  }
  return g_pc_cus;
}
int pc_grid(long items) {
  const long cap = 2L * pc_num_cus();
  return (int)(items < cap ? (items > 0 ? items : 1) : cap);
}
}  // namespace

extern "C" int pbx_colsum_add(const float* src, int rows, int cols, float* dst, const float* scale, hipStream_t st);

// s1/h2 [B, L, 128] bf16; g1/be1/g2/be2/bl [128] fp32; wl [128, 128] bf16 (torch Linear layout);
// stats [B*L] float4 (mean1, rstd1, mean2, rstd2)
PBX_EXPORT int pbx_pc_ln_linear_fwd(const void* s1, const float* g1, const float* be1, const void* wl, const float* bl,
                                    const float* g2, const float* be2, void* h2, void* stats, int B, int L, float eps,
                                    hipStream_t st) {
  if (B <= 0 || L <= 0) return (int)hipErrorInvalidValue;
  const long items = (long)B * ((L + TR - 1) / TR);
  const int lds = 32768 + TR * 256 + TR * YS * 4;
  hipLaunchKernelGGL(pc_ln_linear_fwd_kernel, dim3(pc_grid(items)), dim3(512), lds, st, (const bf16_t*)s1, g1, be1,
                     (const bf16_t*)wl, bl, g2, be2, (bf16_t*)h2, (float4*)stats, B, L, eps);
  return pbx_launch_status();
}

// dh2a / dh2b / dh2c: bf16 [B, L, 128] or null (summed); ds1 bf16 [B, L, 128] (written); dgbp fp32
// [B, ceil(L/32), 128] (written); dg2/db2/dg1/db1/dbl [128] and dwl [128, 128] fp32 accumulated into.
PBX_EXPORT int pbx_pc_ln_linear_bwd(const void* dh2a, const void* dh2b, const void* dh2c, const void* s1,
                                    const void* stats,
                                    const float* g1, const float* be1, const void* wl, const float* bl, const float* g2,
                                    void* ds1, float* dgbp, float* dg2, float* db2, float* dg1, float* db1, float* dwl,
                                    float* dbl, float* dwl_slab, int slab_rows, int B, int L, hipStream_t st) {
  if (B <= 0 || L <= 0) return (int)hipErrorInvalidValue;
  const long items = (long)B * ((L + TR - 1) / TR);
  const int lds = 32768 + 2 * TR * 256 + TR * YS * 4;
  const int grid = pc_grid(items);
  float* slab = dwl_slab != nullptr && grid <= slab_rows ? dwl_slab : nullptr;
  hipLaunchKernelGGL(pc_ln_linear_bwd_kernel, dim3(grid), dim3(512), lds, st, (const bf16_t*)dh2a,
                     (const bf16_t*)dh2b, (const bf16_t*)dh2c, (const bf16_t*)s1, (const float4*)stats, g1, be1, (const bf16_t*)wl, bl, g2,
                     (bf16_t*)ds1, dgbp, dg2, db2, dg1, db1, dwl, dbl, slab, B, L);
  if (slab != nullptr) {
    const int rc = pbx_launch_status();
    if (rc != 0) return rc;
    return pbx_colsum_add(slab, grid, CH * CH, dwl, nullptr, st);
  }
  return pbx_launch_status();
}
