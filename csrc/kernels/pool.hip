// Pooling kernels, NHWC bf16.
//  * max pool fwd stores a uint8 window-argmax per output element; bwd gathers through it
//    (TF MaxPoolGrad routes the gradient to the first maximum of each window).
//  * avg pool: TF SAME semantics divide by the number of in-bounds taps (count_pad=0), or
//    by kh*kw (count_pad=1).
//  * global mean over H*W (slim resnet 'pool5', reference vgg/nets/resnet_v1.py:244).
// Eight channels per lane (16-B loads) when C % 8 == 0.
#include "common.h"

namespace dtm {

struct PoolArgs {
  int N, H, W, C, P, Q, KH, KW, SH, SW, PH, PW;
};
// first window index p >= 0 with p*S >= num  (num = h + pad - k + 1)
__device__ __forceinline__ int first_win(int num, int S) { return num <= 0 ? 0 : (num + S - 1) / S; }

template <int V>
__device__ __forceinline__ void ld(const bf16_t* p, float* f) {
  if constexpr (V == 8) {
    uint4 u = *(const uint4*)p;
    f[0] = lo_bf(u.x); f[1] = hi_bf(u.x); f[2] = lo_bf(u.y); f[3] = hi_bf(u.y);
    f[4] = lo_bf(u.z); f[5] = hi_bf(u.z); f[6] = lo_bf(u.w); f[7] = hi_bf(u.w);
  } else {
    f[0] = bf2f(*p);
  }
}
template <int V>
__device__ __forceinline__ void st(bf16_t* p, const float* f) {
  if constexpr (V == 8) {
    *(uint4*)p = make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
  } else {
    *p = f2bf(f[0]);
  }
}

template <int V>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, PoolArgs a) {
  const int cols = a.C / V;
  const long total = (long)a.N * a.P * a.Q * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int cv = (int)(i % cols) * V;
    long o = i / cols;
    int q = o % a.Q; long t = o / a.Q;
    int p = t % a.P; int n = (int)(t / a.P);
    float best[V];
    uint8_t bi[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    for (int r = 0; r < a.KH; ++r) {
      int h = p * a.SH - a.PH + r;
      if (h < 0 || h >= a.H) continue;
      for (int s = 0; s < a.KW; ++s) {
        int w = q * a.SW - a.PW + s;
        if (w < 0 || w >= a.W) continue;
        float f[V];
        ld<V>(x + (((long)n * a.H + h) * a.W + w) * a.C + cv, f);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (f[e] > best[e]) { best[e] = f[e]; bi[e] = (uint8_t)(r * a.KW + s); }
      }
    }
    st<V>(y + o * a.C + cv, best);
    if (arg) {
#pragma unroll
      for (int e = 0; e < V; ++e) arg[o * a.C + cv + e] = bi[e];
    }
  }
}

// dx[n,h,w,c] = sum over windows (p,q) covering (h,w) whose argmax is (h,w) of dy[n,p,q,c]
template <int V>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                          bf16_t* __restrict__ dx, PoolArgs a) {
  const int cols = a.C / V;
  const long total = (long)a.N * a.H * a.W * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int cv = (int)(i % cols) * V;
    long o = i / cols;
    int w = o % a.W; long t = o / a.W;
    int h = t % a.H; int n = (int)(t / a.H);
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    // windows p with p*SH - PH <= h <= p*SH - PH + KH - 1
    int plo = first_win(h + a.PH - a.KH + 1, a.SH), phi = (h + a.PH) / a.SH;
    int qlo = first_win(w + a.PW - a.KW + 1, a.SW), qhi = (w + a.PW) / a.SW;
    for (int p = plo; p <= min(phi, a.P - 1); ++p) {
      int r = h - (p * a.SH - a.PH);
      if (r < 0 || r >= a.KH) continue;
      for (int q = qlo; q <= min(qhi, a.Q - 1); ++q) {
        int s = w - (q * a.SW - a.PW);
        if (s < 0 || s >= a.KW) continue;
        long oo = (((long)n * a.P + p) * a.Q + q) * a.C + cv;
        float g[V];
        ld<V>(dy + oo, g);
        uint8_t want = (uint8_t)(r * a.KW + s);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (arg[oo + e] == want) acc[e] += g[e];
      }
    }
    st<V>(dx + o * a.C + cv, acc);
  }
}

template <int V>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, PoolArgs a,
                                                          int count_pad) {
  const int cols = a.C / V;
  const long total = (long)a.N * a.P * a.Q * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int cv = (int)(i % cols) * V;
    long o = i / cols;
    int q = o % a.Q; long t = o / a.Q;
    int p = t % a.P; int n = (int)(t / a.P);
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    int cnt = 0;
    for (int r = 0; r < a.KH; ++r) {
      int h = p * a.SH - a.PH + r;
      if (h < 0 || h >= a.H) continue;
      for (int s = 0; s < a.KW; ++s) {
        int w = q * a.SW - a.PW + s;
        if (w < 0 || w >= a.W) continue;
        float f[V];
        ld<V>(x + (((long)n * a.H + h) * a.W + w) * a.C + cv, f);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += f[e];
        ++cnt;
      }
    }
    float inv = 1.f / (float)(count_pad ? a.KH * a.KW : max(cnt, 1));
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] *= inv;
    st<V>(y + o * a.C + cv, acc);
  }
}

template <int V>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, PoolArgs a,
                                                          int count_pad) {
  const int cols = a.C / V;
  const long total = (long)a.N * a.H * a.W * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int cv = (int)(i % cols) * V;
    long o = i / cols;
    int w = o % a.W; long t = o / a.W;
    int h = t % a.H; int n = (int)(t / a.H);
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    int plo = first_win(h + a.PH - a.KH + 1, a.SH), phi = min(a.P - 1, (h + a.PH) / a.SH);
    int qlo = first_win(w + a.PW - a.KW + 1, a.SW), qhi = min(a.Q - 1, (w + a.PW) / a.SW);
    for (int p = plo; p <= phi; ++p) {
      int h0 = p * a.SH - a.PH;
      if (h < h0 || h >= h0 + a.KH) continue;
      int hc = min(h0 + a.KH, a.H) - max(h0, 0);
      for (int q = qlo; q <= qhi; ++q) {
        int w0 = q * a.SW - a.PW;
        if (w < w0 || w >= w0 + a.KW) continue;
        int wcnt = min(w0 + a.KW, a.W) - max(w0, 0);
        float inv = 1.f / (float)(count_pad ? a.KH * a.KW : max(hc * wcnt, 1));
        float g[V];
        ld<V>(dy + (((long)n * a.P + p) * a.Q + q) * a.C + cv, g);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += g[e] * inv;
      }
    }
    st<V>(dx + o * a.C + cv, acc);
  }
}

// The generic avg pool with 8 channels per lane and 32-bit magic-number index math (the 64-bit divisions of the
// V-template forms above dominated their time: 30 us for the backward of Inception's 5x5/3 aux-head pool over
// 17x17x768).  Same tap order and divisor as those, so the results match them exactly.  The backward can add into
// dx (accum != 0): the aux head's pool gradient folded into the block-input gradient the main path produced
// (ops/nn.py avg_pool grad_tail) instead of a separate add over the whole map.
__global__ __launch_bounds__(256) void avgpool_fwd8_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                           PoolArgs a, int count_pad, FastDiv fcols, FastDiv fQ,
                                                           FastDiv fP, int total) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t o = fdiv(i, fcols);
    const int cv = (int)(i - o * fcols.d) * 8;
    const uint32_t t = fdiv(o, fQ);
    const int q = (int)(o - t * fQ.d);
    const int n = (int)fdiv(t, fP), p = (int)(t - n * fP.d);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    int cnt = 0;
    for (int r = 0; r < a.KH; ++r) {
      const int h = p * a.SH - a.PH + r;
      if (h < 0 || h >= a.H) continue;
      for (int s = 0; s < a.KW; ++s) {
        const int w = q * a.SW - a.PW + s;
        if (w < 0 || w >= a.W) continue;
        float f[8];
        ld<8>(x + ((n * a.H + h) * a.W + w) * a.C + cv, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += f[e];
        ++cnt;
      }
    }
    const float inv = 1.f / (float)(count_pad ? a.KH * a.KW : max(cnt, 1));
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    st<8>(y + o * a.C + cv, acc);
  }
}
__global__ __launch_bounds__(256) void avgpool_bwd8_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                                           PoolArgs a, int count_pad, int accum, FastDiv fcols,
                                                           FastDiv fW, FastDiv fH, int total) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t o = fdiv(i, fcols);
    const int cv = (int)(i - o * fcols.d) * 8;
    const uint32_t t = fdiv(o, fW);
    const int w = (int)(o - t * fW.d);
    const int n = (int)fdiv(t, fH), h = (int)(t - n * fH.d);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const int plo = first_win(h + a.PH - a.KH + 1, a.SH), phi = min(a.P - 1, (h + a.PH) / a.SH);
    const int qlo = first_win(w + a.PW - a.KW + 1, a.SW), qhi = min(a.Q - 1, (w + a.PW) / a.SW);
    for (int p = plo; p <= phi; ++p) {
      const int h0 = p * a.SH - a.PH;
      if (h < h0 || h >= h0 + a.KH) continue;
      const int hc = min(h0 + a.KH, a.H) - max(h0, 0);
      for (int q = qlo; q <= qhi; ++q) {
        const int w0 = q * a.SW - a.PW;
        if (w < w0 || w >= w0 + a.KW) continue;
        const int wcnt = min(w0 + a.KW, a.W) - max(w0, 0);
        const float inv = 1.f / (float)(count_pad ? a.KH * a.KW : max(hc * wcnt, 1));
        float g[8];
        ld<8>(dy + ((n * a.P + p) * a.Q + q) * a.C + cv, g);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += g[e] * inv;
      }
    }
    if (accum) {
      float f[8];
      ld<8>(dx + o * a.C + cv, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
    }
    st<8>(dx + o * a.C + cv, acc);
  }
}

// VALID K x K / stride S average pool with every window in bounds (Inception's 5x5/3 aux-head pool): the tap
// loops are compile-time, so a lane issues all its loads back to back instead of one dependent load per runtime
// loop trip (the generic kernels above were load-latency bound: 18 us forward / 29 us backward for that pool).
// One lane per output (forward) or input (backward) 8-channel chunk, no grid-stride loop; same tap order and
// divisor as the generic kernels, so the results match them bit for bit.
template <int K>
__global__ __launch_bounds__(256) void avgpool_fwd_valid_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                                PoolArgs a, FastDiv fcols, FastDiv fQ, FastDiv fP,
                                                                int total) {
  const int i = xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x;  // (overlapping windows: one L2)
  if (i >= total) return;
  const uint32_t o = fdiv(i, fcols);
  const int cv = (int)(i - o * fcols.d) * 8;
  const uint32_t t = fdiv(o, fQ);
  const int q = (int)(o - t * fQ.d);
  const int n = (int)fdiv(t, fP), p = (int)(t - n * fP.d);
  const bf16_t* base = x + ((n * a.H + p * a.SH) * a.W + q * a.SW) * a.C + cv;
  uint4 v[K * K];
#pragma unroll
  for (int r = 0; r < K; ++r)
#pragma unroll
    for (int s = 0; s < K; ++s) v[r * K + s] = *(const uint4*)(base + (r * a.W + s) * a.C);
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
  for (int k = 0; k < K * K; ++k) {
    const uint4 u = v[k];
    acc[0] += lo_bf(u.x); acc[1] += hi_bf(u.x); acc[2] += lo_bf(u.y); acc[3] += hi_bf(u.y);
    acc[4] += lo_bf(u.z); acc[5] += hi_bf(u.z); acc[6] += lo_bf(u.w); acc[7] += hi_bf(u.w);
  }
  const float inv = 1.f / (float)(K * K);
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] *= inv;
  st<8>(y + o * a.C + cv, acc);
}
template <int K, int S>
__global__ __launch_bounds__(256) void avgpool_bwd_valid_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                                                PoolArgs a, int accum, FastDiv fcols, FastDiv fW,
                                                                FastDiv fH, int total, const bf16_t* __restrict__ zero) {
  constexpr int MW = (K + S - 1) / S;  // windows covering a pixel, per dimension, at most
  const int i = xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x;  // (a dy chunk's 25 readers: one L2)
  if (i >= total) return;
  const uint32_t o = fdiv(i, fcols);
  const int cv = (int)(i - o * fcols.d) * 8;
  const uint32_t t = fdiv(o, fW);
  const int w = (int)(o - t * fW.d);
  const int n = (int)fdiv(t, fH), h = (int)(t - n * fH.d);
  const int plo = first_win(h - K + 1, S), phi = min(a.P - 1, h / S);
  const int qlo = first_win(w - K + 1, S), qhi = min(a.Q - 1, w / S);
  uint4 g[MW * MW];
#pragma unroll
  for (int dp = 0; dp < MW; ++dp)
#pragma unroll
    for (int dq = 0; dq < MW; ++dq) {
      const bool ok = plo + dp <= phi && qlo + dq <= qhi;
      const bf16_t* src = ok ? dy + ((n * a.P + plo + dp) * a.Q + qlo + dq) * a.C + cv : zero;
      g[dp * MW + dq] = *(const uint4*)src;
    }
  uint4 prev = make_uint4(0, 0, 0, 0);
  if (accum) prev = *(const uint4*)(dx + o * a.C + cv);
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  const float inv = 1.f / (float)(K * K);
#pragma unroll
  for (int dp = 0; dp < MW; ++dp)
#pragma unroll
    for (int dq = 0; dq < MW; ++dq) {
      if (plo + dp > phi || qlo + dq > qhi) continue;
      const uint4 u = g[dp * MW + dq];
      acc[0] += lo_bf(u.x) * inv; acc[1] += hi_bf(u.x) * inv; acc[2] += lo_bf(u.y) * inv; acc[3] += hi_bf(u.y) * inv;
      acc[4] += lo_bf(u.z) * inv; acc[5] += hi_bf(u.z) * inv; acc[6] += lo_bf(u.w) * inv; acc[7] += hi_bf(u.w) * inv;
    }
  if (accum) {
    acc[0] += lo_bf(prev.x); acc[1] += hi_bf(prev.x); acc[2] += lo_bf(prev.y); acc[3] += hi_bf(prev.y);
    acc[4] += lo_bf(prev.z); acc[5] += hi_bf(prev.z); acc[6] += lo_bf(prev.w); acc[7] += hi_bf(prev.w);
  }
  st<8>(dx + o * a.C + cv, acc);
}

// global mean over H*W: x[N][HW][C] -> y[N][C] (fp32 out, or bf16 when it only feeds the logits GEMM: the cast
// launch of its input disappears, same rounding)
template <typename TO>
__global__ __launch_bounds__(256) void global_avg_fwd_kernel(const bf16_t* __restrict__ x, TO* __restrict__ y, int HW,
                                                             int C) {
  const int n = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const bf16_t* p = x + (long)n * HW * C + c;
  float s = 0.f;
  for (int i = 0; i < HW; ++i) s += bf2f(p[(long)i * C]);
  if constexpr (sizeof(TO) == 2) y[(long)n * C + c] = f2bf(s / (float)HW);
  else y[(long)n * C + c] = s / (float)HW;
}
template <typename TI>
__global__ __launch_bounds__(256) void global_avg_bwd_kernel(const TI* __restrict__ dy, bf16_t* __restrict__ dx, int N,
                                                             int HW, int C) {
  const long total = (long)N * HW * C;
  const float inv = 1.f / (float)HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c = i % C;
    long n = i / ((long)HW * C);
    float g;
    if constexpr (sizeof(TI) == 2) g = bf2f(dy[n * C + c]);
    else g = dy[n * C + c];
    dx[i] = f2bf(g * inv);
  }
}

// The same two with 8 channels per lane (C % 8 == 0).  Forward: a block is one image and 512 channels, its four
// waves split the H*W rows (16-B loads, four in flight per lane) and combine through LDS in a fixed order (the
// one-lane-per-channel form ran H*W dependent 2-B loads per lane: 17.6 us for Inception's 8x8x2048 logits pool).
// Backward: one lane per 8-channel output chunk, 32-bit magic-number indexing, no grid-stride loop (the form above
// spent its time in 64-bit divisions: 27 us Inception / 40 us ResNet-50 for a write of 17 / 51 MB).
template <typename TO>
__global__ __launch_bounds__(256) void global_avg_fwd8_kernel(const bf16_t* __restrict__ x, TO* __restrict__ y, int HW,
                                                              int C) {
  __shared__ float red[3][8][64];
  const int n = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 8;
  const bool live = c < C;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  if (live) {
    const bf16_t* p = x + (long)n * HW * C + c;
    int i = wv;
    for (; i + 12 < HW; i += 16) {
      uint4 u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) u[k] = *(const uint4*)(p + (long)(i + 4 * k) * C);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[0] += lo_bf(u[k].x); acc[1] += hi_bf(u[k].x); acc[2] += lo_bf(u[k].y); acc[3] += hi_bf(u[k].y);
        acc[4] += lo_bf(u[k].z); acc[5] += hi_bf(u[k].z); acc[6] += lo_bf(u[k].w); acc[7] += hi_bf(u[k].w);
      }
    }
    for (; i < HW; i += 4) {
      const uint4 u = *(const uint4*)(p + (long)i * C);
      acc[0] += lo_bf(u.x); acc[1] += hi_bf(u.x); acc[2] += lo_bf(u.y); acc[3] += hi_bf(u.y);
      acc[4] += lo_bf(u.z); acc[5] += hi_bf(u.z); acc[6] += lo_bf(u.w); acc[7] += hi_bf(u.w);
    }
  }
  if (wv) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wv - 1][e][lane] = acc[e];
  }
  __syncthreads();
  if (wv || !live) return;
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = ((acc[e] + red[0][e][lane]) + (red[1][e][lane] + red[2][e][lane])) / (float)HW;
  if constexpr (sizeof(TO) == 2) {
    st<8>((bf16_t*)y + (long)n * C + c, o);
  } else {
    float4* q = (float4*)((float*)y + (long)n * C + c);
    q[0] = make_float4(o[0], o[1], o[2], o[3]);
    q[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
}
template <typename TI>
__global__ __launch_bounds__(256) void global_avg_bwd8_kernel(const TI* __restrict__ dy, bf16_t* __restrict__ dx, int C,
                                                              FastDiv fcols, FastDiv fHW, int total, float inv) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const uint32_t o = fdiv(i, fcols);  // pixel n*HW + hw
  const int cv = (int)(i - o * fcols.d) * 8;
  const int n = (int)fdiv(o, fHW);
  float g[8];
  if constexpr (sizeof(TI) == 2) {
    ld<8>((const bf16_t*)dy + (long)n * C + cv, g);
  } else {
    const float4* q = (const float4*)((const float*)dy + (long)n * C + cv);
    const float4 a = q[0], b = q[1];
    g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w; g[4] = b.x; g[5] = b.y; g[6] = b.z; g[7] = b.w;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] *= inv;
  st<8>(dx + (long)o * C + cv, g);
}

// ---- BatchNorm-apply + ReLU fused into a max pool (ResNet stem: conv1 -> BN -> ReLU -> 3x3/2 pool) ----
// The normalised activation relu(x*scale + shift) is formed on the fly from the raw conv output and
// never stored.  Backward: each input pixel gathers the gradient of the windows whose argmax it is,
// applies the ReLU mask (recomputed from x) and the BN scale, and accumulates the BN parameter-gradient
// partial sums (sum g*x, sum g) per block (reduced by reduce_rows), exactly as bn_apply_bwd does.
__global__ __launch_bounds__(256) void maxpool_bnrelu_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ ss,
                                                                 bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                                 PoolArgs a, FastDiv fd_cols, FastDiv fd_Q, FastDiv fd_P) {
  const uint32_t cols = a.C >> 3, total = (uint32_t)a.N * a.P * a.Q * cols;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t o = fdiv(i, fd_cols), cv = (i - o * cols) * 8;
    const uint32_t t = fdiv(o, fd_Q), q = o - t * a.Q;
    const uint32_t n = fdiv(t, fd_P), p = t - n * a.P;
    float sc[8], sh[8], best[8];
    uint32_t bi[8];
    {
      const float4 s0 = *(const float4*)(ss + cv), s1 = *(const float4*)(ss + cv + 4);
      const float4 h0 = *(const float4*)(ss + a.C + cv), h1 = *(const float4*)(ss + a.C + cv + 4);
      sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
      sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    for (int r = 0; r < a.KH; ++r) {
      const int h = (int)p * a.SH - a.PH + r;
      if (h < 0 || h >= a.H) continue;
      for (int s = 0; s < a.KW; ++s) {
        const int w = (int)q * a.SW - a.PW + s;
        if (w < 0 || w >= a.W) continue;
        float f[8];
        ld<8>(x + (((size_t)n * a.H + h) * a.W + w) * a.C + cv, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = fmaxf(fmaf(f[e], sc[e], sh[e]), 0.f);
          if (v > best[e]) { best[e] = v; bi[e] = (uint32_t)(r * a.KW + s); }
        }
      }
    }
    st<8>(y + (size_t)o * a.C + cv, best);
    *(uint2*)(arg + (size_t)o * a.C + cv) = make_uint2(bi[0] | bi[1] << 8 | bi[2] << 16 | bi[3] << 24,
                                                      bi[4] | bi[5] << 8 | bi[6] << 16 | bi[7] << 24);
  }
}

// WM = max windows covering one input pixel per dimension (ceil(k / stride)); all candidate window
// loads of FU rows are issued before any is consumed (predicated, no data-dependent branches).
template <int WM, int FU>
__global__ __launch_bounds__(256) void maxpool_bnrelu_bwd_kernel(const bf16_t* __restrict__ dy,
                                                                 const uint8_t* __restrict__ arg,
                                                                 const bf16_t* __restrict__ x, const float* __restrict__ ss,
                                                                 bf16_t* __restrict__ dx, float* __restrict__ part,
                                                                 PoolArgs a, FastDiv fd_W, FastDiv fd_H, int unscaled,
                                                                 int rpb) {
  __shared__ float red[2][256][8];
  const int cols = a.C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  float sc[8], sh[8], a1[8], a0[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sc[e] = ss[c0 + e]; sh[e] = ss[a.C + c0 + e]; a1[e] = 0.f; a0[e] = 0.f; }
  const int M = a.N * a.H * a.W;
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  for (int row0 = lr0 < RP ? r0 + lr0 : r1; row0 < r1; row0 += RP * FU) {
    uint4 gv[FU][WM * WM];
    uint2 av[FU][WM * WM];
    uint32_t want[FU][WM * WM];
    uint4 xvv[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const int row = row0 + u * RP;
      const bool rok = row < r1;
      const uint32_t rr = rok ? (uint32_t)row : (uint32_t)r0;
      const uint32_t tt = fdiv(rr, fd_W), w = rr - tt * a.W;
      const uint32_t n = fdiv(tt, fd_H), h = tt - n * a.H;
      const int plo = first_win((int)h + a.PH - a.KH + 1, a.SH);
      const int qlo = first_win((int)w + a.PW - a.KW + 1, a.SW);
#pragma unroll
      for (int i = 0; i < WM; ++i) {
#pragma unroll
        for (int j = 0; j < WM; ++j) {
          const int p = plo + i, q = qlo + j;
          const int r = (int)h - (p * a.SH - a.PH), s = (int)w - (q * a.SW - a.PW);
          const bool ok = rok && p < a.P && q < a.Q && r >= 0 && r < a.KH && s >= 0 && s < a.KW;
          const size_t oo = ok ? (((size_t)n * a.P + p) * a.Q + q) * a.C + c0 : (size_t)c0;
          gv[u][i * WM + j] = *(const uint4*)(dy + oo);
          av[u][i * WM + j] = *(const uint2*)(arg + oo);
          want[u][i * WM + j] = ok ? (uint32_t)(r * a.KW + s) : 0xffffffffu;
        }
      }
      xvv[u] = *(const uint4*)(x + (size_t)rr * a.C + c0);
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      const int row = row0 + u * RP;
      if (row >= r1) break;
      float acc[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
      for (int k = 0; k < WM * WM; ++k) {
        float g[8];
        g[0] = lo_bf(gv[u][k].x); g[1] = hi_bf(gv[u][k].x); g[2] = lo_bf(gv[u][k].y); g[3] = hi_bf(gv[u][k].y);
        g[4] = lo_bf(gv[u][k].z); g[5] = hi_bf(gv[u][k].z); g[6] = lo_bf(gv[u][k].w); g[7] = hi_bf(gv[u][k].w);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t b = ((e < 4 ? av[u][k].x : av[u][k].y) >> (8 * (e & 3))) & 0xffu;
          if (b == want[u][k]) acc[e] += g[e];
        }
      }
      float xv[8], d[8];
      xv[0] = lo_bf(xvv[u].x); xv[1] = hi_bf(xvv[u].x); xv[2] = lo_bf(xvv[u].y); xv[3] = hi_bf(xvv[u].y);
      xv[4] = lo_bf(xvv[u].z); xv[5] = hi_bf(xvv[u].z); xv[6] = lo_bf(xvv[u].w); xv[7] = hi_bf(xvv[u].w);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = fmaf(xv[e], sc[e], sh[e]) > 0.f ? acc[e] : 0.f;
        d[e] = unscaled ? g : g * sc[e];
        a1[e] += g * xv[e];
        a0[e] += g;
      }
      st<8>(dx + (size_t)row * a.C + c0, d);
    }
  }
  float* prow = part + (size_t)blockIdx.x * 2 * a.C;
  col_reduce8(red, a1, a0, prow, prow + a.C, cols, c0);
}

// ---- 3x3 / stride-2 specialisations (the ResNet-50 and Inception-v3 stem pools; BN = false: the plain max pools
// of Inception's grid-reduction blocks) ----
// Forward: one lane = two vertically adjacent outputs (p, p + 1) of one 8-channel column: their windows share an
// input row, so 15 16-B loads (5 rows x 3 columns) instead of 18, all issued before any is used (compile-time
// window, predicated: an out-of-range tap reads a zero chunk and is never selected).  Same scan order and strict
// comparison as maxpool_bnrelu_fwd_kernel / maxpool_fwd_kernel: the same maxima and first-maximum argmax bytes.
template <bool BN>
__global__ __launch_bounds__(256) void maxpool_bnrelu_fwd_k3s2_kernel(const bf16_t* __restrict__ x,
                                                                      const float* __restrict__ ss,
                                                                      bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                                      PoolArgs a, FastDiv fd_cols, FastDiv fd_Q,
                                                                      FastDiv fd_P2, const bf16_t* __restrict__ zero) {
  const uint32_t cols = a.C >> 3, P2 = (a.P + 1) >> 1, total = (uint32_t)a.N * P2 * a.Q * cols;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t o = fdiv(i, fd_cols), cv = (i - o * cols) * 8;
    const uint32_t t = fdiv(o, fd_Q), q = o - t * a.Q;
    const uint32_t n = fdiv(t, fd_P2), p0 = (t - n * P2) * 2;
    float sc[8], sh[8];
    if constexpr (BN) {
      const float4 s0 = *(const float4*)(ss + cv), s1 = *(const float4*)(ss + cv + 4);
      const float4 h0 = *(const float4*)(ss + a.C + cv), h1 = *(const float4*)(ss + a.C + cv + 4);
      sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
      sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
    }
    const int h0 = (int)p0 * 2 - a.PH, w0 = (int)q * 2 - a.PW;
    uint4 v[5][3];
    bool ok[5][3];
#pragma unroll
    for (int r = 0; r < 5; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int h = h0 + r, w = w0 + c;
        ok[r][c] = h >= 0 && h < a.H && w >= 0 && w < a.W;
        v[r][c] = *(const uint4*)(ok[r][c] ? x + (((size_t)n * a.H + h) * a.W + w) * a.C + cv : zero);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t p = p0 + u;
      if (p >= (uint32_t)a.P) break;
      float best[8];
      uint32_t bi[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if (!ok[2 * u + r][c]) continue;
          const uint4 w4 = v[2 * u + r][c];
          const float f[8] = {lo_bf(w4.x), hi_bf(w4.x), lo_bf(w4.y), hi_bf(w4.y),
                              lo_bf(w4.z), hi_bf(w4.z), lo_bf(w4.w), hi_bf(w4.w)};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float val = BN ? fmaxf(fmaf(f[e], sc[e], sh[e]), 0.f) : f[e];
            if (val > best[e]) { best[e] = val; bi[e] = (uint32_t)(r * 3 + c); }
          }
        }
      }
      const size_t oo = (((size_t)n * a.P + p) * a.Q + q) * a.C + cv;
      st<8>(y + oo, best);
      *(uint2*)(arg + oo) = make_uint2(bi[0] | bi[1] << 8 | bi[2] << 16 | bi[3] << 24,
                                       bi[4] | bi[5] << 8 | bi[6] << 16 | bi[7] << 24);
    }
  }
}

// Backward: one lane = a 2 x 2 block of input pixels (rows 2bi - PH + {0, 1}, columns 2bj - PW + {0, 1}) of one
// 8-channel column.  Every window that covers a pixel of the block is one of the 2 x 2 windows (bi - 1 .. bi,
// bj - 1 .. bj), so their gradient and argmax are loaded once for four pixels (the per-pixel gather of
// maxpool_bnrelu_bwd_kernel loaded them for each pixel: 4x the L2 traffic); each pixel adds its matching windows
// in the same ascending (p, q) order as that kernel - bit-identical dx.  BN-apply backward and the per-block
// partial sums (sum g*x, sum g) as there (BN = false: the plain max-pool gradient, maxpool_bwd_kernel's).
template <bool BN>
__global__ __launch_bounds__(256) void maxpool_bnrelu_bwd_k3s2_kernel(const bf16_t* __restrict__ dy,
                                                                      const uint8_t* __restrict__ arg,
                                                                      const bf16_t* __restrict__ x,
                                                                      const float* __restrict__ ss,
                                                                      bf16_t* __restrict__ dx, float* __restrict__ part,
                                                                      PoolArgs a, FastDiv fd_BW, FastDiv fd_BH,
                                                                      int unscaled, int rpb, const bf16_t* __restrict__ zero,
                                                                      int ldy) {
  // ldy: dy's pixel pitch in elements (a.C; more when dy is the channel slice of a concat's gradient, read in place)
  const int cols = a.C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  const int BH = (a.H + a.PH + 1) >> 1, BW = (a.W + a.PW + 1) >> 1;
  float sc[8], sh[8], a1[8], a0[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = BN ? ss[c0 + e] : 1.f;
    sh[e] = BN ? ss[a.C + c0 + e] : 0.f;
    a1[e] = 0.f;
    a0[e] = 0.f;
  }
  const int M = a.N * BH * BW;
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  for (int blk = lr0 < RP ? r0 + lr0 : r1; blk < r1; blk += RP) {
    const uint32_t tt = fdiv((uint32_t)blk, fd_BW), bj = blk - tt * BW;
    const uint32_t n = fdiv(tt, fd_BH), bi = tt - n * BH;
    uint4 gv[2][2];
    uint2 av[2][2];
    bool wv[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int p = (int)bi - 1 + i, q = (int)bj - 1 + j;
        wv[i][j] = p >= 0 && p < a.P && q >= 0 && q < a.Q;
        const size_t po = wv[i][j] ? ((size_t)n * a.P + p) * a.Q + q : 0;
        gv[i][j] = *(const uint4*)(wv[i][j] ? dy + po * ldy + c0 : zero);
        av[i][j] = wv[i][j] ? *(const uint2*)(arg + po * a.C + c0) : make_uint2(0xffffffffu, 0xffffffffu);
      }
    }
    uint4 xv[2][2];
    bool pv[2][2];
    const int hb = (int)bi * 2 - a.PH, wb = (int)bj * 2 - a.PW;
#pragma unroll
    for (int di = 0; di < 2; ++di) {
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) {
        const int h = hb + di, w = wb + dj;
        pv[di][dj] = h >= 0 && h < a.H && w >= 0 && w < a.W;
        if constexpr (BN)
          xv[di][dj] = *(const uint4*)(pv[di][dj] ? x + (((size_t)n * a.H + h) * a.W + w) * a.C + c0 : zero);
      }
    }
#pragma unroll
    for (int di = 0; di < 2; ++di) {
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) {
        if (!pv[di][dj]) continue;
        float acc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            // pixel (hb + di, wb + dj) in window (bi - 1 + i, bj - 1 + j): tap r = di + 2 (1 - i), s = dj + 2 (1 - j)
            const int r = di + 2 * (1 - i), sidx = dj + 2 * (1 - j);
            if (!wv[i][j] || r > 2 || sidx > 2) continue;
            const uint32_t want = (uint32_t)(r * 3 + sidx);
            const uint4 g4 = gv[i][j];
            const float g[8] = {lo_bf(g4.x), hi_bf(g4.x), lo_bf(g4.y), hi_bf(g4.y),
                                lo_bf(g4.z), hi_bf(g4.z), lo_bf(g4.w), hi_bf(g4.w)};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t b = ((e < 4 ? av[i][j].x : av[i][j].y) >> (8 * (e & 3))) & 0xffu;
              if (b == want) acc[e] += g[e];
            }
          }
        }
        float d[8];
        if constexpr (BN) {
          const uint4 x4 = xv[di][dj];
          const float xf[8] = {lo_bf(x4.x), hi_bf(x4.x), lo_bf(x4.y), hi_bf(x4.y),
                               lo_bf(x4.z), hi_bf(x4.z), lo_bf(x4.w), hi_bf(x4.w)};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float g = fmaf(xf[e], sc[e], sh[e]) > 0.f ? acc[e] : 0.f;
            d[e] = unscaled ? g : g * sc[e];
            a1[e] += g * xf[e];
            a0[e] += g;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = acc[e];
        }
        st<8>(dx + (((size_t)n * a.H + hb + di) * a.W + wb + dj) * a.C + c0, d);
      }
    }
  }
  if constexpr (BN) {
    __shared__ float red[2][256][8];
    float* prow = part + (size_t)blockIdx.x * 2 * a.C;
    col_reduce8(red, a1, a0, prow, prow + a.C, cols, c0);
  }
}

// ---- 3x3 / stride-1 average pools (Inception's pool branches, SAME or VALID): one lane = a vertical strip of
// AVG_R outputs (forward) / input pixels (backward) of one 8-channel column; the (AVG_R + 2) x 3 chunks the strip's
// windows touch are loaded once, all in flight (the generic kernels re-read every chunk for each of the 3 rows that
// use it, one dependent load at a time: 1.8-2 TB/s on 35x35 / 17x17 maps).  Every output (input-gradient) pixel
// adds its taps (windows) in the generic kernels' order with their divisors: bit-identical results.
constexpr int AVG_R = 4;
__global__ __launch_bounds__(256) void avgpool_fwd_k3s1_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                               PoolArgs a, int count_pad, FastDiv fd_cols, FastDiv fd_Q,
                                                               FastDiv fd_PR, const bf16_t* __restrict__ zero) {
  const uint32_t cols = a.C >> 3, PR = (a.P + AVG_R - 1) / AVG_R, total = (uint32_t)a.N * PR * a.Q * cols;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t o = fdiv(i, fd_cols), cv = (i - o * cols) * 8;
    const uint32_t t = fdiv(o, fd_Q), q = o - t * a.Q;
    const uint32_t n = fdiv(t, fd_PR), p0 = (t - n * PR) * AVG_R;
    const int h0 = (int)p0 - a.PH, w0 = (int)q - a.PW;
    uint4 v[AVG_R + 2][3];
    bool ok[AVG_R + 2][3];
#pragma unroll
    for (int r = 0; r < AVG_R + 2; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int h = h0 + r, w = w0 + c;
        ok[r][c] = h >= 0 && h < a.H && w >= 0 && w < a.W;
        v[r][c] = *(const uint4*)(ok[r][c] ? x + (((size_t)n * a.H + h) * a.W + w) * a.C + cv : zero);
      }
    }
#pragma unroll
    for (int u = 0; u < AVG_R; ++u) {
      const uint32_t p = p0 + u;
      if (p >= (uint32_t)a.P) break;
      float acc[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
      int cnt = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if (!ok[u + r][c]) continue;
          const uint4 w4 = v[u + r][c];
          const float f[8] = {lo_bf(w4.x), hi_bf(w4.x), lo_bf(w4.y), hi_bf(w4.y),
                              lo_bf(w4.z), hi_bf(w4.z), lo_bf(w4.w), hi_bf(w4.w)};
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += f[e];
          ++cnt;
        }
      }
      const float inv = 1.f / (float)(count_pad ? 9 : max(cnt, 1));
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] *= inv;
      st<8>(y + (((size_t)n * a.P + p) * a.Q + q) * a.C + cv, acc);
    }
  }
}

__global__ __launch_bounds__(256) void avgpool_bwd_k3s1_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                                               PoolArgs a, int count_pad, FastDiv fd_cols, FastDiv fd_W,
                                                               FastDiv fd_HR, const bf16_t* __restrict__ zero) {
  const uint32_t cols = a.C >> 3, HR = (a.H + AVG_R - 1) / AVG_R, total = (uint32_t)a.N * HR * a.W * cols;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t o = fdiv(i, fd_cols), cv = (i - o * cols) * 8;
    const uint32_t t = fdiv(o, fd_W), w = o - t * a.W;
    const uint32_t n = fdiv(t, fd_HR), hs = (t - n * HR) * AVG_R;
    // windows p covering rows hs .. hs + AVG_R - 1: p = h + PH - 2 .. h + PH (stride 1), i.e. rows pr0 .. pr0 + AVG_R + 1
    const int pr0 = (int)hs + a.PH - 2, qc0 = (int)w + a.PW - 2;
    uint4 g[AVG_R + 2][3];
    float inv[AVG_R + 2][3];
    bool wv[AVG_R + 2][3];
#pragma unroll
    for (int r = 0; r < AVG_R + 2; ++r) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int p = pr0 + r, q = qc0 + c;
        wv[r][c] = p >= 0 && p < a.P && q >= 0 && q < a.Q;
        g[r][c] = *(const uint4*)(wv[r][c] ? dy + (((size_t)n * a.P + p) * a.Q + q) * a.C + cv : zero);
        const int hw0 = p - a.PH, ww0 = q - a.PW;  // window origin (stride 1)
        const int hc = min(hw0 + 3, a.H) - max(hw0, 0), wc = min(ww0 + 3, a.W) - max(ww0, 0);
        inv[r][c] = 1.f / (float)(count_pad ? 9 : max(hc * wc, 1));
      }
    }
#pragma unroll
    for (int u = 0; u < AVG_R; ++u) {
      const uint32_t h = hs + u;
      if (h >= (uint32_t)a.H) break;
      float acc[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
      // windows of pixel h: p = h + PH - 2 .. h + PH (ascending) = strip rows u .. u + 2; same for q
#pragma unroll
      for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if (!wv[u + r][c]) continue;
          const uint4 g4 = g[u + r][c];
          const float gf[8] = {lo_bf(g4.x), hi_bf(g4.x), lo_bf(g4.y), hi_bf(g4.y),
                               lo_bf(g4.z), hi_bf(g4.z), lo_bf(g4.w), hi_bf(g4.w)};
          const float iv = inv[u + r][c];
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += gf[e] * iv;
        }
      }
      st<8>(dx + (((size_t)n * a.H + h) * a.W + w) * a.C + cv, acc);
    }
  }
}

}  // namespace dtm
using namespace dtm;

static int pgrid(long work) {
  long b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

static int g_pool_k3s2 = 1;  // A/B knob (dtm_pool_set_k3s2): the 3x3 / stride-2 specialised stem-pool kernels
DTM_API void dtm_pool_set_k3s2(int on) { g_pool_k3s2 = on; }
static bool k3s2(const PoolArgs* a) {
  return g_pool_k3s2 && a->KH == 3 && a->KW == 3 && a->SH == 2 && a->SW == 2 && a->PH >= 0 && a->PH <= 1 &&
         a->PW >= 0 && a->PW <= 1;
}
const void* dtm_zero_chunk();  // >= 16 B of device zeros (conv_igemm.hip)

DTM_API void dtm_maxpool_fwd(const void* x, void* y, void* arg, const PoolArgs* a, void* stream) {
  long work = (long)a->N * a->P * a->Q * a->C;
  if (a->C % 8 == 0 && arg && k3s2(a) && (long)a->N * a->H * a->W * a->C < (1l << 31)) {
    const long w2 = (long)a->N * ((a->P + 1) / 2) * a->Q * (a->C / 8);
    hipLaunchKernelGGL(maxpool_bnrelu_fwd_k3s2_kernel<false>, dim3(pgrid(w2)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, (const float*)nullptr, (bf16_t*)y, (uint8_t*)arg, *a, make_fastdiv(a->C / 8),
                       make_fastdiv(a->Q), make_fastdiv((a->P + 1) / 2), (const bf16_t*)dtm_zero_chunk());
    return;
  }
  if (a->C % 8 == 0)
    hipLaunchKernelGGL(maxpool_fwd_kernel<8>, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (bf16_t*)y, (uint8_t*)arg, *a);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<1>, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (bf16_t*)y, (uint8_t*)arg, *a);
}
static void maxpool_bwd_k3s2(const void* dy, int ldy, const void* arg, void* dx, const PoolArgs* a, void* stream);
DTM_API void dtm_maxpool_bwd(const void* dy, const void* arg, void* dx, const PoolArgs* a, void* stream) {
  long work = (long)a->N * a->H * a->W * a->C;
  if (a->C % 8 == 0 && a->C / 8 <= 256 && k3s2(a) && (long)a->N * a->H * a->W * a->C < (1l << 31)) {
    maxpool_bwd_k3s2(dy, a->C, arg, dx, a, stream);
    return;
  }
  if (a->C % 8 == 0)
    hipLaunchKernelGGL(maxpool_bwd_kernel<8>, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const uint8_t*)arg, (bf16_t*)dx, *a);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<1>, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const uint8_t*)arg, (bf16_t*)dx, *a);
}
// dy read in place with a pixel pitch of ldy elements (the max-pool branch's slice of a concat gradient): 3x3 / stride 2
// only (-1 otherwise: the caller makes dy contiguous)
DTM_API int dtm_maxpool_bwd_ld(const void* dy, int ldy, const void* arg, void* dx, const PoolArgs* a, void* stream) {
  if (!(a->C % 8 == 0 && a->C / 8 <= 256 && k3s2(a) && (long)a->N * a->H * a->W * a->C < (1l << 31)) || ldy < a->C ||
      ldy % 8 || ((uintptr_t)dy & 15) || (long)a->N * a->P * a->Q * ldy >= (1l << 31))
    return -1;
  maxpool_bwd_k3s2(dy, ldy, arg, dx, a, stream);
  return 0;
}
static void maxpool_bwd_k3s2(const void* dy, int ldy, const void* arg, void* dx, const PoolArgs* a, void* stream) {
  const int cols = a->C / 8, RP = 256 / cols;  // (the BN kernel's row mapping: one row = a 2 x 2 pixel block)
  const int BH = (a->H + a->PH + 1) / 2, BW = (a->W + a->PW + 1) / 2;
  const long MB = (long)a->N * BH * BW;
  long b = MB * cols / (256 * 2);
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  long rpb = (MB + b - 1) / b;
  rpb = (rpb + RP - 1) / RP * RP;
  const int blocks = (int)((MB + rpb - 1) / rpb);
  hipLaunchKernelGGL(maxpool_bnrelu_bwd_k3s2_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)dy, (const uint8_t*)arg, (const bf16_t*)nullptr, (const float*)nullptr,
                     (bf16_t*)dx, (float*)nullptr, *a, make_fastdiv(BW), make_fastdiv(BH), 0, (int)rpb,
                     (const bf16_t*)dtm_zero_chunk(), ldy);
}
static bool k3s1(const PoolArgs* a) {
  return g_pool_k3s2 && a->KH == 3 && a->KW == 3 && a->SH == 1 && a->SW == 1 && a->PH >= 0 && a->PH <= 1 &&
         a->PW >= 0 && a->PW <= 1 && a->C % 8 == 0 && (long)a->N * a->H * a->W * a->C < (1l << 31);
}
static bool avg8(const PoolArgs* a) {  // the 32-bit-index 8-channel kernels apply
  return a->C % 8 == 0 && (long)a->N * a->H * a->W * a->C < (1l << 31) && (long)a->N * a->P * a->Q * a->C < (1l << 31);
}
static bool valid53(const PoolArgs* a) {  // the 5x5/3 VALID pool with every window in bounds (aux head)
  return a->KH == 5 && a->KW == 5 && a->SH == 3 && a->SW == 3 && a->PH == 0 && a->PW == 0 &&
         (a->P - 1) * 3 + 5 <= a->H && (a->Q - 1) * 3 + 5 <= a->W;
}
static void avgpool_bwd8(const void* dy, void* dx, const PoolArgs* a, int count_pad, int accum, void* stream) {
  const long work = (long)a->N * a->H * a->W * a->C;
  if (valid53(a)) {
    hipLaunchKernelGGL((avgpool_bwd_valid_kernel<5, 3>), dim3((unsigned)((work / 8 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)dy, (bf16_t*)dx, *a, accum, make_fastdiv(a->C / 8),
                       make_fastdiv(a->W), make_fastdiv(a->H), (int)(work / 8), (const bf16_t*)dtm_zero_chunk());
    return;
  }
  hipLaunchKernelGGL(avgpool_bwd8_kernel, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                     (bf16_t*)dx, *a, count_pad, accum, make_fastdiv(a->C / 8), make_fastdiv(a->W), make_fastdiv(a->H),
                     (int)(work / 8));
}
// dx += avgpool_bwd(dy) (-1 when the 8-channel kernel does not apply: the caller adds itself)
DTM_API int dtm_avgpool_bwd_acc(const void* dy, void* dx, const PoolArgs* a, int count_pad, void* stream) {
  if (!avg8(a) || ((uintptr_t)dy & 15) || ((uintptr_t)dx & 15)) return -1;
  avgpool_bwd8(dy, dx, a, count_pad, 1, stream);
  return 0;
}
DTM_API void dtm_avgpool_fwd(const void* x, void* y, const PoolArgs* a, int count_pad, void* stream) {
  long work = (long)a->N * a->P * a->Q * a->C;
  if (k3s1(a)) {
    const int PR = (a->P + AVG_R - 1) / AVG_R;
    hipLaunchKernelGGL(avgpool_fwd_k3s1_kernel, dim3(pgrid((long)a->N * PR * a->Q * (a->C / 8))), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y, *a, count_pad, make_fastdiv(a->C / 8),
                       make_fastdiv(a->Q), make_fastdiv(PR), (const bf16_t*)dtm_zero_chunk());
    return;
  }
  if (avg8(a) && valid53(a))
    hipLaunchKernelGGL(avgpool_fwd_valid_kernel<5>, dim3((unsigned)((work / 8 + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y, *a, make_fastdiv(a->C / 8),
                       make_fastdiv(a->Q), make_fastdiv(a->P), (int)(work / 8));
  else if (avg8(a))
    hipLaunchKernelGGL(avgpool_fwd8_kernel, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (bf16_t*)y, *a, count_pad, make_fastdiv(a->C / 8), make_fastdiv(a->Q), make_fastdiv(a->P),
                       (int)(work / 8));
  else if (a->C % 8 == 0)
    hipLaunchKernelGGL(avgpool_fwd_kernel<8>, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (bf16_t*)y, *a, count_pad);
  else
    hipLaunchKernelGGL(avgpool_fwd_kernel<1>, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (bf16_t*)y, *a, count_pad);
}
DTM_API void dtm_avgpool_bwd(const void* dy, void* dx, const PoolArgs* a, int count_pad, void* stream) {
  long work = (long)a->N * a->H * a->W * a->C;
  if (k3s1(a)) {
    const int HR = (a->H + AVG_R - 1) / AVG_R;
    hipLaunchKernelGGL(avgpool_bwd_k3s1_kernel, dim3(pgrid((long)a->N * HR * a->W * (a->C / 8))), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)dy, (bf16_t*)dx, *a, count_pad, make_fastdiv(a->C / 8),
                       make_fastdiv(a->W), make_fastdiv(HR), (const bf16_t*)dtm_zero_chunk());
    return;
  }
  if (avg8(a))
    avgpool_bwd8(dy, dx, a, count_pad, 0, stream);
  else if (a->C % 8 == 0)
    hipLaunchKernelGGL(avgpool_bwd_kernel<8>, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (bf16_t*)dx, *a, count_pad);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel<1>, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (bf16_t*)dx, *a, count_pad);
}
static bool gavg8(const void* x, const void* y, long N, long HW, int C) {
  return C % 8 == 0 && !((uintptr_t)x & 15) && !((uintptr_t)y & 15) && N * HW * C < (1l << 31) && N <= 65535;
}
template <typename TO>
static void global_avg_fwd(const void* x, TO* y, int N, int HW, int C, void* stream) {
  if (gavg8(x, y, N, HW, C))
    hipLaunchKernelGGL(global_avg_fwd8_kernel<TO>, dim3((C / 8 + 63) / 64, N), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, y, HW, C);
  else
    hipLaunchKernelGGL(global_avg_fwd_kernel<TO>, dim3((C + 255) / 256, N), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, y, HW, C);
}
template <typename TI>
static void global_avg_bwd(const TI* dy, void* dx, int N, int HW, int C, void* stream) {
  if (gavg8(dy, dx, N, HW, C)) {
    const int total = N * HW * (C / 8);
    hipLaunchKernelGGL(global_avg_bwd8_kernel<TI>, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, dy,
                       (bf16_t*)dx, C, make_fastdiv(C / 8), make_fastdiv(HW), total, 1.f / (float)HW);
  } else {
    hipLaunchKernelGGL(global_avg_bwd_kernel<TI>, dim3(pgrid((long)N * HW * C)), dim3(256), 0, (hipStream_t)stream,
                       dy, (bf16_t*)dx, N, HW, C);
  }
}
DTM_API void dtm_global_avg_fwd(const void* x, float* y, int N, int HW, int C, void* stream) {
  global_avg_fwd<float>(x, y, N, HW, C, stream);
}
DTM_API void dtm_global_avg_bwd(const float* dy, void* dx, int N, int HW, int C, void* stream) {
  global_avg_bwd<float>(dy, dx, N, HW, C, stream);
}
// bf16 output / bf16 incoming gradient (the pooled features feed a bf16 logits layer)
DTM_API void dtm_global_avg_fwd_bf16(const void* x, void* y, int N, int HW, int C, void* stream) {
  global_avg_fwd<bf16_t>(x, (bf16_t*)y, N, HW, C, stream);
}
DTM_API void dtm_global_avg_bwd_bf16(const void* dy, void* dx, int N, int HW, int C, void* stream) {
  global_avg_bwd<bf16_t>((const bf16_t*)dy, dx, N, HW, C, stream);
}

// y = maxpool(relu(x*scale + shift)) with a uint8 argmax per output element (ss = [scale; shift; ...])
DTM_API int dtm_maxpool_bnrelu_fwd(const void* x, const float* ss, void* y, void* arg, const PoolArgs* a, void* stream) {
  if (a->C % 8 || a->KH * a->KW > 255 || (long)a->N * a->H * a->W * a->C >= (1l << 31)) return -1;
  if (k3s2(a)) {
    const long work = (long)a->N * ((a->P + 1) / 2) * a->Q * (a->C / 8);
    hipLaunchKernelGGL(maxpool_bnrelu_fwd_k3s2_kernel<true>, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, ss, (bf16_t*)y, (uint8_t*)arg, *a, make_fastdiv(a->C / 8), make_fastdiv(a->Q),
                       make_fastdiv((a->P + 1) / 2), (const bf16_t*)dtm_zero_chunk());
    return 0;
  }
  const long work = (long)a->N * a->P * a->Q * (a->C / 8);
  hipLaunchKernelGGL(maxpool_bnrelu_fwd_kernel, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     ss, (bf16_t*)y, (uint8_t*)arg, *a, make_fastdiv(a->C / 8), make_fastdiv(a->Q), make_fastdiv(a->P));
  return 0;
}

// dx = [x*scale+shift > 0] * scale * maxpool_grad(dy);  sums[0..1][C] += (sum g*x, sum g)
DTM_API int dtm_maxpool_bnrelu_bwd(const void* dy, const void* arg, const void* x, const float* ss, void* dx,
                                   float* sums, const PoolArgs* a, int unscaled, void* stream) {
  if (a->C % 8 || a->C / 8 > 256 || (long)a->N * a->H * a->W * a->C >= (1l << 31)) return -1;
  if ((a->KH + a->SH - 1) / a->SH > 3 || (a->KW + a->SW - 1) / a->SW > 3) return -2;
  const int cols = a->C / 8, RP = 256 / cols;
  if (k3s2(a)) {  // one row = a 2 x 2 block of input pixels
    const int BH = (a->H + a->PH + 1) / 2, BW = (a->W + a->PW + 1) / 2;
    const long MB = (long)a->N * BH * BW;
    long b = MB * cols / (256 * 2);
    if (b < 1) b = 1;
    if (b > 2048) b = 2048;
    long rpb = (MB + b - 1) / b;
    rpb = (rpb + RP - 1) / RP * RP;
    const int blocks = (int)((MB + rpb - 1) / rpb);
    float* ws = dtm_ws_get_stream((size_t)blocks * 2 * a->C, (hipStream_t)stream);
    if (!ws) return -4;
    hipLaunchKernelGGL(maxpool_bnrelu_bwd_k3s2_kernel<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dy, (const uint8_t*)arg, (const bf16_t*)x, ss, (bf16_t*)dx, ws, *a,
                       make_fastdiv(BW), make_fastdiv(BH), unscaled, (int)rpb, (const bf16_t*)dtm_zero_chunk(), a->C);
    dtm_reduce_rows(ws, blocks, 2 * a->C, 2 * a->C, sums, (hipStream_t)stream);
    return 0;
  }
  const long M = (long)a->N * a->H * a->W;
  long b = M * cols / (256 * 8);
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  long rpb = (M + b - 1) / b;
  rpb = (rpb + RP - 1) / RP * RP;
  const int blocks = (int)((M + rpb - 1) / rpb);
  float* ws = dtm_ws_get_stream((size_t)blocks * 2 * a->C, (hipStream_t)stream);
  if (!ws) return -4;
  const int wm = max((a->KH + a->SH - 1) / a->SH, (a->KW + a->SW - 1) / a->SW);
  if (wm <= 2)
    hipLaunchKernelGGL((maxpool_bnrelu_bwd_kernel<2, 2>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dy, (const uint8_t*)arg, (const bf16_t*)x, ss, (bf16_t*)dx, ws, *a,
                       make_fastdiv(a->W), make_fastdiv(a->H), unscaled, (int)rpb);
  else
    hipLaunchKernelGGL((maxpool_bnrelu_bwd_kernel<3, 1>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dy, (const uint8_t*)arg, (const bf16_t*)x, ss, (bf16_t*)dx, ws, *a,
                       make_fastdiv(a->W), make_fastdiv(a->H), unscaled, (int)rpb);
  dtm_reduce_rows(ws, blocks, 2 * a->C, 2 * a->C, sums, (hipStream_t)stream);
  return 0;
}
