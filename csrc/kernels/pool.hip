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

// global mean over H*W: x[N][HW][C] -> y[N][C] (fp32 out, feeds the logits GEMM)
__global__ __launch_bounds__(256) void global_avg_fwd_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, int HW,
                                                             int C) {
  const int n = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const bf16_t* p = x + (long)n * HW * C + c;
  float s = 0.f;
  for (int i = 0; i < HW; ++i) s += bf2f(p[(long)i * C]);
  y[(long)n * C + c] = s / (float)HW;
}
__global__ __launch_bounds__(256) void global_avg_bwd_kernel(const float* __restrict__ dy, bf16_t* __restrict__ dx, int N,
                                                             int HW, int C) {
  const long total = (long)N * HW * C;
  const float inv = 1.f / (float)HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c = i % C;
    long n = i / ((long)HW * C);
    dx[i] = f2bf(dy[n * C + c] * inv);
  }
}

}  // namespace dtm
using namespace dtm;

static int pgrid(long work) {
  long b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

DTM_API void dtm_maxpool_fwd(const void* x, void* y, void* arg, const PoolArgs* a, void* stream) {
  long work = (long)a->N * a->P * a->Q * a->C;
  if (a->C % 8 == 0)
    hipLaunchKernelGGL(maxpool_fwd_kernel<8>, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (bf16_t*)y, (uint8_t*)arg, *a);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<1>, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (bf16_t*)y, (uint8_t*)arg, *a);
}
DTM_API void dtm_maxpool_bwd(const void* dy, const void* arg, void* dx, const PoolArgs* a, void* stream) {
  long work = (long)a->N * a->H * a->W * a->C;
  if (a->C % 8 == 0)
    hipLaunchKernelGGL(maxpool_bwd_kernel<8>, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const uint8_t*)arg, (bf16_t*)dx, *a);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<1>, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const uint8_t*)arg, (bf16_t*)dx, *a);
}
DTM_API void dtm_avgpool_fwd(const void* x, void* y, const PoolArgs* a, int count_pad, void* stream) {
  long work = (long)a->N * a->P * a->Q * a->C;
  if (a->C % 8 == 0)
    hipLaunchKernelGGL(avgpool_fwd_kernel<8>, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (bf16_t*)y, *a, count_pad);
  else
    hipLaunchKernelGGL(avgpool_fwd_kernel<1>, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (bf16_t*)y, *a, count_pad);
}
DTM_API void dtm_avgpool_bwd(const void* dy, void* dx, const PoolArgs* a, int count_pad, void* stream) {
  long work = (long)a->N * a->H * a->W * a->C;
  if (a->C % 8 == 0)
    hipLaunchKernelGGL(avgpool_bwd_kernel<8>, dim3(pgrid(work / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (bf16_t*)dx, *a, count_pad);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel<1>, dim3(pgrid(work)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (bf16_t*)dx, *a, count_pad);
}
DTM_API void dtm_global_avg_fwd(const void* x, float* y, int N, int HW, int C, void* stream) {
  hipLaunchKernelGGL(global_avg_fwd_kernel, dim3((C + 255) / 256, N), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, y, HW, C);
}
DTM_API void dtm_global_avg_bwd(const float* dy, void* dx, int N, int HW, int C, void* stream) {
  hipLaunchKernelGGL(global_avg_bwd_kernel, dim3(pgrid((long)N * HW * C)), dim3(256), 0, (hipStream_t)stream, dy,
                     (bf16_t*)dx, N, HW, C);
}
