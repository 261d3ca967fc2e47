// Depthwise 2-D convolution (NHWC, TF weight layout [R][S][C][M]) - SURVEY.md K16
// (slim.separable_conv2d / depthwise_conv2d in MobileNet v1/v2, NASNet, Inception-v2).
// Bandwidth-bound op: 8 channels per lane (16-B loads) for depth_multiplier 1; scalar lanes for M > 1.
//   fwd:   y[n,p,q,c*M+m] = sum_{r,s} x[n, p*st-ph+r*d, q*st-pw+s*d, c] * w[r,s,c,m]
//   dgrad: gather over the taps that touched (h, w)
//   wgrad: per-block partial sums over pixels for all R*S taps, then the two-stage row reduction.
#include "common.h"

namespace dtm {

struct DwArgs {
  int N, H, W, C, M, R, S, P, Q, stride, ph, pw, dil;
};

__device__ __forceinline__ void ld8(const bf16_t* p, float* f) {
  uint4 u = *(const uint4*)p;
  f[0] = lo_bf(u.x); f[1] = hi_bf(u.x); f[2] = lo_bf(u.y); f[3] = hi_bf(u.y);
  f[4] = lo_bf(u.z); f[5] = hi_bf(u.z); f[6] = lo_bf(u.w); f[7] = hi_bf(u.w);
}
__device__ __forceinline__ void st8(bf16_t* p, const float* f) {
  *(uint4*)p = make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
}

__global__ __launch_bounds__(256) void dw_fwd8(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                               bf16_t* __restrict__ y, DwArgs a) {
  const int cols = a.C / 8;
  const long total = (long)a.N * a.P * a.Q * cols;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c0 = (int)(i % cols) * 8;
    long o = i / cols;
    const int q = o % a.Q;
    long t = o / a.Q;
    const int p = t % a.P, n = (int)(t / a.P);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < a.R; ++r) {
      int h = p * a.stride - a.ph + r * a.dil;
      if (h < 0 || h >= a.H) continue;
      for (int s = 0; s < a.S; ++s) {
        int ww = q * a.stride - a.pw + s * a.dil;
        if (ww < 0 || ww >= a.W) continue;
        float xv[8];
        ld8(x + (((long)n * a.H + h) * a.W + ww) * a.C + c0, xv);
        const float* wp = w + ((long)r * a.S + s) * a.C + c0;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += xv[e] * wp[e];
      }
    }
    st8(y + o * a.C + c0, acc);
  }
}

__global__ __launch_bounds__(256) void dw_dgrad8(const bf16_t* __restrict__ dy, const float* __restrict__ w,
                                                 bf16_t* __restrict__ dx, DwArgs a) {
  const int cols = a.C / 8;
  const long total = (long)a.N * a.H * a.W * cols;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c0 = (int)(i % cols) * 8;
    long o = i / cols;
    const int ww = o % a.W;
    long t = o / a.W;
    const int h = t % a.H, n = (int)(t / a.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < a.R; ++r) {
      int ph = h + a.ph - r * a.dil;
      if (ph < 0 || ph % a.stride) continue;
      int p = ph / a.stride;
      if (p >= a.P) continue;
      for (int s = 0; s < a.S; ++s) {
        int pq = ww + a.pw - s * a.dil;
        if (pq < 0 || pq % a.stride) continue;
        int q = pq / a.stride;
        if (q >= a.Q) continue;
        float g[8];
        ld8(dy + (((long)n * a.P + p) * a.Q + q) * a.C + c0, g);
        const float* wp = w + ((long)r * a.S + s) * a.C + c0;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += g[e] * wp[e];
      }
    }
    st8(dx + o * a.C + c0, acc);
  }
}

// each block: a range of output pixels, 256 lanes = (C/8 columns) x (256/(C/8) row lanes) when C/8 <= 256
// partial row per block: [R*S*C] floats
__global__ __launch_bounds__(256) void dw_wgrad8(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                 float* __restrict__ ws, DwArgs a, int pix_per_block) {
  extern __shared__ float red[];  // [256][8] per tap, reused tap by tap
  const int cols = a.C / 8, RP = 256 / cols, t = threadIdx.x;
  const int c0 = (t % cols) * 8, rl = t / cols;
  const long M = (long)a.N * a.P * a.Q;
  const long m0 = (long)blockIdx.x * pix_per_block, m1 = min(M, m0 + pix_per_block);
  float* out = ws + (size_t)blockIdx.x * a.R * a.S * a.C;
  for (int r = 0; r < a.R; ++r) {
    for (int s = 0; s < a.S; ++s) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (rl < RP) {
        for (long m = m0 + rl; m < m1; m += RP) {
          const int q = m % a.Q;
          long tt = m / a.Q;
          const int p = tt % a.P, n = (int)(tt / a.P);
          int h = p * a.stride - a.ph + r * a.dil, ww = q * a.stride - a.pw + s * a.dil;
          if (h < 0 || h >= a.H || ww < 0 || ww >= a.W) continue;
          float xv[8], g[8];
          ld8(x + (((long)n * a.H + h) * a.W + ww) * a.C + c0, xv);
          ld8(dy + m * a.C + c0, g);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += xv[e] * g[e];
        }
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) red[t * 8 + e] = acc[e];
      __syncthreads();
      if (t < cols) {
        float sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < RP; ++k)
#pragma unroll
          for (int e = 0; e < 8; ++e) sum[e] += red[(k * cols + t) * 8 + e];
#pragma unroll
        for (int e = 0; e < 8; ++e) out[((size_t)r * a.S + s) * a.C + c0 + e] = sum[e];
      }
    }
  }
}

// generic scalar path (any C, depth multiplier M): one lane per output element
__global__ void dw_fwd_generic(const bf16_t* __restrict__ x, const float* __restrict__ w, bf16_t* __restrict__ y,
                               DwArgs a) {
  const int CM = a.C * a.M;
  const long total = (long)a.N * a.P * a.Q * CM;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int cm = i % CM, c = cm / a.M, m = cm % a.M;
    long o = i / CM;
    const int q = o % a.Q;
    long t = o / a.Q;
    const int p = t % a.P, n = (int)(t / a.P);
    float acc = 0.f;
    for (int r = 0; r < a.R; ++r) {
      int h = p * a.stride - a.ph + r * a.dil;
      if (h < 0 || h >= a.H) continue;
      for (int s = 0; s < a.S; ++s) {
        int ww = q * a.stride - a.pw + s * a.dil;
        if (ww < 0 || ww >= a.W) continue;
        acc += bf2f(x[(((long)n * a.H + h) * a.W + ww) * a.C + c]) * w[(((long)r * a.S + s) * a.C + c) * a.M + m];
      }
    }
    y[i] = f2bf(acc);
  }
}

__global__ void dw_dgrad_generic(const bf16_t* __restrict__ dy, const float* __restrict__ w, bf16_t* __restrict__ dx,
                                 DwArgs a) {
  const long total = (long)a.N * a.H * a.W * a.C;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = i % a.C;
    long o = i / a.C;
    const int ww = o % a.W;
    long t = o / a.W;
    const int h = t % a.H, n = (int)(t / a.H);
    float acc = 0.f;
    for (int r = 0; r < a.R; ++r) {
      int ph = h + a.ph - r * a.dil;
      if (ph < 0 || ph % a.stride || ph / a.stride >= a.P) continue;
      for (int s = 0; s < a.S; ++s) {
        int pq = ww + a.pw - s * a.dil;
        if (pq < 0 || pq % a.stride || pq / a.stride >= a.Q) continue;
        long base = (((long)n * a.P + ph / a.stride) * a.Q + pq / a.stride) * a.C * a.M + (long)c * a.M;
        for (int m = 0; m < a.M; ++m) acc += bf2f(dy[base + m]) * w[(((long)r * a.S + s) * a.C + c) * a.M + m];
      }
    }
    dx[i] = f2bf(acc);
  }
}

__global__ void dw_wgrad_generic(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, float* __restrict__ dw,
                                 DwArgs a) {
  // one block per (r, s, c, m) weight; lanes stride over output pixels
  __shared__ float red[256];
  const int idx = blockIdx.x;
  const int m = idx % a.M, c = (idx / a.M) % a.C, s = (idx / (a.M * a.C)) % a.S, r = idx / (a.M * a.C * a.S);
  const long Mp = (long)a.N * a.P * a.Q;
  float acc = 0.f;
  for (long o = threadIdx.x; o < Mp; o += 256) {
    const int q = o % a.Q;
    long t = o / a.Q;
    const int p = t % a.P, n = (int)(t / a.P);
    int h = p * a.stride - a.ph + r * a.dil, ww = q * a.stride - a.pw + s * a.dil;
    if (h < 0 || h >= a.H || ww < 0 || ww >= a.W) continue;
    acc += bf2f(x[(((long)n * a.H + h) * a.W + ww) * a.C + c]) * bf2f(dy[o * a.C * a.M + (long)c * a.M + m]);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) dw[idx] += red[0];
}

}  // namespace dtm
using namespace dtm;

static int dgrid(long work) {
  long b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}
static bool fast8(const DwArgs& a) { return a.M == 1 && a.C % 8 == 0 && a.C / 8 <= 256 && 256 % (a.C / 8) == 0; }

// w: fp32 [R][S][C][M]
DTM_API int dtm_depthwise_fwd(const void* x, const float* w, void* y, const DwArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (fast8(*a))
    hipLaunchKernelGGL(dw_fwd8, dim3(dgrid((long)a->N * a->P * a->Q * a->C / 8)), dim3(256), 0, st, (const bf16_t*)x,
                       w, (bf16_t*)y, *a);
  else
    hipLaunchKernelGGL(dw_fwd_generic, dim3(dgrid((long)a->N * a->P * a->Q * a->C * a->M)), dim3(256), 0, st,
                       (const bf16_t*)x, w, (bf16_t*)y, *a);
  return 0;
}

DTM_API int dtm_depthwise_dgrad(const void* dy, const float* w, void* dx, const DwArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (fast8(*a))
    hipLaunchKernelGGL(dw_dgrad8, dim3(dgrid((long)a->N * a->H * a->W * a->C / 8)), dim3(256), 0, st,
                       (const bf16_t*)dy, w, (bf16_t*)dx, *a);
  else
    hipLaunchKernelGGL(dw_dgrad_generic, dim3(dgrid((long)a->N * a->H * a->W * a->C)), dim3(256), 0, st,
                       (const bf16_t*)dy, w, (bf16_t*)dx, *a);
  return 0;
}

// dw (fp32, [R][S][C][M]) += gradient
DTM_API int dtm_depthwise_wgrad(const void* x, const void* dy, float* dw, const DwArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (fast8(*a)) {
    long M = (long)a->N * a->P * a->Q;
    int blocks = (int)((M + 2047) / 2048);
    if (blocks > 1024) blocks = 1024;
    int ppb = (int)((M + blocks - 1) / blocks);
    int width = a->R * a->S * a->C;
    float* ws = dtm_ws_get_stream((size_t)blocks * width, st);
    if (!ws) return -4;
    hipLaunchKernelGGL(dw_wgrad8, dim3(blocks), dim3(256), 256 * 8 * sizeof(float), st, (const bf16_t*)x,
                       (const bf16_t*)dy, ws, *a, ppb);
    dtm_reduce_rows(ws, blocks, width, width, dw, st);
  } else {
    hipLaunchKernelGGL(dw_wgrad_generic, dim3(a->R * a->S * a->C * a->M), dim3(256), 0, st, (const bf16_t*)x,
                       (const bf16_t*)dy, dw, *a);
  }
  return 0;
}
