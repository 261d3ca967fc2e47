// Local response normalisation across channels (NHWC), TF semantics (reference
// cnn/cifar10.py:231,245 tf.nn.lrn(depth_radius=4, bias=1, alpha=0.001/9, beta=0.75)):
//   s_c = bias + alpha * sum_{|c'-c|<=r} x_c'^2 ;  y_c = x_c * s_c^-beta
//   dx_i = dy_i s_i^-beta - 2 alpha beta x_i sum_{|j-i|<=r} dy_j y_j / s_j
// One lane per (pixel, channel); the pixel's channel vector is staged in LDS (C <= 1024).
#include "common.h"

namespace dtm {
template <bool BWD>
__global__ __launch_bounds__(256) void lrn_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                  bf16_t* __restrict__ out, long npix, int C, int r, float bias,
                                                  float alpha, float beta) {
  extern __shared__ float sm[];  // per block: PPB pixels x C (x, and for bwd dy*y/s)
  const int ppb = max(1, 256 / C);
  const long p0 = (long)blockIdx.x * ppb;
  float* xs = sm;
  float* ts = sm + ppb * C;
  for (int i = threadIdx.x; i < ppb * C; i += blockDim.x) {
    long p = p0 + i / C;
    xs[i] = p < npix ? bf2f(x[p * C + i % C]) : 0.f;
  }
  __syncthreads();
  if (BWD) {
    for (int i = threadIdx.x; i < ppb * C; i += blockDim.x) {
      long p = p0 + i / C;
      int c = i % C, b = i - c;
      float s = 0.f;
      for (int k = max(0, c - r); k <= min(C - 1, c + r); ++k) s += xs[b + k] * xs[b + k];
      s = bias + alpha * s;
      float yv = xs[i] * __powf(s, -beta);
      ts[i] = p < npix ? bf2f(dy[p * C + c]) * yv / s : 0.f;
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < ppb * C; i += blockDim.x) {
    long p = p0 + i / C;
    if (p >= npix) continue;
    int c = i % C, b = i - c;
    float s = 0.f;
    for (int k = max(0, c - r); k <= min(C - 1, c + r); ++k) s += xs[b + k] * xs[b + k];
    s = bias + alpha * s;
    if (!BWD) {
      out[p * C + c] = f2bf(xs[i] * __powf(s, -beta));
    } else {
      float acc = 0.f;
      for (int k = max(0, c - r); k <= min(C - 1, c + r); ++k) acc += ts[b + k];
      float g = bf2f(dy[p * C + c]) * __powf(s, -beta) - 2.f * alpha * beta * xs[i] * acc;
      out[p * C + c] = f2bf(g);
    }
  }
}
}  // namespace dtm
using namespace dtm;

DTM_API int dtm_lrn(const void* x, const void* dy, void* out, long npix, int C, int r, float bias, float alpha,
                    float beta, int backward, void* stream) {
  if (C > 1024) return -1;
  int ppb = C >= 256 ? 1 : 256 / C;
  long blocks = (npix + ppb - 1) / ppb;
  size_t sm = (size_t)ppb * C * sizeof(float) * (backward ? 2 : 1);
  if (backward)
    hipLaunchKernelGGL(lrn_kernel<true>, dim3((unsigned)blocks), dim3(256), sm, (hipStream_t)stream,
                       (const bf16_t*)x, (const bf16_t*)dy, (bf16_t*)out, npix, C, r, bias, alpha, beta);
  else
    hipLaunchKernelGGL(lrn_kernel<false>, dim3((unsigned)blocks), dim3(256), sm, (hipStream_t)stream,
                       (const bf16_t*)x, nullptr, (bf16_t*)out, npix, C, r, bias, alpha, beta);
  return 0;
}
