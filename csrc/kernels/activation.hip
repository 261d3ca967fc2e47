// Activations, instance normalisation and reflect padding for the model-zoo call sites that are not
// fused into a conv / BatchNorm kernel:
//   * ReLU6 (MobileNet v1/v2: reference vgg/nets/mobilenet_v1.py:428-472 via slim arg_scope
//     activation_fn=tf.nn.relu6), leaky ReLU (DCGAN discriminator, vgg/nets/dcgan.py:89), ELU;
//   * instance normalisation + reflect padding (CycleGAN generator, vgg/nets/cyclegan.py:66-117,
//     tf.contrib.layers.instance_norm / tf.pad(..., 'REFLECT')).
// NHWC, bf16 or fp32 storage, fp32 math.  Elementwise kernels move 8 elements (16 B of bf16) per
// thread.  Instance norm: one block per (sample, 64-channel group); 8 chunk-lanes x 32 pixel-lanes
// stride over H*W with shifted sums (x - x[first pixel]) so a large mean does not cancel the variance.
#include "common.h"

namespace dtm {

enum ActKind { ACT_RELU6 = 0, ACT_LEAKY = 1, ACT_ELU = 2 };

__device__ __forceinline__ float act_f(float x, int kind, float alpha) {
  if (kind == ACT_RELU6) return fminf(fmaxf(x, 0.f), 6.f);
  if (kind == ACT_LEAKY) return x > 0.f ? x : alpha * x;
  return x > 0.f ? x : expm1f(x);
}
// derivative from the forward input x (TF: relu6 grad is 1 on (0, 6), leaky alpha below 0, elu exp(x))
__device__ __forceinline__ float act_d(float x, int kind, float alpha) {
  if (kind == ACT_RELU6) return (x > 0.f && x < 6.f) ? 1.f : 0.f;
  if (kind == ACT_LEAKY) return x > 0.f ? 1.f : alpha;
  return x > 0.f ? 1.f : expf(x);
}

template <bool BF16>
__device__ __forceinline__ void load8(const void* p, long i, long n, float (&v)[8]) {
  if (BF16) {
    const bf16_t* x = (const bf16_t*)p;
    if (i + 8 <= n) {
      const uint4 u = *(const uint4*)(x + i);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf(w[j]); v[2 * j + 1] = hi_bf(w[j]); }
    } else {
      for (int j = 0; j < 8; ++j) v[j] = i + j < n ? bf2f(x[i + j]) : 0.f;
    }
  } else {
    const float* x = (const float*)p;
    if (i + 8 <= n) {
      const float4 a = *(const float4*)(x + i), b = *(const float4*)(x + i + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      for (int j = 0; j < 8; ++j) v[j] = i + j < n ? x[i + j] : 0.f;
    }
  }
}

template <bool BF16>
__device__ __forceinline__ void store8(void* p, long i, long n, const float (&v)[8]) {
  if (BF16) {
    bf16_t* y = (bf16_t*)p;
    if (i + 8 <= n) {
      *(uint4*)(y + i) = make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
    } else {
      for (int j = 0; j < 8; ++j)
        if (i + j < n) y[i + j] = f2bf(v[j]);
    }
  } else {
    float* y = (float*)p;
    if (i + 8 <= n) {
      *(float4*)(y + i) = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(y + i + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      for (int j = 0; j < 8; ++j)
        if (i + j < n) y[i + j] = v[j];
    }
  }
}

template <bool BF16>
__global__ __launch_bounds__(256) void act_fwd_kernel(const void* __restrict__ x, void* __restrict__ y, long n,
                                                      int kind, float alpha) {
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += (long)gridDim.x * 256 * 8) {
    float v[8];
    load8<BF16>(x, i, n, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_f(v[j], kind, alpha);
    store8<BF16>(y, i, n, v);
  }
}

template <bool BF16>
__global__ __launch_bounds__(256) void act_bwd_kernel(const void* __restrict__ dy, const void* __restrict__ x,
                                                      void* __restrict__ dx, long n, int kind, float alpha) {
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += (long)gridDim.x * 256 * 8) {
    float g[8], v[8];
    load8<BF16>(dy, i, n, g);
    load8<BF16>(x, i, n, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= act_d(v[j], kind, alpha);
    store8<BF16>(dx, i, n, g);
  }
}

// ------------------------------------------------------------------------------------------
// instance norm.  stats[n][c] = (mean, rstd) saved for backward.
template <bool BF16>
__device__ __forceinline__ void load_chunk(const void* base, size_t off, float (&v)[8]) {
  load8<BF16>(base, (long)off, (long)off + 8, v);
}

// red: [2][32][64] floats; lanes: ch = tid & 7 (8-channel chunk of the 64-channel group), pl = tid >> 3
template <bool BF16>
__global__ __launch_bounds__(256) void instnorm_fwd_kernel(const void* __restrict__ x, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, void* __restrict__ y,
                                                           float* __restrict__ stats, int HW, int C, float eps,
                                                           int relu) {
  __shared__ float red[2][32][64];
  const int n = blockIdx.y, cg = blockIdx.x * 64;
  const int ch = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int c = cg + ch * 8;
  const bool cin = c < C;
  const size_t base = (size_t)n * HW * C;
  float shift[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (cin) load_chunk<BF16>(x, base + c, shift);  // pixel 0 of this (n, chunk): the shift K
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (cin) {
    for (int p = pl; p < HW; p += 32) {
      float v[8];
      load_chunk<BF16>(x, base + (size_t)p * C + c, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[e] - shift[e];
        s[e] += d;
        q[e] = fmaf(d, d, q[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][pl][ch * 8 + e] = s[e]; red[1][pl][ch * 8 + e] = q[e]; }
  __syncthreads();
  __shared__ float mr[2][64];
  if (threadIdx.x < 64) {
    const int cc = threadIdx.x;
    float ts = 0.f, tq = 0.f;
    for (int r = 0; r < 32; ++r) { ts += red[0][r][cc]; tq += red[1][r][cc]; }
    const float inv = 1.f / (float)HW;
    const float dm = ts * inv;
    const float var = fmaxf(tq * inv - dm * dm, 0.f);
    float k = 0.f;
    if (cg + cc < C) {
      float sh[8];
      load_chunk<BF16>(x, base + cg + (cc & ~7), sh);
      k = sh[cc & 7];
    }
    mr[0][cc] = k + dm;
    mr[1][cc] = rsqrtf(var + eps);
    if (cg + cc < C) {
      stats[((size_t)n * C + cg + cc) * 2] = mr[0][cc];
      stats[((size_t)n * C + cg + cc) * 2 + 1] = mr[1][cc];
    }
  }
  __syncthreads();
  if (!cin) return;
  float a[8], b[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float gm = gamma ? gamma[c + e] : 1.f, bt = beta ? beta[c + e] : 0.f;
    a[e] = mr[1][ch * 8 + e] * gm;
    b[e] = bt - mr[0][ch * 8 + e] * a[e];
  }
  for (int p = pl; p < HW; p += 32) {
    float v[8];
    const size_t off = base + (size_t)p * C + c;
    load_chunk<BF16>(x, off, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = fmaf(v[e], a[e], b[e]);
      if (relu) v[e] = fmaxf(v[e], 0.f);
    }
    store8<BF16>(y, (long)off, (long)off + 8, v);
  }
}

// dy here is the gradient w.r.t. the affine output (the host applies the fused ReLU mask first).
// sums[n][c] = (sum dy, sum dy*xhat) -> dgamma / dbeta reduced over n on the host side.
template <bool BF16>
__global__ __launch_bounds__(256) void instnorm_bwd_kernel(const void* __restrict__ x, const void* __restrict__ dy,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ stats, void* __restrict__ dx,
                                                           float* __restrict__ sums, int HW, int C) {
  __shared__ float red[2][32][64];
  __shared__ float mr[2][64];
  const int n = blockIdx.y, cg = blockIdx.x * 64;
  const int ch = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int c = cg + ch * 8;
  const bool cin = c < C;
  const size_t base = (size_t)n * HW * C;
  float mean[8], rstd[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] = cin ? stats[((size_t)n * C + c + e) * 2] : 0.f;
    rstd[e] = cin ? stats[((size_t)n * C + c + e) * 2 + 1] : 0.f;
  }
  float sg[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, sgx[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (cin) {
    for (int p = pl; p < HW; p += 32) {
      float v[8], g[8];
      const size_t off = base + (size_t)p * C + c;
      load_chunk<BF16>(x, off, v);
      load_chunk<BF16>(dy, off, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sg[e] += g[e];
        sgx[e] = fmaf(g[e], (v[e] - mean[e]) * rstd[e], sgx[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][pl][ch * 8 + e] = sg[e]; red[1][pl][ch * 8 + e] = sgx[e]; }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int cc = threadIdx.x;
    float a = 0.f, b = 0.f;
    for (int r = 0; r < 32; ++r) { a += red[0][r][cc]; b += red[1][r][cc]; }
    mr[0][cc] = a;
    mr[1][cc] = b;
    if (cg + cc < C) {
      sums[((size_t)n * C + cg + cc) * 2] = a;
      sums[((size_t)n * C + cg + cc) * 2 + 1] = b;
    }
  }
  __syncthreads();
  if (!cin) return;
  const float inv = 1.f / (float)HW;
  float k[8], mg[8], mgx[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    k[e] = rstd[e] * (gamma ? gamma[c + e] : 1.f);
    mg[e] = mr[0][ch * 8 + e] * inv;
    mgx[e] = mr[1][ch * 8 + e] * inv;
  }
  for (int p = pl; p < HW; p += 32) {
    float v[8], g[8];
    const size_t off = base + (size_t)p * C + c;
    load_chunk<BF16>(x, off, v);
    load_chunk<BF16>(dy, off, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (v[e] - mean[e]) * rstd[e];
      g[e] = k[e] * (g[e] - mg[e] - xh * mgx[e]);
    }
    store8<BF16>(dx, (long)off, (long)off + 8, g);
  }
}

// ------------------------------------------------------------------------------------------
// tf.pad(..., 'REFLECT') on NHWC: the edge row/column is not repeated (index -1 -> 1).
__device__ __forceinline__ int reflect_idx(int i, int n) {
  if (i < 0) return -i;
  if (i >= n) return 2 * (n - 1) - i;
  return i;
}

// one thread per 8-channel chunk of an output pixel (C % 8 == 0)
template <bool BF16>
__global__ __launch_bounds__(256) void reflect_pad_fwd_kernel(const void* __restrict__ x, void* __restrict__ y, int N,
                                                              int H, int W, int C, int Ho, int Wo, int top, int left) {
  const int cpp = C / 8;
  const long total = (long)N * Ho * Wo * cpp;
  for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const int cc = (int)(t % cpp);
    long r = t / cpp;
    const int ow = (int)(r % Wo);
    r /= Wo;
    const int oh = (int)(r % Ho);
    const int n = (int)(r / Ho);
    const int ih = reflect_idx(oh - top, H), iw = reflect_idx(ow - left, W);
    float v[8];
    load_chunk<BF16>(x, (((size_t)n * H + ih) * W + iw) * C + cc * 8, v);
    store8<BF16>(y, (long)t * 8, (long)t * 8 + 8, v);
  }
}

// gradient as a gather (deterministic, no atomics): every input row h receives from the output rows
// oh = h + top, top - h (top reflection, 0 < h <= top) and top + 2(H-1) - h (bottom reflection,
// 0 < H-1-h <= bottom); the same per column; up to 3 x 3 sources per input pixel
template <bool BF16>
__global__ __launch_bounds__(256) void reflect_pad_bwd_kernel(const void* __restrict__ dy, void* __restrict__ dx,
                                                              int N, int H, int W, int C, int Ho, int Wo, int top,
                                                              int left) {
  const int cpp = C / 8;
  const long total = (long)N * H * W * cpp;
  const int bottom = Ho - H - top, right = Wo - W - left;
  for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const int cc = (int)(t % cpp);
    long r = t / cpp;
    const int w = (int)(r % W);
    r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    int hs[3], ws[3], nh = 0, nw = 0;
    hs[nh++] = h + top;
    if (h > 0 && h <= top) hs[nh++] = top - h;
    if (H - 1 - h > 0 && H - 1 - h <= bottom) hs[nh++] = top + 2 * (H - 1) - h;
    ws[nw++] = w + left;
    if (w > 0 && w <= left) ws[nw++] = left - w;
    if (W - 1 - w > 0 && W - 1 - w <= right) ws[nw++] = left + 2 * (W - 1) - w;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int a = 0; a < nh; ++a)
      for (int b = 0; b < nw; ++b) {
        float v[8];
        load_chunk<BF16>(dy, (((size_t)n * Ho + hs[a]) * Wo + ws[b]) * C + cc * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    store8<BF16>(dx, (long)t * 8, (long)t * 8 + 8, acc);
  }
}

static int grid_for(long work) {
  long b = (work + 255) / 256;
  if (b > 16384) b = 16384;
  return b < 1 ? 1 : (int)b;
}

}  // namespace dtm

using namespace dtm;

DTM_API int dtm_act_fwd(const void* x, void* y, long n, int kind, float alpha, int bf16, void* stream) {
  const int g = grid_for((n + 7) / 8);
  if (bf16) hipLaunchKernelGGL(act_fwd_kernel<true>, dim3(g), dim3(256), 0, (hipStream_t)stream, x, y, n, kind, alpha);
  else hipLaunchKernelGGL(act_fwd_kernel<false>, dim3(g), dim3(256), 0, (hipStream_t)stream, x, y, n, kind, alpha);
  return 0;
}

DTM_API int dtm_act_bwd(const void* dy, const void* x, void* dx, long n, int kind, float alpha, int bf16, void* stream) {
  const int g = grid_for((n + 7) / 8);
  if (bf16)
    hipLaunchKernelGGL(act_bwd_kernel<true>, dim3(g), dim3(256), 0, (hipStream_t)stream, dy, x, dx, n, kind, alpha);
  else
    hipLaunchKernelGGL(act_bwd_kernel<false>, dim3(g), dim3(256), 0, (hipStream_t)stream, dy, x, dx, n, kind, alpha);
  return 0;
}

DTM_API int dtm_instnorm_fwd(const void* x, const float* gamma, const float* beta, void* y, float* stats, int N, int HW,
                             int C, float eps, int relu, int bf16, void* stream) {
  if (C % 8) return -1;
  dim3 grid((C + 63) / 64, N);
  if (bf16)
    hipLaunchKernelGGL(instnorm_fwd_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, x, gamma, beta, y, stats,
                       HW, C, eps, relu);
  else
    hipLaunchKernelGGL(instnorm_fwd_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, x, gamma, beta, y, stats,
                       HW, C, eps, relu);
  return 0;
}

DTM_API int dtm_instnorm_bwd(const void* x, const void* dy, const float* gamma, const float* stats, void* dx,
                             float* sums, int N, int HW, int C, int bf16, void* stream) {
  if (C % 8) return -1;
  dim3 grid((C + 63) / 64, N);
  if (bf16)
    hipLaunchKernelGGL(instnorm_bwd_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, x, dy, gamma, stats, dx,
                       sums, HW, C);
  else
    hipLaunchKernelGGL(instnorm_bwd_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, x, dy, gamma, stats, dx,
                       sums, HW, C);
  return 0;
}

DTM_API int dtm_reflect_pad(const void* x, void* y, int N, int H, int W, int C, int top, int bottom, int left,
                            int right, int bf16, void* stream) {
  if (C % 8 || top >= H || bottom >= H || left >= W || right >= W || top < 0 || bottom < 0 || left < 0 || right < 0)
    return -1;
  const int Ho = H + top + bottom, Wo = W + left + right;
  const int g = grid_for((long)N * Ho * Wo * (C / 8));
  if (bf16)
    hipLaunchKernelGGL(reflect_pad_fwd_kernel<true>, dim3(g), dim3(256), 0, (hipStream_t)stream, x, y, N, H, W, C, Ho,
                       Wo, top, left);
  else
    hipLaunchKernelGGL(reflect_pad_fwd_kernel<false>, dim3(g), dim3(256), 0, (hipStream_t)stream, x, y, N, H, W, C,
                       Ho, Wo, top, left);
  return 0;
}

DTM_API int dtm_reflect_pad_bwd(const void* dy, void* dx, int N, int H, int W, int C, int top, int bottom, int left,
                                int right, int bf16, void* stream) {
  if (C % 8 || top >= H || bottom >= H || left >= W || right >= W) return -1;
  const int Ho = H + top + bottom, Wo = W + left + right;
  const int g = grid_for((long)N * H * W * (C / 8));
  if (bf16)
    hipLaunchKernelGGL(reflect_pad_bwd_kernel<true>, dim3(g), dim3(256), 0, (hipStream_t)stream, dy, dx, N, H, W, C,
                       Ho, Wo, top, left);
  else
    hipLaunchKernelGGL(reflect_pad_bwd_kernel<false>, dim3(g), dim3(256), 0, (hipStream_t)stream, dy, dx, N, H, W, C,
                       Ho, Wo, top, left);
  return 0;
}
