// Fused softmax cross-entropy (+label smoothing) and multi-tensor optimizer kernels.
//
// Loss: replaces SoftmaxCrossEntropyWithLogits / sparse variant and slim cross_entropy_loss
// with label smoothing y*(1-eps) + eps/K (reference
// inception/slim/losses.py:142-174, cnn/cifar10.py:298-306).
//
// Optimizer: one launch updates every parameter tensor (chunk table built once on the host),
// with TF 1.x update rules:
//   SGD            p -= lr*g
//   Momentum       a = mu*a + g;  p -= lr*a            (use_nesterov=False)
//   RMSProp (TF)   ms = rho*ms + (1-rho)*g^2;  mom = mu*mom + lr*g/sqrt(ms+eps);  p -= mom
// with g = grad*grad_scale + wd*p (coupled L2, the gradient of wd*sum(p^2)/2), an optional
// fused ExponentialMovingAverage shadow update (decay already min'd with (1+n)/(10+n) on the
// host) and a bf16 copy-out of the updated weight for the next forward.
#include "common.h"

namespace dtm {

template <typename T>
__device__ __forceinline__ float ldf(const T* p, long i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, long i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p, long i) { return bf2f(p[i]); }

// one block per row; labels int32; out_loss[row]; dlogits fp32 or bf16 (same type as logits)
template <typename T>
__global__ __launch_bounds__(256) void softmax_xent_kernel(const T* __restrict__ logits, const int* __restrict__ labels,
                                                           float* __restrict__ loss, T* __restrict__ dlogits, int K,
                                                           float smoothing, float gscale, const float* row_weight,
                                                           int ldx) {
  __shared__ float red[8];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const T* x = logits + (long)row * ldx;  // (ldx: row pitch - an FC's padded output read in place)
  float m = -INFINITY;
  for (int k = tid; k < K; k += 256) m = fmaxf(m, ldf(x, k));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) red[wv] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f, sx = 0.f;
  for (int k = tid; k < K; k += 256) {
    float v = ldf(x, k);
    s += __expf(v - m);
    sx += v;
  }
  s = warp_sum(s);
  sx = warp_sum(sx);
  if (lane == 0) { red[wv] = s; red[4 + wv] = sx; }
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  sx = red[4] + red[5] + red[6] + red[7];
  const float lse = m + __logf(s);
  const int lab = labels[row];
  const float on = 1.f - smoothing + smoothing / K, off = smoothing / K;
  const float w = row_weight ? row_weight[row] : 1.f;
  if (tid == 0) {
    float xl = (lab >= 0 && lab < K) ? ldf(x, lab) : 0.f;
    // -sum_k t_k log p_k = lse - sum_k t_k x_k
    loss[row] = w * (lse - (off * sx + (on - off) * xl));
  }
  if (dlogits) {
    T* d = dlogits + (long)row * K;
    for (int k = tid; k < K; k += 256) {
      float p = __expf(ldf(x, k) - lse);
      float t = (k == lab) ? on : off;
      float gv = (p - t) * gscale * w;
      if constexpr (sizeof(T) == 4) d[k] = gv;
      else d[k] = f2bf(gv);
    }
  }
}

struct OptTensor {
  float* p;
  const float* g;
  float* s1;      // momentum accumulator / RMSProp mom
  float* s2;      // RMSProp ms
  bf16_t* pcopy;  // optional bf16 copy of the updated weight
  float* ema;     // optional EMA shadow
  long n;
  float wd;
  float lr_mult;
};
struct OptChunk {
  int t;
  int pad;
  long start;
};
struct OptHyper {
  int kind;  // 0 sgd, 1 momentum, 2 rmsprop
  float lr, mu, rho, eps, grad_scale, ema_decay;
  int use_ema;
  const int* skip_flag;  // optional: non-zero -> skip the update (non-finite gradients)
  const float* dyn;      // optional device scalars [lr, ema_decay, grad_scale] (graph-replay safe)
};
constexpr int OPT_CHUNK = 8192;

__global__ __launch_bounds__(256) void multi_tensor_opt_kernel(const OptTensor* __restrict__ tens,
                                                               const OptChunk* __restrict__ chunks, OptHyper h) {
  if (h.skip_flag && *h.skip_flag) return;
  const OptChunk c = chunks[blockIdx.x];
  const OptTensor t = tens[c.t];
  const long end = min(t.n, c.start + (long)OPT_CHUNK);
  const float lr = (h.dyn ? h.dyn[0] : h.lr) * t.lr_mult;
  const float ema_decay = h.dyn ? h.dyn[1] : h.ema_decay;
  const float grad_scale = h.dyn ? h.dyn[2] : h.grad_scale;
  if (!t.g) {  // EMA-only row (BN moving statistics): shadow -= (1-d)(shadow - value)
    if (h.use_ema && t.ema)
      for (long i = c.start + threadIdx.x; i < end; i += 256) t.ema[i] -= (1.f - ema_decay) * (t.ema[i] - t.p[i]);
    return;
  }
  for (long i = c.start + threadIdx.x; i < end; i += 256) {
    float p = t.p[i];
    float g = t.g[i] * grad_scale + t.wd * p;
    if (h.kind == 0) {
      p -= lr * g;
    } else if (h.kind == 1) {
      float a = h.mu * t.s1[i] + g;
      t.s1[i] = a;
      p -= lr * a;
    } else {
      float ms = h.rho * t.s2[i] + (1.f - h.rho) * g * g;
      t.s2[i] = ms;
      float mom = h.mu * t.s1[i] + lr * g * rsqrtf(ms + h.eps);
      t.s1[i] = mom;
      p -= mom;
    }
    t.p[i] = p;
    if (t.pcopy) t.pcopy[i] = f2bf(p);
    if (h.use_ema && t.ema) t.ema[i] -= (1.f - ema_decay) * (t.ema[i] - p);
  }
}

__global__ void check_finite_kernel(const float* __restrict__ x, long n, int* __restrict__ flag) {
  bool bad = false;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float v = x[i];
    bad |= !(fabsf(v) <= 3.4e38f);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = f2bf(x[i]);
}
__global__ void scale_kernel(float* __restrict__ x, long n, float s) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] *= s;
}

// Backward of the per-row loss: out[r][c] = dl[r][c] * gl[r * gstride] for c < N, 0 for N <= c < ldo (the zero
// columns of the padded logits operand of the FC backward, written here instead of a zero fill + copy).  One pass in
// place of the float cast, broadcast multiply and bf16 cast autograd would launch; gstride 0: one scale for every row.
template <typename T>
__global__ __launch_bounds__(256) void scale_rows_pad_kernel(const T* __restrict__ dl, const float* __restrict__ gl,
                                                             int gstride, T* __restrict__ out, int B, int N,
                                                             int ldo) {
  // rows grid-stride over blockIdx.y (grid.y <= 65535 whatever the batch)
  for (int r = blockIdx.y; r < B; r += gridDim.y) {
    const float g = gl[(long)r * gstride];
    const T* src = dl + (long)r * N;
    T* dst = out + (long)r * ldo;
    for (int c = blockIdx.x * 256 + threadIdx.x; c < ldo; c += gridDim.x * 256) {
      const float v = c < N ? ldf(src, c) * g : 0.f;
      if constexpr (sizeof(T) == 2) dst[c] = f2bf(v);
      else dst[c] = v;
    }
  }
}

// The scalar training loss from up to 4 per-row loss vectors: out = sum_h w_h * sum_r loss[h][r] (w_h = the head's
// weight / batch: the mean, the aux-head weight and the batch weight in one launch, one block, fixed order).
struct LossW {
  float w[4];
};
__global__ __launch_bounds__(256) void loss_combine_kernel(const float* __restrict__ loss, int heads, int B, LossW lw,
                                                           float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int h = 0; h < heads; ++h) {
    float s = 0.f;
    for (int r = threadIdx.x; r < B; r += 256) s += loss[(long)h * B + r];
    acc += s * lw.w[h];
  }
  acc = warp_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace dtm
using namespace dtm;

DTM_API int dtm_scale_rows_pad(const void* dl, int bf16, const float* gl, int gstride, void* out, int B, int N, int ldo,
                               void* stream) {
  if (B <= 0 || N <= 0 || ldo < N) return -1;
  const int bx = (ldo + 255) / 256 > 8 ? 8 : (ldo + 255) / 256;
  const int by = B > 65535 ? 65535 : B;
  if (bf16)
    hipLaunchKernelGGL(scale_rows_pad_kernel<bf16_t>, dim3(bx, by), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dl, gl, gstride, (bf16_t*)out, B, N, ldo);
  else
    hipLaunchKernelGGL(scale_rows_pad_kernel<float>, dim3(bx, by), dim3(256), 0, (hipStream_t)stream,
                       (const float*)dl, gl, gstride, (float*)out, B, N, ldo);
  return 0;
}

DTM_API void dtm_softmax_xent(const void* logits, int logits_bf16, const int* labels, float* loss, void* dlogits,
                              int B, int K, float smoothing, float gscale, const float* row_weight, int ldx,
                              void* stream) {
  if (ldx < K) ldx = K;
  if (logits_bf16)
    hipLaunchKernelGGL(softmax_xent_kernel<bf16_t>, dim3(B), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)logits,
                       labels, loss, (bf16_t*)dlogits, K, smoothing, gscale, row_weight, ldx);
  else
    hipLaunchKernelGGL(softmax_xent_kernel<float>, dim3(B), dim3(256), 0, (hipStream_t)stream, (const float*)logits,
                       labels, loss, (float*)dlogits, K, smoothing, gscale, row_weight, ldx);
}

DTM_API int dtm_loss_combine(const float* loss, int heads, int B, const float* w, float* out, void* stream) {
  if (heads < 1 || heads > 4 || B < 1) return -1;
  LossW lw{};
  for (int h = 0; h < heads; ++h) lw.w[h] = w[h];
  hipLaunchKernelGGL(loss_combine_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, loss, heads, B, lw, out);
  return 0;
}

DTM_API int dtm_opt_chunk_size() { return OPT_CHUNK; }
DTM_API int dtm_opt_tensor_bytes() { return (int)sizeof(OptTensor); }
DTM_API int dtm_opt_chunk_bytes() { return (int)sizeof(OptChunk); }

DTM_API void dtm_multi_tensor_opt(const void* tensors_dev, const void* chunks_dev, int num_chunks, int kind, float lr,
                                  float mu, float rho, float eps, float grad_scale, float ema_decay, int use_ema,
                                  const int* skip_flag, const float* dyn, void* stream) {
  OptHyper h;
  h.dyn = dyn;
  h.kind = kind; h.lr = lr; h.mu = mu; h.rho = rho; h.eps = eps; h.grad_scale = grad_scale;
  h.ema_decay = ema_decay; h.use_ema = use_ema; h.skip_flag = skip_flag;
  if (num_chunks <= 0) return;
  hipLaunchKernelGGL(multi_tensor_opt_kernel, dim3(num_chunks), dim3(256), 0, (hipStream_t)stream,
                     (const OptTensor*)tensors_dev, (const OptChunk*)chunks_dev, h);
}

DTM_API void dtm_check_finite(const float* x, long n, int* flag, void* stream) {
  long b = (n + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(check_finite_kernel, dim3((int)b), dim3(256), 0, (hipStream_t)stream, x, n, flag);
}
DTM_API void dtm_f32_to_bf16(const float* x, void* y, long n, void* stream) {
  long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((int)b), dim3(256), 0, (hipStream_t)stream, x, (bf16_t*)y, n);
}
DTM_API void dtm_scale(float* x, long n, float s, void* stream) {
  long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(scale_kernel, dim3((int)b), dim3(256), 0, (hipStream_t)stream, x, n, s);
}
