// GPU image augmentation (replaces the CPU-pinned TF image ops of the reference input pipelines:
// random_crop, random_flip_left_right, random_brightness, random_contrast,
// per_image_standardization, central crop/pad - SURVEY.md §2.8 C45/C47, K19).
// One workgroup per image: the uint8 source image is staged in LDS, the crop/flip gather and the
// brightness delta are applied, per-channel means (contrast) and the whole-image mean/std
// (standardisation) are reduced in LDS, and the NHWC result is written as bf16 or fp32.
// All random parameters come from the host per batch (reproducible, seedable).
#include "common.h"

namespace dtm {

struct AugParams {
  int oy, ox;         // crop offset in the (possibly padded) source
  int flip;           // horizontal flip
  float brightness;   // additive delta (in [0,255] units like TF on uint8->float images)
  float contrast;     // factor (1 = identity)
  float pad0;
};

// src: [B][H][W][C] uint8; dst: [B][S][S][C]; crop window S x S at (oy, ox); offsets may be negative
// (zero padding, tf.image.resize_image_with_crop_or_pad semantics).  mode bit0: standardize.
template <typename T>
__global__ __launch_bounds__(256) void augment_kernel(const uint8_t* __restrict__ src, T* __restrict__ dst,
                                                      const AugParams* __restrict__ params, int H, int W, int C,
                                                      int S, int standardize, float scale, float shift) {
  extern __shared__ float buf[];  // S*S*C floats
  __shared__ float red[2][256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const AugParams p = params[b];
  const int n = S * S * C;
  const uint8_t* img = src + (size_t)b * H * W * C;
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i = tid; i < n; i += 256) {
    int c = i % C, q = (i / C) % S, r = i / (C * S);
    int y = r + p.oy, x = (p.flip ? (S - 1 - q) : q) + p.ox;
    float v = (y >= 0 && y < H && x >= 0 && x < W) ? (float)img[((size_t)y * W + x) * C + c] : 0.f;
    v += p.brightness;
    buf[i] = v;
  }
  __syncthreads();
  if (p.contrast != 1.f) {
    // per-channel mean (C <= 4)
    for (int c = 0; c < C; ++c) {
      float s = 0.f;
      for (int i = tid * C + c; i < n; i += 256 * C) s += buf[i];
      red[0][tid] = s;
      __syncthreads();
      for (int h = 128; h > 0; h >>= 1) {
        if (tid < h) red[0][tid] += red[0][tid + h];
        __syncthreads();
      }
      csum[c] = red[0][0] / (float)(S * S);
      __syncthreads();
    }
    for (int i = tid; i < n; i += 256) {
      int c = i % C;
      buf[i] = (buf[i] - csum[c]) * p.contrast + csum[c];
    }
    __syncthreads();
  }
  float mean = 0.f, inv = 1.f;
  if (standardize) {
    float s = 0.f, q = 0.f;
    for (int i = tid; i < n; i += 256) { s += buf[i]; q += buf[i] * buf[i]; }
    red[0][tid] = s;
    red[1][tid] = q;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (tid < h) { red[0][tid] += red[0][tid + h]; red[1][tid] += red[1][tid + h]; }
      __syncthreads();
    }
    mean = red[0][0] / n;
    float var = fmaxf(red[1][0] / n - mean * mean, 0.f);
    // tf.image.per_image_standardization: (x - mean) / max(stddev, 1/sqrt(N))
    inv = 1.f / fmaxf(sqrtf(var), rsqrtf((float)n));
  }
  T* out = dst + (size_t)b * n;
  for (int i = tid; i < n; i += 256) {
    float v = standardize ? (buf[i] - mean) * inv : buf[i] * scale + shift;
    if constexpr (sizeof(T) == 4) out[i] = v;
    else out[i] = f2bf(v);
  }
}
}  // namespace dtm
using namespace dtm;

DTM_API int dtm_augment(const void* src, void* dst, int dst_bf16, const void* params, int B, int H, int W, int C,
                        int S, int standardize, float scale, float shift, void* stream) {
  if (C > 4) return -1;
  size_t sm = (size_t)S * S * C * sizeof(float);
  if (sm > 64 * 1024) return -2;
  if (dst_bf16)
    hipLaunchKernelGGL(augment_kernel<bf16_t>, dim3(B), dim3(256), sm, (hipStream_t)stream, (const uint8_t*)src,
                       (bf16_t*)dst, (const AugParams*)params, H, W, C, S, standardize, scale, shift);
  else
    hipLaunchKernelGGL(augment_kernel<float>, dim3(B), dim3(256), sm, (hipStream_t)stream, (const uint8_t*)src,
                       (float*)dst, (const AugParams*)params, H, W, C, S, standardize, scale, shift);
  return 0;
}
