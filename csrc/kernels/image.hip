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

// ------------------------------------------------------------------------------------------
// ImageNet (Inception) preprocessing on the GPU: reference inception/image_processing.py:164-276
// (distort_image: sample_distorted_bounding_box crop -> resize_images(method = thread_id % 4) ->
// random flip -> distort_color in one of two orders -> clip) and :278-300 (eval_image: central crop
// + bilinear resize), then (x - 0.5) * 2.  The host decodes the JPEGs (a process pool) into one
// ragged uint8 buffer and samples every per-image random parameter; two kernels do the rest:
//   prep:   one thread per output pixel: crop + TF-1 legacy resample (bilinear / nearest / bicubic
//           with the 1/1024-quantised Keys table / area box) of the [0,1] image, flip, brightness and
//           (ordering 0) saturation + hue in HSV; fp32 to a staging tensor; per-image channel sums for
//           the contrast mean (block partial sums, one atomic per channel per block);
//   finish: contrast (ordering 0: last; ordering 1: before saturation + hue), clip, [-1, 1], bf16/fp32.
struct PrepParams {
  long long src_off;          // byte offset of the image in the ragged uint8 buffer ([h][w][3])
  int h, w, y0, x0, ch, cw;   // source size and crop window
  int method, flip, color, ordering;
  float bright, sat, hue, contrast;
};

__device__ __forceinline__ void rgb2hsv(float r, float g, float b, float& h, float& s, float& v) {
  v = fmaxf(r, fmaxf(g, b));
  const float rng = v - fminf(r, fminf(g, b));
  s = v > 0.f ? rng / v : 0.f;
  if (rng > 0.f) {
    if (r == v) h = (g - b) / rng;
    else if (g == v) h = (b - r) / rng + 2.f;
    else h = (r - g) / rng + 4.f;
    h *= (1.f / 6.f);
    if (h < 0.f) h += 1.f;
  } else {
    h = 0.f;
  }
}
__device__ __forceinline__ void hsv2rgb(float h, float s, float v, float& r, float& g, float& b) {
  const float c = s * v, m = v - c, dh = h * 6.f;
  const float x = c * (1.f - fabsf(fmodf(dh, 2.f) - 1.f));
  int k = (int)floorf(dh) % 6;
  if (k < 0) k += 6;
  float rr, gg, bb;
  switch (k) {
    case 0: rr = c; gg = x; bb = 0.f; break;
    case 1: rr = x; gg = c; bb = 0.f; break;
    case 2: rr = 0.f; gg = c; bb = x; break;
    case 3: rr = 0.f; gg = x; bb = c; break;
    case 4: rr = x; gg = 0.f; bb = c; break;
    default: rr = c; gg = 0.f; bb = x; break;
  }
  r = rr + m; g = gg + m; b = bb + m;
}
// taps of one axis for output coordinate o (at most 4 for bilinear/nearest/bicubic; area loops)
__device__ __forceinline__ int axis_taps(int method, int o, int n, int out, int* idx, float* wt) {
  const float scale = (float)n / (float)out;
  const float f = o * scale;
  if (method == 0) {  // bilinear
    const int i0 = (int)floorf(f);
    const int i1 = min(i0 + 1, n - 1);
    const float d = f - i0;
    idx[0] = i0; wt[0] = 1.f - d; idx[1] = i1; wt[1] = d;
    return 2;
  }
  if (method == 1) {  // nearest
    idx[0] = min((int)floorf(f), n - 1); wt[0] = 1.f;
    return 1;
  }
  // bicubic (TF legacy: Keys a = -0.75 from a 1024-entry table)
  const int i = (int)floorf(f);
  const int off = __float2int_rn((f - i) * 1024.f);
  const float a = -0.75f, x = off / 1024.f, y = (1024 - off) / 1024.f;
  const float x1 = x + 1.f, y1 = y + 1.f;
  wt[0] = ((a * x1 - 5.f * a) * x1 + 8.f * a) * x1 - 4.f * a;
  wt[1] = ((a + 2.f) * x - (a + 3.f)) * x * x + 1.f;
  wt[2] = ((a + 2.f) * y - (a + 3.f)) * y * y + 1.f;
  wt[3] = ((a * y1 - 5.f * a) * y1 + 8.f * a) * y1 - 4.f * a;
#pragma unroll
  for (int k = 0; k < 4; ++k) idx[k] = min(max(i - 1 + k, 0), n - 1);
  return 4;
}

template <int MAXA>
__device__ __forceinline__ void sample_pixel(const uint8_t* img, int w, const PrepParams& p, int oy, int ox, int S,
                                             float (&v)[3]) {
  v[0] = v[1] = v[2] = 0.f;
  const uint8_t* base = img + ((size_t)p.y0 * w + p.x0) * 3;
  if (p.method == 3) {  // area: fractional box [o*scale, (o+1)*scale) on both axes
    const float sy = (float)p.ch / S, sx = (float)p.cw / S;
    const float fy0 = oy * sy, fy1 = (oy + 1) * sy, fx0 = ox * sx, fx1 = (ox + 1) * sx;
    const float inv = 1.f / (sy * sx);
    for (int i = (int)floorf(fy0); (float)i < fy1; ++i) {
      const float wy = fminf(fy1, (float)(i + 1)) - fmaxf(fy0, (float)i);
      if (wy <= 0.f) continue;
      const uint8_t* row = base + (size_t)min(i, p.ch - 1) * w * 3;
      for (int j = (int)floorf(fx0); (float)j < fx1; ++j) {
        const float wx = fminf(fx1, (float)(j + 1)) - fmaxf(fx0, (float)j);
        if (wx <= 0.f) continue;
        const uint8_t* px = row + (size_t)min(j, p.cw - 1) * 3;
        const float ww = wy * wx * inv;
        v[0] += ww * px[0]; v[1] += ww * px[1]; v[2] += ww * px[2];
      }
    }
  } else {
    int iy[4], ix[4];
    float wy[4], wx[4];
    const int ny = axis_taps(p.method, oy, p.ch, S, iy, wy);
    const int nx = axis_taps(p.method, ox, p.cw, S, ix, wx);
    for (int a = 0; a < ny; ++a) {
      const uint8_t* row = base + (size_t)iy[a] * w * 3;
      float r[3] = {0.f, 0.f, 0.f};
      for (int b = 0; b < nx; ++b) {
        const uint8_t* px = row + (size_t)ix[b] * 3;
        r[0] += wx[b] * px[0]; r[1] += wx[b] * px[1]; r[2] += wx[b] * px[2];
      }
      v[0] += wy[a] * r[0]; v[1] += wy[a] * r[1]; v[2] += wy[a] * r[2];
    }
  }
  v[0] *= (1.f / 255.f); v[1] *= (1.f / 255.f); v[2] *= (1.f / 255.f);
}

__device__ __forceinline__ void saturate_hue(float (&v)[3], float sat, float hue) {
  float h, s, val;
  rgb2hsv(v[0], v[1], v[2], h, s, val);
  s = fminf(fmaxf(s * sat, 0.f), 1.f);
  hsv2rgb(h, s, val, v[0], v[1], v[2]);
  rgb2hsv(v[0], v[1], v[2], h, s, val);
  h += hue;
  if (h < 0.f) h += 1.f;
  else if (h >= 1.f) h -= 1.f;
  hsv2rgb(h, s, val, v[0], v[1], v[2]);
}

__global__ __launch_bounds__(256) void imagenet_prep_kernel(const uint8_t* __restrict__ src,
                                                            const PrepParams* __restrict__ params,
                                                            float* __restrict__ stage, float* __restrict__ sums,
                                                            int S) {
  __shared__ float red[3][256];
  const int b = blockIdx.y;
  const PrepParams p = params[b];
  const int pix = blockIdx.x * 256 + threadIdx.x;
  float v[3] = {0.f, 0.f, 0.f};
  if (pix < S * S) {
    const int oy = pix / S, oxo = pix - oy * S;
    const int ox = p.flip ? S - 1 - oxo : oxo;
    sample_pixel<0>(src + p.src_off, p.w, p, oy, ox, S, v);
    if (p.color) {
      v[0] += p.bright; v[1] += p.bright; v[2] += p.bright;
      if (p.ordering == 0) saturate_hue(v, p.sat, p.hue);
    }
    float* o = stage + ((size_t)b * S * S + pix) * 3;
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
  } else {
    v[0] = v[1] = v[2] = 0.f;
  }
  if (!p.color) return;  // (uniform per block: every thread of the block has the same image)
  red[0][threadIdx.x] = v[0]; red[1][threadIdx.x] = v[1]; red[2][threadIdx.x] = v[2];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
      red[2][threadIdx.x] += red[2][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x < 3) atomicAdd(sums + b * 3 + threadIdx.x, red[threadIdx.x][0]);
}

template <typename T>
__global__ __launch_bounds__(256) void imagenet_finish_kernel(const float* __restrict__ stage,
                                                              const PrepParams* __restrict__ params,
                                                              const float* __restrict__ sums, T* __restrict__ out,
                                                              int S) {
  const int b = blockIdx.y;
  const PrepParams p = params[b];
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= S * S) return;
  const size_t e = ((size_t)b * S * S + pix) * 3;
  float v[3] = {stage[e], stage[e + 1], stage[e + 2]};
  if (p.color) {
    const float inv = 1.f / (float)(S * S);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float m = sums[b * 3 + c] * inv;
      v[c] = (v[c] - m) * p.contrast + m;
    }
    if (p.ordering == 1) saturate_hue(v, p.sat, p.hue);
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = fminf(fmaxf(v[c], 0.f), 1.f);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float y = (v[c] - 0.5f) * 2.f;
    if constexpr (sizeof(T) == 4) out[e + c] = y;
    else out[e + c] = f2bf(y);
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

DTM_API int dtm_prep_params_bytes() { return (int)sizeof(PrepParams); }

// src: ragged uint8 images; params: B PrepParams (device); stage: B*S*S*3 fp32 scratch; sums: B*3 fp32
// (zeroed here); out: [B][S][S][3] bf16 or fp32
DTM_API int dtm_imagenet_prep(const void* src, const void* params, float* stage, float* sums, void* out, int out_bf16,
                              int B, int S, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(sums, 0, (size_t)B * 3 * sizeof(float), st) != hipSuccess) return -1;
  dim3 grid((S * S + 255) / 256, B);
  hipLaunchKernelGGL(imagenet_prep_kernel, grid, dim3(256), 0, st, (const uint8_t*)src, (const PrepParams*)params,
                     stage, sums, S);
  if (out_bf16)
    hipLaunchKernelGGL(imagenet_finish_kernel<bf16_t>, grid, dim3(256), 0, st, stage, (const PrepParams*)params, sums,
                       (bf16_t*)out, S);
  else
    hipLaunchKernelGGL(imagenet_finish_kernel<float>, grid, dim3(256), 0, st, stage, (const PrepParams*)params, sums,
                       (float*)out, S);
  return 0;
}
