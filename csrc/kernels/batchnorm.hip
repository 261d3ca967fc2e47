// Training / inference BatchNorm (+ReLU, +residual) kernels, NHWC bf16 activations, fp32 stats.
//
// Replaces TF's FusedBatchNorm / moments + batch_normalization (SURVEY.md §2.12c K4/K5;
// reference resnet/resnet_model.py:45-48, inception/slim/ops.py:117-131,
// vgg/nets/resnet_utils.py:254).  Semantics kept from TF 1.x:
//   * normalisation uses the biased batch variance;
//   * the moving variance update uses the Bessel-corrected variance when `bessel` is set
//     (fused BN path of the contrib-slim zoo) and the biased one otherwise (old slim
//     tf.nn.moments path, inception/slim/ops.py:117-124);
//   * moving_x -= (moving_x - batch_x) * (1 - decay).
// Activations are processed 8 channels (16 B) per lane; per-channel partial sums are reduced
// through LDS and committed with one fp32 atomic per channel per block.
#include "common.h"

namespace dtm {

template <int V>
struct Vec;
template <>
struct Vec<8> {
  uint4 u;
  __device__ __forceinline__ void load(const bf16_t* p) { u = *(const uint4*)p; }
  __device__ __forceinline__ void store(bf16_t* p) const { *(uint4*)p = u; }
  __device__ __forceinline__ float get(int e) const {
    uint32_t w = e < 2 ? u.x : e < 4 ? u.y : e < 6 ? u.z : u.w;
    return (e & 1) ? hi_bf(w) : lo_bf(w);
  }
  __device__ __forceinline__ void unpack(float* f) const {
    f[0] = lo_bf(u.x); f[1] = hi_bf(u.x); f[2] = lo_bf(u.y); f[3] = hi_bf(u.y);
    f[4] = lo_bf(u.z); f[5] = hi_bf(u.z); f[6] = lo_bf(u.w); f[7] = hi_bf(u.w);
  }
  __device__ __forceinline__ void pack(const float* f) {
    u = make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
  }
};
template <>
struct Vec<1> {
  bf16_t u;
  __device__ __forceinline__ void load(const bf16_t* p) { u = *p; }
  __device__ __forceinline__ void store(bf16_t* p) const { *p = u; }
  __device__ __forceinline__ void unpack(float* f) const { f[0] = bf2f(u); }
  __device__ __forceinline__ void pack(const float* f) { u = f2bf(f[0]); }
};

// ---- per-channel sum / sumsq over rows ---------------------------------------------------
template <int V>
__global__ __launch_bounds__(256) void bn_stats_kernel(const bf16_t* __restrict__ x, float* __restrict__ stats,
                                                       long M, int C, long rows_per_block) {
  __shared__ float red[2][256][V];
  const int cols = C / V;
  const int tid = threadIdx.x;
  const int rpi = cols >= 256 ? 1 : 256 / cols;
  const long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (int cb = 0; cb < cols; cb += 256) {
    const int tcol = cb + (cols >= 256 ? tid : tid % cols);
    const int trow = cols >= 256 ? 0 : tid / cols;
    float s[V], q[V];
#pragma unroll
    for (int e = 0; e < V; ++e) s[e] = q[e] = 0.f;
    if (trow < rpi && tcol < cols) {
      for (long r = r0 + trow; r < r1; r += rpi) {
        Vec<V> v; v.load(x + r * C + tcol * V);
        float f[V]; v.unpack(f);
#pragma unroll
        for (int e = 0; e < V; ++e) { s[e] += f[e]; q[e] += f[e] * f[e]; }
      }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) { red[0][tid][e] = s[e]; red[1][tid][e] = q[e]; }
    __syncthreads();
    if (cols >= 256) {
      if (tcol < cols) {
#pragma unroll
        for (int e = 0; e < V; ++e) {
          atomicAdd(stats + tcol * V + e, s[e]);
          atomicAdd(stats + C + tcol * V + e, q[e]);
        }
      }
    } else if (tid < cols) {
      float S[V], Q[V];
#pragma unroll
      for (int e = 0; e < V; ++e) S[e] = Q[e] = 0.f;
      for (int rr = 0; rr < rpi; ++rr)
#pragma unroll
        for (int e = 0; e < V; ++e) { S[e] += red[0][rr * cols + tid][e]; Q[e] += red[1][rr * cols + tid][e]; }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        atomicAdd(stats + tid * V + e, S[e]);
        atomicAdd(stats + C + tid * V + e, Q[e]);
      }
    }
    __syncthreads();
  }
}

// ---- finalize: stats -> scale/shift (+ moving average update) -----------------------------
// out: [4][C] = scale, shift, mean, rstd
__global__ void bn_finalize_kernel(const float* __restrict__ stats, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float* __restrict__ mov_mean,
                                   float* __restrict__ mov_var, float* __restrict__ out, int C, float count,
                                   float eps, float decay, int update, int bessel) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mean = stats[c] / count;
  float var = fmaxf(stats[C + c] / count - mean * mean, 0.f);
  float rstd = rsqrtf(var + eps);
  float g = gamma ? gamma[c] : 1.f;
  float b = beta ? beta[c] : 0.f;
  float sc = g * rstd;
  out[c] = sc;
  out[C + c] = b - mean * sc;
  out[2 * C + c] = mean;
  out[3 * C + c] = rstd;
  if (update) {
    float uvar = (bessel && count > 1.f) ? var * count / (count - 1.f) : var;
    mov_mean[c] -= (mov_mean[c] - mean) * (1.f - decay);
    mov_var[c] -= (mov_var[c] - uvar) * (1.f - decay);
  }
}

// inference: scale/shift from moving statistics
__global__ void bn_inference_params_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                           const float* __restrict__ mov_mean, const float* __restrict__ mov_var,
                                           float* __restrict__ out, int C, float eps) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float rstd = rsqrtf(mov_var[c] + eps);
  float g = gamma ? gamma[c] : 1.f;
  float sc = g * rstd;
  out[c] = sc;
  out[C + c] = (beta ? beta[c] : 0.f) - mov_mean[c] * sc;
  out[2 * C + c] = mov_mean[c];
  out[3 * C + c] = rstd;
}

// ---- apply: y = act(x*scale + shift [+ res | + res*rscale + rshift]) -----------------------
// res_mode: 0 none, 1 identity residual, 2 BN'd residual (projection shortcut)
template <int V>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x, const float* __restrict__ ss,
                                                       const bf16_t* __restrict__ res, const float* __restrict__ rss,
                                                       bf16_t* __restrict__ y, long M, int C, int res_mode, int relu) {
  const int cols = C / V;
  const long total = M * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % cols) * V;
    Vec<V> v; v.load(x + i * V);
    float f[V]; v.unpack(f);
#pragma unroll
    for (int e = 0; e < V; ++e) f[e] = fmaf(f[e], ss[cv + e], ss[C + cv + e]);
    if (res_mode) {
      Vec<V> r; r.load(res + i * V);
      float g[V]; r.unpack(g);
      if (res_mode == 2) {
#pragma unroll
        for (int e = 0; e < V; ++e) f[e] += fmaf(g[e], rss[cv + e], rss[C + cv + e]);
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) f[e] += g[e];
      }
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < V; ++e) f[e] = fmaxf(f[e], 0.f);
    }
    Vec<V> o; o.pack(f); o.store(y + i * V);
  }
}

// ---- backward -------------------------------------------------------------------------------
// g = dy * mask, mask: mode 0 none, 1 (y > 0) from tensor y, 2 recompute (x*scale+shift > 0)
// sums: [2][C] += sum(g), sum(g * xhat),  xhat = (x - mean) * rstd
template <int V>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ ymask, const float* __restrict__ ss,
                                                            float* __restrict__ sums, long M, int C, int mask_mode,
                                                            long rows_per_block) {
  __shared__ float red[2][256][V];
  const int cols = C / V;
  const int tid = threadIdx.x;
  const int rpi = cols >= 256 ? 1 : 256 / cols;
  const long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const float* scale = ss;
  const float* shift = ss + C;
  const float* mean = ss + 2 * C;
  const float* rstd = ss + 3 * C;
  for (int cb = 0; cb < cols; cb += 256) {
    const int tcol = cb + (cols >= 256 ? tid : tid % cols);
    const int trow = cols >= 256 ? 0 : tid / cols;
    float s[V], q[V];
#pragma unroll
    for (int e = 0; e < V; ++e) s[e] = q[e] = 0.f;
    if (trow < rpi && tcol < cols) {
      const int cv = tcol * V;
      float mu[V], rs[V], sc[V], sh[V];
#pragma unroll
      for (int e = 0; e < V; ++e) { mu[e] = mean[cv + e]; rs[e] = rstd[cv + e]; sc[e] = scale[cv + e]; sh[e] = shift[cv + e]; }
      for (long r = r0 + trow; r < r1; r += rpi) {
        Vec<V> a, b; a.load(dy + r * C + cv); b.load(x + r * C + cv);
        float g[V], xv[V]; a.unpack(g); b.unpack(xv);
        if (mask_mode == 1) {
          Vec<V> m; m.load(ymask + r * C + cv);
          float mv[V]; m.unpack(mv);
#pragma unroll
          for (int e = 0; e < V; ++e) g[e] = mv[e] > 0.f ? g[e] : 0.f;
        } else if (mask_mode == 2) {
#pragma unroll
          for (int e = 0; e < V; ++e) g[e] = fmaf(xv[e], sc[e], sh[e]) > 0.f ? g[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < V; ++e) { s[e] += g[e]; q[e] += g[e] * (xv[e] - mu[e]) * rs[e]; }
      }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) { red[0][tid][e] = s[e]; red[1][tid][e] = q[e]; }
    __syncthreads();
    if (cols >= 256) {
      if (tcol < cols) {
#pragma unroll
        for (int e = 0; e < V; ++e) {
          atomicAdd(sums + tcol * V + e, s[e]);
          atomicAdd(sums + C + tcol * V + e, q[e]);
        }
      }
    } else if (tid < cols) {
      float S[V], Q[V];
#pragma unroll
      for (int e = 0; e < V; ++e) S[e] = Q[e] = 0.f;
      for (int rr = 0; rr < rpi; ++rr)
#pragma unroll
        for (int e = 0; e < V; ++e) { S[e] += red[0][rr * cols + tid][e]; Q[e] += red[1][rr * cols + tid][e]; }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        atomicAdd(sums + tid * V + e, S[e]);
        atomicAdd(sums + C + tid * V + e, Q[e]);
      }
    }
    __syncthreads();
  }
}

// dx = scale * (g - sum_g/M - xhat * sum_gx/M);  optional gout = g (masked dy, for the
// residual branch).  training=0: dx = scale * g (inference-mode BN, frozen statistics).
template <int V>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                           const bf16_t* __restrict__ ymask, const float* __restrict__ ss,
                                                           const float* __restrict__ sums, bf16_t* __restrict__ dx,
                                                           bf16_t* __restrict__ gout, long M, int C, int mask_mode,
                                                           int training) {
  const int cols = C / V;
  const long total = M * cols;
  const float invM = 1.f / (float)M;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cv = (int)(i % cols) * V;
    Vec<V> a, b; a.load(dy + i * V); b.load(x + i * V);
    float g[V], xv[V]; a.unpack(g); b.unpack(xv);
    if (mask_mode == 1) {
      Vec<V> m; m.load(ymask + i * V);
      float mv[V]; m.unpack(mv);
#pragma unroll
      for (int e = 0; e < V; ++e) g[e] = mv[e] > 0.f ? g[e] : 0.f;
    } else if (mask_mode == 2) {
#pragma unroll
      for (int e = 0; e < V; ++e) g[e] = fmaf(xv[e], ss[cv + e], ss[C + cv + e]) > 0.f ? g[e] : 0.f;
    }
    if (gout) { Vec<V> o; o.pack(g); o.store(gout + i * V); }
    float r[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int c = cv + e;
      if (training) {
        float xh = (xv[e] - ss[2 * C + c]) * ss[3 * C + c];
        r[e] = ss[c] * (g[e] - sums[c] * invM - xh * sums[C + c] * invM);
      } else {
        r[e] = ss[c] * g[e];
      }
    }
    Vec<V> o; o.pack(r); o.store(dx + i * V);
  }
}

// dgamma = sum(g*xhat), dbeta = sum(g)  (accumulated into fp32 grads)
__global__ void bn_param_grad_kernel(const float* __restrict__ sums, float* __restrict__ dgamma,
                                     float* __restrict__ dbeta, int C) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dgamma) dgamma[c] += sums[C + c];
  if (dbeta) dbeta[c] += sums[c];
}


// ---------------------------------------------------------------------------------------------
// Bandwidth-oriented variants for C % 8 == 0 and 256 % (C/8) == 0 (every ResNet/VGG width):
// each lane owns one fixed 8-channel column (per-channel parameters live in registers) and walks
// rows with stride 256/(C/8); U independent 16-B loads are in flight per lane.
constexpr int FU = 4;

__device__ __forceinline__ void unpack8(uint4 u, float* f) {
  f[0] = lo_bf(u.x); f[1] = hi_bf(u.x); f[2] = lo_bf(u.y); f[3] = hi_bf(u.y);
  f[4] = lo_bf(u.z); f[5] = hi_bf(u.z); f[6] = lo_bf(u.w); f[7] = hi_bf(u.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
}


__global__ __launch_bounds__(256) void bn_stats_fast(const bf16_t* __restrict__ x, float* __restrict__ stats, int M,
                                                     int C, int rpb) {
  __shared__ float red[2][256][8];
  const int cols = C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.f;
  for (int r = lr0 < RP ? r0 + lr0 : r1; r < r1; r += RP * FU) {
    uint4 v[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      int rr = r + u * RP;
      v[u] = rr < r1 ? *(const uint4*)(x + (size_t)rr * C + c0) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      float f[8]; unpack8(v[u], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) { s[e] += f[e]; q[e] += f[e] * f[e]; }
    }
  }
  col_reduce8(red, s, q, stats + (size_t)blockIdx.x * 2 * C, stats + (size_t)blockIdx.x * 2 * C + C, cols, c0);
}

// mask (optional, relu only): one bit per output element, bit e of byte (row*C + c0)/8 = [y > 0] for
// channel c0+e -- the ReLU mask the backward needs, 1/16 of the bytes of y.
typedef unsigned int v4u_bn_t __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld16_bn(const bf16_t* p) {
  if (NT) {
    v4u_bn_t v = __builtin_nontemporal_load((const v4u_bn_t*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *(const uint4*)p;
}

template <bool NT>
__global__ __launch_bounds__(256) void bn_apply_fast(const bf16_t* __restrict__ x, const float* __restrict__ ss,
                                                     const bf16_t* __restrict__ res, const float* __restrict__ rss,
                                                     bf16_t* __restrict__ y, uint8_t* __restrict__ mask, int M, int C,
                                                     int res_mode, int relu, int rpb, int ldy) {
  const int cols = C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  float sc[8], sh[8], rsc[8], rsh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = ss[c0 + e]; sh[e] = ss[C + c0 + e];
    rsc[e] = res_mode == 2 ? rss[c0 + e] : 1.f;
    rsh[e] = res_mode == 2 ? rss[C + c0 + e] : 0.f;
  }
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  for (int r = lr0 < RP ? r0 + lr0 : r1; r < r1; r += RP * FU) {
    uint4 v[FU], w[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      int rr = r + u * RP;
      bool ok = rr < r1;
      v[u] = ok ? ld16_bn<NT>(x + (size_t)rr * C + c0) : make_uint4(0, 0, 0, 0);
      if (res_mode) w[u] = ok ? ld16_bn<NT>(res + (size_t)rr * C + c0) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      int rr = r + u * RP;
      if (rr >= r1) break;
      float f[8]; unpack8(v[u], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fmaf(f[e], sc[e], sh[e]);
      if (res_mode) {
        float g[8]; unpack8(w[u], g);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += fmaf(g[e], rsc[e], rsh[e]);
      }
      if (relu) {
        uint32_t bits = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          bits |= (f[e] > 0.f ? 1u : 0u) << e;
          f[e] = fmaxf(f[e], 0.f);
        }
        if (mask) mask[((size_t)rr * C + c0) >> 3] = (uint8_t)bits;
      }
      *(uint4*)(y + (size_t)rr * ldy + c0) = pack8(f);  // ldy > C: a channel slice of a concat
    }
  }
}

// y = act(x*scale + shift + res[n][h*s][w*s]): identity residual read through a 1x1 stride-s
// subsample of the block input (slim resnet_v1 `subsample`), so the subsampled tensor is never stored.
__global__ __launch_bounds__(256) void bn_apply_res_strided(const bf16_t* __restrict__ x, const float* __restrict__ ss,
                                                            const bf16_t* __restrict__ res, bf16_t* __restrict__ y,
                                                            uint8_t* __restrict__ mask,
                                                            uint32_t M, int C, int relu, FastDiv fd_cols, FastDiv fd_Wo,
                                                            FastDiv fd_Ho, int Ho, int Wo, int Hi, int Wi, int s) {
  const uint32_t cols = C >> 3, total = M * cols;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t r = fdiv(i, fd_cols), c0 = (i - r * cols) * 8;
    const uint32_t t = fdiv(r, fd_Wo), w = r - t * Wo;
    const uint32_t n = fdiv(t, fd_Ho), h = t - n * Ho;
    const size_t rr = ((size_t)n * Hi + (size_t)h * s) * Wi + (size_t)w * s;
    float f[8], g[8];
    unpack8(*(const uint4*)(x + (size_t)r * C + c0), f);
    unpack8(*(const uint4*)(res + rr * C + c0), g);
    uint32_t bits = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      f[e] = fmaf(f[e], ss[c0 + e], ss[C + c0 + e]) + g[e];
      bits |= (f[e] > 0.f ? 1u : 0u) << e;
      if (relu) f[e] = fmaxf(f[e], 0.f);
    }
    if (relu && mask) mask[((size_t)r * C + c0) >> 3] = (uint8_t)bits;
    *(uint4*)(y + (size_t)r * C + c0) = pack8(f);
  }
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_fast(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ ym, const float* __restrict__ ss,
                                                          float* __restrict__ sums, int M, int C, int mask_mode, int rpb) {
  __shared__ float red[2][256][8];
  const int cols = C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  float sc[8], sh[8], mu[8], rs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = ss[c0 + e]; sh[e] = ss[C + c0 + e]; mu[e] = ss[2 * C + c0 + e]; rs[e] = ss[3 * C + c0 + e];
  }
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.f;
  for (int r = lr0 < RP ? r0 + lr0 : r1; r < r1; r += RP * FU) {
    uint4 a[FU], b[FU], m[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      int rr = r + u * RP;
      bool ok = rr < r1;
      size_t o = (size_t)rr * C + c0;
      a[u] = ok ? *(const uint4*)(dy + o) : make_uint4(0, 0, 0, 0);
      b[u] = ok ? *(const uint4*)(x + o) : make_uint4(0, 0, 0, 0);
      if (mask_mode == 1) m[u] = ok ? *(const uint4*)(ym + o) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      float g[8], xv[8];
      unpack8(a[u], g); unpack8(b[u], xv);
      if (mask_mode == 1) {
        float mv[8]; unpack8(m[u], mv);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = mv[e] > 0.f ? g[e] : 0.f;
      } else if (mask_mode == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = fmaf(xv[e], sc[e], sh[e]) > 0.f ? g[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) { s[e] += g[e]; q[e] += g[e] * (xv[e] - mu[e]) * rs[e]; }
    }
  }
  col_reduce8(red, s, q, sums + (size_t)blockIdx.x * 2 * C, sums + (size_t)blockIdx.x * 2 * C + C, cols, c0);
}

__global__ __launch_bounds__(256) void bn_bwd_apply_fast(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                         const bf16_t* __restrict__ ym, const float* __restrict__ ss,
                                                         const float* __restrict__ sums, bf16_t* __restrict__ dx,
                                                         bf16_t* __restrict__ gout, int M, int C, int mask_mode,
                                                         int training, int rpb) {
  const int cols = C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  const float invM = 1.f / (float)M;
  float sc[8], sh[8], mu[8], rs[8], A[8], Bq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = ss[c0 + e]; sh[e] = ss[C + c0 + e]; mu[e] = ss[2 * C + c0 + e]; rs[e] = ss[3 * C + c0 + e];
    A[e] = training ? sums[c0 + e] * invM : 0.f;
    Bq[e] = training ? sums[C + c0 + e] * invM : 0.f;
  }
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  for (int r = lr0 < RP ? r0 + lr0 : r1; r < r1; r += RP * FU) {
    uint4 a[FU], b[FU], m[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      int rr = r + u * RP;
      bool ok = rr < r1;
      size_t o = (size_t)rr * C + c0;
      a[u] = ok ? *(const uint4*)(dy + o) : make_uint4(0, 0, 0, 0);
      b[u] = ok ? *(const uint4*)(x + o) : make_uint4(0, 0, 0, 0);
      if (mask_mode == 1) m[u] = ok ? *(const uint4*)(ym + o) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < FU; ++u) {
      int rr = r + u * RP;
      if (rr >= r1) break;
      size_t o = (size_t)rr * C + c0;
      float g[8], xv[8];
      unpack8(a[u], g); unpack8(b[u], xv);
      if (mask_mode == 1) {
        float mv[8]; unpack8(m[u], mv);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = mv[e] > 0.f ? g[e] : 0.f;
      } else if (mask_mode == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = fmaf(xv[e], sc[e], sh[e]) > 0.f ? g[e] : 0.f;
      }
      if (gout) *(uint4*)(gout + o) = pack8(g);
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = sc[e] * (g[e] - A[e] - (xv[e] - mu[e]) * rs[e] * Bq[e]);
      *(uint4*)(dx + o) = pack8(d);
    }
  }
}

static bool fast_ok(long M, int C) {
  if (C % 8) return false;
  int cols = C / 8;
  return cols <= 256 && M < (1l << 31) && M * (long)C < (1l << 40);
}
// grid / rows-per-block for the column-fixed kernels: >= ~8 chunks per lane, <= 2048 blocks
static void fast_grid(long M, int C, int* blocks, int* rpb) {
  int cols = C / 8, RP = 256 / cols;
  long chunks = M * cols;
  long b = chunks / (256 * 8);
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  long r = (M + b - 1) / b;
  r = (r + RP - 1) / RP * RP;
  *rpb = (int)r;
  *blocks = (int)((M + r - 1) / r);
}
// ---- statistics reduction + finalize in one launch -------------------------------------------
// Partial rows ws[rows][2K] (sum | sumsq per producer tile) are summed column-wise by a 2-D grid into
// a self-cleaning fp32 accumulator with memory-side atomics; the last block to finish (counter) reads
// the totals back with atomic exchanges (which also re-zero the accumulator), and writes
// ss = [scale; shift; mean; rstd] and the moving averages -- the finalize of bn_finalize_kernel
// without a separate launch.  Correctness of the hand-off: each block's atomics complete (s_waitcnt in
// the issuing wave) before its counter increment, and the totals are read with memory-side atomics
// (never a stale L2 line of another XCD).
template <bool MULTI>
__global__ __launch_bounds__(256) void stats_reduce_finalize_kernel(
    const float* __restrict__ ws, int rows, int K, int rpb, float* acc, unsigned* counter,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ mov_mean,
    float* __restrict__ mov_var, float* __restrict__ out, float count, float eps, float decay, int update, int bessel,
    FinGroup grp) {
  __shared__ float4 red[16][16];
  __shared__ int is_last;
  const int width = 2 * K;
  const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = (blockIdx.x * 16 + cg) * 4;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < width) {
    int r = r0 + rl;
    for (; r + 48 < r1; r += 64) {
      float4 a = *(const float4*)(ws + (size_t)r * width + col);
      float4 b = *(const float4*)(ws + (size_t)(r + 16) * width + col);
      float4 c = *(const float4*)(ws + (size_t)(r + 32) * width + col);
      float4 d = *(const float4*)(ws + (size_t)(r + 48) * width + col);
      s.x += (a.x + b.x) + (c.x + d.x); s.y += (a.y + b.y) + (c.y + d.y);
      s.z += (a.z + b.z) + (c.z + d.z); s.w += (a.w + b.w) + (c.w + d.w);
    }
    for (; r < r1; r += 16) {
      float4 a = *(const float4*)(ws + (size_t)r * width + col);
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
  }
  red[rl][cg] = s;
  __syncthreads();
  if (rl == 0 && col < width) {
    float4 t = red[0][cg];
    for (int i = 1; i < 16; ++i) { float4 u = red[i][cg]; t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w; }
    atomicAdd(acc + col, t.x); atomicAdd(acc + col + 1, t.y);
    atomicAdd(acc + col + 2, t.z); atomicAdd(acc + col + 3, t.w);
  }
  // The partial-total atomics above are issued by wave 0 (rl == 0 <=> threadIdx.x < 16), the same wave
  // that bumps the counter: waiting for its memory counters to drain orders them before the bump
  // without an L2 write-back fence (all traffic here is memory-side atomics).
  static_assert(16 <= 64, "partial-total atomics must come from wave 0");
  if (threadIdx.x == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned nblk = gridDim.x * gridDim.y;
    is_last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1;
  }
  __syncthreads();
  if (!is_last) return;
  for (int cb = 0; cb < K; cb += 2048) {
    // all totals of this chunk are fetched (and re-zeroed) before any is used: 16 atomics in flight
    float sv[8], qv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = cb + i * 256 + threadIdx.x;
      sv[i] = c < K ? atomicExch(acc + c, 0.f) : 0.f;
      qv[i] = c < K ? atomicExch(acc + K + c, 0.f) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = cb + i * 256 + threadIdx.x;
      if (c >= K) break;
      if constexpr (MULTI) {
        FinMember mb = grp.m[0];
#pragma unroll
        for (int j = 1; j < 8; ++j)  // (constant indices: no scratch copy of the argument table)
          if (j < grp.n && c >= grp.m[j].off) mb = grp.m[j];
        if (mb.out)
          bn_fin_channel(sv[i], qv[i], c - mb.off, mb.K, mb.gamma, mb.beta, mb.mov_mean, mb.mov_var, mb.out, count,
                         eps, decay, update, bessel);
      } else {
        bn_fin_channel(sv[i], qv[i], c, K, gamma, beta, mov_mean, mov_var, out, count, eps, decay, update, bessel);
      }
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The same reduction + finalize when ONE block per column group covers every row (no cross-block sum): block b owns
// channels [32b, 32b + 32) - the 8 column quads of their sums AND the 8 of their sums of squares (16 quads x 16 row
// lanes) - so it finalizes them itself: no accumulator atomics, no completion counter, no last-block tail (the
// direct path measured 4-6 us cheaper per launch than the counter hand-off on ResNet-50's 196-row 14x14 / 7x7 maps).
// Summation order: per row lane a fixed row sequence, then the 16 lanes in order - deterministic.
template <bool MULTI>
__global__ __launch_bounds__(256) void stats_finalize_direct_kernel(
    const float* __restrict__ ws, int rows, int K, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ mov_mean, float* __restrict__ mov_var, float* __restrict__ out, float count, float eps,
    float decay, int update, int bessel, FinGroup grp) {
  __shared__ float4 red[16][16];
  const int width = 2 * K;
  const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int c0 = blockIdx.x * 32;
  // quads 0..7: sums of channels c0 + 4q .. +3; quads 8..15: their sums of squares
  const int ch = c0 + (cg & 7) * 4;
  const int col = (cg < 8 ? 0 : K) + ch;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ch < K) {
    int r = rl;
    for (; r + 48 < rows; r += 64) {
      float4 a = *(const float4*)(ws + (size_t)r * width + col);
      float4 b = *(const float4*)(ws + (size_t)(r + 16) * width + col);
      float4 c = *(const float4*)(ws + (size_t)(r + 32) * width + col);
      float4 d = *(const float4*)(ws + (size_t)(r + 48) * width + col);
      s.x += (a.x + b.x) + (c.x + d.x); s.y += (a.y + b.y) + (c.y + d.y);
      s.z += (a.z + b.z) + (c.z + d.z); s.w += (a.w + b.w) + (c.w + d.w);
    }
    for (; r < rows; r += 16) {
      float4 a = *(const float4*)(ws + (size_t)r * width + col);
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
  }
  red[rl][cg] = s;
  __syncthreads();
  if (threadIdx.x < 16) {
    float4 t = red[0][threadIdx.x];
    for (int i = 1; i < 16; ++i) { float4 u = red[i][threadIdx.x]; t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w; }
    red[0][threadIdx.x] = t;
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int c = c0 + threadIdx.x;
    if (c < K) {
      const float* q = (const float*)&red[0][0];
      const float sum = q[threadIdx.x], sq = q[32 + threadIdx.x];  // quad j holds channels 4j..4j+3
      if constexpr (MULTI) {
        FinMember mb = grp.m[0];
#pragma unroll
        for (int j = 1; j < 8; ++j)  // (constant indices: no scratch copy of the argument table)
          if (j < grp.n && c >= grp.m[j].off) mb = grp.m[j];
        if (mb.out)
          bn_fin_channel(sum, sq, c - mb.off, mb.K, mb.gamma, mb.beta, mb.mov_mean, mb.mov_var, mb.out, count, eps,
                         decay, update, bessel);
      } else {
        bn_fin_channel(sum, sq, c, K, gamma, beta, mov_mean, mov_var, out, count, eps, decay, update, bessel);
      }
    }
  }
}

}  // namespace dtm
using namespace dtm;

static int g_fin_direct = 1;  // A/B API (dtm_set_fin_direct): the one-block-per-channel-group finalize
DTM_API void dtm_set_fin_direct(int on) { g_fin_direct = on; }

static int grid_for(long work, int cap = 2048) {
  long b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}
static long rows_per_block_for(long M, int C) {
  // aim for ~1024 blocks, >= 64 rows each
  long r = (M + 1023) / 1024;
  if (r < 64) r = 64;
  return r;
}

// Backward of stats = [sum y; sum y^2] (per channel): dy = [g +] dstats[0] + 2 * y * dstats[1], bf16 out,
// one pass over y (8 channels per lane; C % 8 == 0).  Replaces five torch elementwise launches
// (float copy, two muls, add, bf16 copy) over the activation per call (Inception pool branches).
__global__ __launch_bounds__(256) void bn_stats_bwd_kernel(const bf16_t* __restrict__ y, const float* __restrict__ dstats,
                                                           const bf16_t* g, bf16_t* dy, long n8, int C8) {
  const int C = C8 * 8;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C8) * 8;
    float f[8];
    unpack8(((const uint4*)y)[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = dstats[c + j] + 2.0f * f[j] * dstats[C + c + j];
    if (g) {  // the tensor's other gradient (may alias dy: each lane reads its chunk before writing it)
      float h[8];
      unpack8(((const uint4*)g)[i], h);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += h[j];
    }
    ((uint4*)dy)[i] = pack8(f);
  }
}

DTM_API int dtm_bn_stats_bwd(const void* y, const float* dstats, const void* g, void* dy, long M, int C, void* stream) {
  if (C % 8) return -1;
  const long n8 = M * (C / 8);
  long blocks = (n8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(bn_stats_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)y,
                     dstats, (const bf16_t*)g, (bf16_t*)dy, n8, C / 8);
  return 0;
}

DTM_API void dtm_bn_stats(const void* x, float* stats, long M, int C, void* stream) {
  if (fast_ok(M, C)) {
    int blocks, rpb; fast_grid(M, C, &blocks, &rpb);
    float* ws = dtm_ws_get_stream((size_t)blocks * 2 * C, (hipStream_t)stream);
    hipLaunchKernelGGL(bn_stats_fast, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ws, (int)M, C, rpb);
    dtm_reduce_rows(ws, blocks, 2 * C, 2 * C, stats, (hipStream_t)stream);
    return;
  }
  long rpb = rows_per_block_for(M, C);
  int blocks = (int)((M + rpb - 1) / rpb);
  if (C % 8 == 0)
    hipLaunchKernelGGL(bn_stats_kernel<8>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, stats, M, C, rpb);
  else
    hipLaunchKernelGGL(bn_stats_kernel<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, stats, M, C, rpb);
}

// Column sums (and sums of squares) of x [M][C] into stats [2][C] (zeroed by the caller) in a fixed summation order:
// the bias gradients (ops/nn.py _col_sums) - deterministic run to run, unlike dtm_bn_stats' policy reduction.
DTM_API int dtm_col_sums(const void* x, float* stats, long M, int C, void* stream) {
  if (!fast_ok(M, C)) return -1;
  int blocks, rpb; fast_grid(M, C, &blocks, &rpb);
  float* ws = dtm_ws_get_stream((size_t)blocks * 2 * C, (hipStream_t)stream);
  if (!ws) return -4;
  hipLaunchKernelGGL(bn_stats_fast, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ws, (int)M, C, rpb);
  dtm_reduce_rows_det(ws, blocks, 2 * C, 2 * C, stats, (hipStream_t)stream);
  return 0;
}

DTM_API void dtm_bn_finalize(const float* stats, const float* gamma, const float* beta, float* mov_mean,
                             float* mov_var, float* out, int C, float count, float eps, float decay, int update,
                             int bessel, void* stream) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, stats, gamma, beta,
                     mov_mean, mov_var, out, C, count, eps, decay, update, bessel);
}

DTM_API void dtm_bn_inference_params(const float* gamma, const float* beta, const float* mov_mean,
                                     const float* mov_var, float* out, int C, float eps, void* stream) {
  hipLaunchKernelGGL(bn_inference_params_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, gamma, beta,
                     mov_mean, mov_var, out, C, eps);
}

// mask: optional ReLU bitmask output (fast path only; returns -7 when it cannot be produced)
DTM_API int dtm_bn_apply2(const void* x, const float* ss, const void* res, const float* rss, void* y, void* mask, long M,
                          int C, int res_mode, int relu, void* stream) {
  if (fast_ok(M, C)) {
    int blocks, rpb; fast_grid(M, C, &blocks, &rpb);
    hipLaunchKernelGGL((dtm_ntld_bits() & 1) ? bn_apply_fast<true> : bn_apply_fast<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ss,
                       (const bf16_t*)res, rss, (bf16_t*)y, (uint8_t*)mask, (int)M, C, res_mode, relu, rpb, C);
    return 0;
  }
  if (mask) return -7;
  if (C % 8 == 0)
    hipLaunchKernelGGL(bn_apply_kernel<8>, dim3(grid_for(M * C / 8)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, ss, (const bf16_t*)res, rss, (bf16_t*)y, M, C, res_mode, relu);
  else
    hipLaunchKernelGGL(bn_apply_kernel<1>, dim3(grid_for(M * C)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, ss, (const bf16_t*)res, rss, (bf16_t*)y, M, C, res_mode, relu);
  return 0;
}

// Zero-copy concat: y = relu?(x*scale + shift) written as channels [0, C) of rows of
// ldy channels -- the caller passes y = concat buffer + channel offset, so an Inception branch output
// lands in its slice of the block output and no concat copy exists.  16-B aligned slices only.
DTM_API int dtm_bn_apply_ld(const void* x, const float* ss, void* y, void* mask, long M, int C, int relu, int ldy,
                            void* stream) {
  if (!fast_ok(M, C) || ldy < C || ldy % 8 || ((uintptr_t)y & 15) || M * (long)ldy >= (1l << 40)) return -1;
  int blocks, rpb; fast_grid(M, C, &blocks, &rpb);
  hipLaunchKernelGGL((dtm_ntld_bits() & 1) ? bn_apply_fast<true> : bn_apply_fast<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ss,
                     (const bf16_t*)nullptr, (const float*)nullptr, (bf16_t*)y, (uint8_t*)mask, (int)M, C, 0, relu, rpb,
                     ldy);
  return 0;
}

DTM_API void dtm_bn_apply(const void* x, const float* ss, const void* res, const float* rss, void* y, long M, int C,
                          int res_mode, int relu, void* stream) {
  dtm_bn_apply2(x, ss, res, rss, y, nullptr, M, C, res_mode, relu, stream);
}

// res [N][Hi][Wi][C] read at (n, h*s, w*s) for every output pixel of x / y [N][Ho][Wo][C]
DTM_API int dtm_bn_apply_res_strided(const void* x, const float* ss, const void* res, void* y, void* mask, int N, int Ho,
                                     int Wo, int C, int Hi, int Wi, int s, int relu, void* stream) {
  if (C % 8 || (long)N * Ho * Wo * (C / 8) >= (1l << 31) || (Ho - 1) * s >= Hi || (Wo - 1) * s >= Wi) return -1;
  const uint32_t M = (uint32_t)N * Ho * Wo;
  const long total = (long)M * (C / 8);
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(bn_apply_res_strided, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ss,
                     (const bf16_t*)res, (bf16_t*)y, (uint8_t*)mask, M, C, relu, make_fastdiv(C / 8), make_fastdiv(Wo),
                     make_fastdiv(Ho), Ho, Wo, Hi, Wi, s);
  return 0;
}

DTM_API void dtm_bn_bwd_reduce(const void* dy, const void* x, const void* ymask, const float* ss, float* sums, long M,
                               int C, int mask_mode, void* stream) {
  if (fast_ok(M, C)) {
    int blocks, rpb; fast_grid(M, C, &blocks, &rpb);
    float* ws = dtm_ws_get_stream((size_t)blocks * 2 * C, (hipStream_t)stream);
    hipLaunchKernelGGL(bn_bwd_reduce_fast, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const bf16_t*)x, (const bf16_t*)ymask, ss, ws, (int)M, C, mask_mode, rpb);
    dtm_reduce_rows(ws, blocks, 2 * C, 2 * C, sums, (hipStream_t)stream);
    return;
  }
  long rpb = rows_per_block_for(M, C);
  int blocks = (int)((M + rpb - 1) / rpb);
  if (C % 8 == 0)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<8>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const bf16_t*)x, (const bf16_t*)ymask, ss, sums, M, C, mask_mode, rpb);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const bf16_t*)x, (const bf16_t*)ymask, ss, sums, M, C, mask_mode, rpb);
}

DTM_API void dtm_bn_bwd_apply(const void* dy, const void* x, const void* ymask, const float* ss, const float* sums,
                              void* dx, void* gout, long M, int C, int mask_mode, int training, void* stream) {
  if (fast_ok(M, C)) {
    int blocks, rpb; fast_grid(M, C, &blocks, &rpb);
    hipLaunchKernelGGL(bn_bwd_apply_fast, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const bf16_t*)x, (const bf16_t*)ymask, ss, sums, (bf16_t*)dx, (bf16_t*)gout, (int)M, C,
                       mask_mode, training, rpb);
    return;
  }
  if (C % 8 == 0)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<8>, dim3(grid_for(M * C / 8)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)ymask, ss, sums, (bf16_t*)dx, (bf16_t*)gout,
                       M, C, mask_mode, training);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<1>, dim3(grid_for(M * C)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)ymask, ss, sums, (bf16_t*)dx, (bf16_t*)gout,
                       M, C, mask_mode, training);
}

DTM_API void dtm_bn_param_grad(const float* sums, float* dgamma, float* dbeta, int C, void* stream) {
  hipLaunchKernelGGL(bn_param_grad_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, sums, dgamma,
                     dbeta, C);
}

// self-cleaning accumulator + completion counter for stats_reduce_finalize (stream-ordered use; one per
// scratch slot: finalizes on concurrent streams never share them)
static float* g_fin_acc[DTM_WS_SLOTS] = {};
static unsigned* g_fin_counter[DTM_WS_SLOTS] = {};
static int g_fin_k[DTM_WS_SLOTS] = {};

// ss[4][K] (+ moving averages) from the partial statistics rows ws[rows][2K], one launch.  fg (optional): the
// K columns belong to several BatchNorms (FinGroup, common.h).
int dtm_bn_stats_finalize(const float* ws, int rows, int K, const float* gamma, const float* beta, float* mov_mean,
                          float* mov_var, float* ss, float count, float eps, float decay, int update, int bessel,
                          hipStream_t st) {
  return dtm_bn_stats_finalize_g(ws, rows, K, gamma, beta, mov_mean, mov_var, ss, count, eps, decay, update, bessel, st,
                                 nullptr);
}
int dtm_bn_stats_finalize_g(const float* ws, int rows, int K, const float* gamma, const float* beta, float* mov_mean,
                            float* mov_var, float* ss, float count, float eps, float decay, int update, int bessel,
                            hipStream_t st, const FinGroup* fg) {
  if (!dtm_device_ok()) return -9;
  const int k = dtm_ws_slot(st);
  if (K > g_fin_k[k]) {
    // graph-safe growth (workspace.hip dtm_ws_get_stream): never inside a capture, the old accumulator kept
    if (dtm_stream_capturing(st)) {
      dtm_ws_set_error(-10);
      return -4;
    }
    unsigned* cnt = nullptr;
    float* acc = nullptr;
    if (hipMalloc(&cnt, 64) != hipSuccess) return -4;
    if (hipMalloc(&acc, (size_t)2 * K * sizeof(float)) != hipSuccess) return -4;
    // zeroed in stream order (kernels still queued on st keep using the old pair)
    hipMemsetAsync(acc, 0, (size_t)2 * K * sizeof(float), st);
    hipMemsetAsync(cnt, 0, 64, st);
    if (g_fin_acc[k]) dtm_ws_note_retired();
    g_fin_acc[k] = acc;
    g_fin_counter[k] = cnt;
    g_fin_k[k] = K;
  }
  if (K % 2) return -1;  // float4 columns over [2K]
  int rpb, ychunks;
  dtm_reduce_split(rows, (2 * K + 63) / 64, &rpb, &ychunks);
  if (ychunks == 1 && K % 4 == 0 && g_fin_direct) {
    // every column's rows in one block: that block finalizes its channels itself
    if (fg) {
      hipLaunchKernelGGL(stats_finalize_direct_kernel<true>, dim3((K + 31) / 32), dim3(256), 0, st, ws, rows, K, gamma,
                         beta, mov_mean, mov_var, ss, count, eps, decay, update, bessel, *fg);
    } else {
      FinGroup none;
      none.n = 0;
      hipLaunchKernelGGL(stats_finalize_direct_kernel<false>, dim3((K + 31) / 32), dim3(256), 0, st, ws, rows, K, gamma,
                         beta, mov_mean, mov_var, ss, count, eps, decay, update, bessel, none);
    }
    return 0;
  }
  if (fg) {
    hipLaunchKernelGGL(stats_reduce_finalize_kernel<true>, dim3((2 * K + 63) / 64, ychunks), dim3(256), 0, st, ws, rows,
                       K, rpb, g_fin_acc[k], g_fin_counter[k], gamma, beta, mov_mean, mov_var, ss, count, eps, decay,
                       update, bessel, *fg);
  } else {
    FinGroup none;
    none.n = 0;
    hipLaunchKernelGGL(stats_reduce_finalize_kernel<false>, dim3((2 * K + 63) / 64, ychunks), dim3(256), 0, st, ws,
                       rows, K, rpb, g_fin_acc[k], g_fin_counter[k], gamma, beta, mov_mean, mov_var, ss, count, eps,
                       decay, update, bessel, none);
  }
  return 0;
}
