// Stand-alone elementwise kernels for the non-fused model-zoo call sites.
//
// Dropout (slim.dropout / old-slim ops.dropout, reference
// inception/slim/ops.py:406-424): a counter-based hash of (seed, element index) gives the keep
// decision, so the mask is never stored - backward regenerates it from the same seed.
// y = keep ? x / keep_prob : 0.  8 elements (one 16-byte bf16 vector / two fp32 vectors) per thread.
//
// InTopK (K21; the evaluators' precision@1 / recall@5, reference inception/inception_eval.py:
// 105-127, cnn/cifar10_eval.py:76): TF semantics - target t is in the top k iff fewer than k
// logits are strictly greater than logit[t] (ties at the boundary count as in), and a non-finite
// target logit or an out-of-range label is never in.  One wave64 per row.
#include "common.h"

namespace dtm {

// 32-bit avalanche hash of a 64-bit counter mixed with the seed (splitmix64 finaliser)
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

// Per-step stream offset: a device counter the training engine advances once per step, read by
// the kernel at run time, so a step replayed from a hipGraph (seed baked in at capture) still
// draws a fresh mask every step.  off == 0 leaves the seed untouched (bit-identical CPU form).
__device__ __forceinline__ uint64_t mix_seed(uint64_t seed, uint64_t off) {
  if (off == 0) return seed;
  uint64_t z = off * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return seed ^ z ^ (z >> 31);
}

// keep iff hash < keep_prob * 2^32 (threshold computed on the host)
template <bool BF16>
__global__ __launch_bounds__(256) void dropout_kernel(const void* __restrict__ xv, void* __restrict__ yv, long n,
                                                      uint32_t thresh, float inv_keep, uint64_t seed0,
                                                      const unsigned long long* __restrict__ seed_off) {
  const long base = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (base >= n) return;
  const uint64_t seed = seed_off ? mix_seed(seed0, *seed_off) : seed0;
  float v[8];
  if (BF16) {
    const bf16_t* x = (const bf16_t*)xv;
    if (base + 8 <= n) {
      uint4 u = *(const uint4*)(x + base);
      uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf(w[j]); v[2 * j + 1] = hi_bf(w[j]); }
    } else {
      for (int j = 0; j < 8; ++j) v[j] = base + j < n ? bf2f(x[base + j]) : 0.f;
    }
  } else {
    const float* x = (const float*)xv;
    if (base + 8 <= n) {
      float4 a = *(const float4*)(x + base), b = *(const float4*)(x + base + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      for (int j = 0; j < 8; ++j) v[j] = base + j < n ? x[base + j] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = hash_u32(seed, (uint64_t)(base + j)) < thresh ? v[j] * inv_keep : 0.f;
  if (BF16) {
    bf16_t* y = (bf16_t*)yv;
    if (base + 8 <= n) {
      uint4 u;
      u.x = pack2bf(v[0], v[1]); u.y = pack2bf(v[2], v[3]); u.z = pack2bf(v[4], v[5]); u.w = pack2bf(v[6], v[7]);
      *(uint4*)(y + base) = u;
    } else {
      for (int j = 0; j < 8; ++j) if (base + j < n) y[base + j] = f2bf(v[j]);
    }
  } else {
    float* y = (float*)yv;
    if (base + 8 <= n) {
      *(float4*)(y + base) = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(y + base + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      for (int j = 0; j < 8; ++j) if (base + j < n) y[base + j] = v[j];
    }
  }
}

template <bool BF16>
__global__ __launch_bounds__(256) void in_top_k_kernel(const void* __restrict__ logits, const int* __restrict__ labels,
                                                       uint8_t* __restrict__ out, int B, int K, int k) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  const int t = labels[row];
  auto ld = [&](long i) -> float {
    return BF16 ? bf2f(((const bf16_t*)logits)[i]) : ((const float*)logits)[i];
  };
  const long off = (long)row * K;
  const bool valid = t >= 0 && t < K;
  const float xt = valid ? ld(off + t) : 0.f;
  int cnt = 0;
  for (int c = lane; c < K; c += 64) cnt += ld(off + c) > xt ? 1 : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (lane == 0) out[row] = (valid && isfinite(xt) && cnt < k) ? 1 : 0;
}

// Packed-row stem input (fused.py _StemConvBNFn): xp[n][h][w][0..3] = x[n][h-pad][w-pad][c] (c < C, else 0),
// zero outside the image, as bf16 -- the zero border, the channel padding to 4 and the dtype conversion
// in one pass (one thread = two 8-byte output pixels = one 16-B store) instead of a fill + a pad copy.
template <bool F32>
__global__ __launch_bounds__(256) void stem_pack_kernel(const void* __restrict__ x, bf16_t* __restrict__ xp, int N,
                                                        int H, int W, int C, int Hp, int Wp, int pad) {
  const long npair = (long)N * Hp * (Wp / 2);
  for (long t = blockIdx.x * 256L + threadIdx.x; t < npair; t += (long)gridDim.x * 256) {
    const int w0 = (int)(t % (Wp / 2)) * 2;
    const long nh = t / (Wp / 2);
    const int h = (int)(nh % Hp), n = (int)(nh / Hp);
    const int ih = h - pad;
    uint32_t o[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int iw = w0 + k - pad;
      if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
        const long base = (((long)n * H + ih) * W + iw) * C;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < C; ++c)
          v[c] = F32 ? ((const float*)x)[base + c] : __uint_as_float((uint32_t)((const uint16_t*)x)[base + c] << 16);
        o[2 * k] = pack2bf(v[0], v[1]);
        o[2 * k + 1] = pack2bf(v[2], v[3]);
      }
    }
    *(uint4*)(xp + (nh * Wp + w0) * 4) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace dtm

using namespace dtm;

// dtype: 0 = fp32, 1 = bf16 input; Wp even, C <= 4
DTM_API int dtm_stem_pack(const void* x, int dtype, void* xp, int N, int H, int W, int C, int Hp, int Wp, int pad,
                          hipStream_t st) {
  if (C < 1 || C > 4 || (Wp & 1) || ((uintptr_t)xp & 15)) return -1;
  const long npair = (long)N * Hp * (Wp / 2);
  long blocks = (npair + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (dtype == 0)
    stem_pack_kernel<true><<<(unsigned)blocks, 256, 0, st>>>(x, (bf16_t*)xp, N, H, W, C, Hp, Wp, pad);
  else
    stem_pack_kernel<false><<<(unsigned)blocks, 256, 0, st>>>(x, (bf16_t*)xp, N, H, W, C, Hp, Wp, pad);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// dtype: 0 = fp32, 1 = bf16.  Same seed => same mask (backward passes the upstream gradient).
DTM_API int dtm_dropout(const void* x, void* y, long n, int dtype, float keep_prob, unsigned long long seed,
                        const unsigned long long* seed_off, hipStream_t st) {
  if (n <= 0) return 0;
  if (!(keep_prob > 0.f && keep_prob <= 1.f)) return 1;
  const double t = (double)keep_prob * 4294967296.0;
  const uint32_t thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  const long threads = (n + 7) / 8;
  const unsigned grid = (unsigned)((threads + 255) / 256);
  if (dtype == 1)
    dropout_kernel<true><<<grid, 256, 0, st>>>(x, y, n, thresh, 1.f / keep_prob, seed, seed_off);
  else
    dropout_kernel<false><<<grid, 256, 0, st>>>(x, y, n, thresh, 1.f / keep_prob, seed, seed_off);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

DTM_API int dtm_in_top_k(const void* logits, const int* labels, uint8_t* out, int B, int K, int k, int dtype,
                         hipStream_t st) {
  if (B <= 0) return 0;
  const unsigned grid = (unsigned)((B + 3) / 4);
  if (dtype == 1)
    in_top_k_kernel<true><<<grid, 256, 0, st>>>(logits, labels, out, B, K, k);
  else
    in_top_k_kernel<false><<<grid, 256, 0, st>>>(logits, labels, out, B, K, k);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
