// Shared device helpers for the gfx950 (CDNA4) kernel library.
// Activations are NHWC bf16, accumulation fp32, per-channel statistics fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // raw bf16 storage
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define DTM_API extern "C" __attribute__((visibility("default")))

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even; hipcc lowers the __bf16 cast to v_cvt_pk_bf16_f32 (NaN-preserving)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// Buffer resource for bounds-checked loads: an offset >= num_bytes reads zero (used for
// implicit zero padding in the implicit-GEMM gathers).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t num_bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)num_bytes, 0x00020000);
}
#define OOB_OFFSET 0x80000000u

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// magic-number unsigned division (host computes m, s): q = mulhi(n, m) >> s  for n < 2^31
struct FastDiv {
  uint32_t d, m, s;
};
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;  // valid for d>=1 with m computed as below
}
__host__ static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f; f.d = d;
  if (d == 1) { f.m = 0; f.s = 0; return f; }
  uint32_t s = 0; while ((1ull << s) < d) ++s;          // s = ceil(log2 d)
  uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  f.m = (uint32_t)m; f.s = s;
  return f;
}

// workspace arena + two-stage reduction (workspace.hip)
float* dtm_ws_get(size_t floats);
void dtm_reduce_rows(const float* ws, int rows, int width, int ld, float* out, hipStream_t st);
