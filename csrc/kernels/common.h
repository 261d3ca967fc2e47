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

// XCD-aware block remap (8 XCDs, each with its own L2; the hardware deals workgroup L to XCD L % 8):
// returns a logical tile id such that the workgroups of one XCD get a contiguous logical range, so
// the tiles that share an operand (all channel tiles of one pixel tile, all tiles of one split, the
// overlapping windows of a pool) hit the same L2.  Bijective for any count (guide T1).
__device__ __forceinline__ int xcd_remap(int L, int nwg) {
  const int xcd = L & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
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
void dtm_reduce_rows(const float* ws, int rows, int width, int ld, float* out, hipStream_t st);
void dtm_reduce_rows_det(const float* ws, int rows, int width, int ld, float* out, hipStream_t st);
// several row-sum reductions over the same rows (column segments of one partial-sum table, each into its own output:
// the split-K slabs of a merged sibling weight gradient) in ONE launch (n <= 8)
void dtm_reduce_rows_multi(const float* const* ws, const int* widths, float* const* outs, int n, int rows, int ld,
                           hipStream_t st);
constexpr int DTM_WS_SLOTS = 5;
float* dtm_ws_get_stream(size_t floats, hipStream_t st);  // scratch arena of the stream's slot
bool dtm_stream_capturing(hipStream_t st);  // st is being captured into a hipGraph
void dtm_ws_set_error(int e);               // -10: growth refused during capture, -4: out of memory
void dtm_ws_note_retired();
int dtm_ws_slot(hipStream_t st);  // 0 = main, 1.. = registered side streams
bool dtm_device_ok();  // false when called from another device than the first one used
int dtm_compute_cus();  // CUs the persistent / split-K grids size for: the device's CUs minus the reserved ones
void dtm_reduce_split(int rows, int xblocks, int* rpb, int* ychunks);
int dtm_reduce_direct_max();
int dtm_ntld_bits();  // non-temporal input-load policy of the BN-apply kernels (fused_bn.hip)  // grids up to this many blocks reduce with atomics in the producer
// FinGroup (merged sibling convs, ops/fused.py): the K columns of one statistics table are several BatchNorms side by
// side - member j owns columns [off_j, off_j + K_j) and its own parameters / moving statistics / ss output (out ==
// nullptr: a member without BatchNorm, e.g. Inception's commuted pool-branch conv, whose statistics are unused)
struct FinMember {
  const float* gamma;
  const float* beta;
  float* mov_mean;
  float* mov_var;
  float* out;
  int off, K;
};
struct FinGroup {
  int n;
  FinMember m[8];
};
int dtm_bn_stats_finalize_g(const float* ws, int rows, int K, const float* gamma, const float* beta, float* mov_mean,
                            float* mov_var, float* ss, float count, float eps, float decay, int update, int bessel,
                            hipStream_t st, const FinGroup* fg);
int dtm_bn_stats_finalize(const float* ws, int rows, int K, const float* gamma, const float* beta, float* mov_mean,
                          float* mov_var, float* ss, float count, float eps, float decay, int update, int bessel,
                          hipStream_t st);

// Column-fixed lane mapping used by the BN kernels: lane t owns channel block (t % cols) * 8 and
// row-lane t / cols; with RP = 256 / cols row-lanes, lanes >= RP*cols idle (C/8 need not divide 256).
// col_reduce8 sums the per-lane [8] partials of the RP row-lanes of each column in LDS and writes
// the per-block partial row out0[c0..c0+7], out1[...] (plain stores; reduced later by reduce_rows).
// atomic: add into the final [C] sums instead (small grids: one launch fewer, <= a few hundred
// adders per address).
template <int NT = 256>
__device__ __forceinline__ void col_reduce8(float (*red)[NT][8], const float* s, const float* q, float* out0,
                                            float* out1, int cols, int c0, bool atomic = false) {
  const int t = threadIdx.x, RP = NT / cols;  // (NT: the red table's rows; blocks of cols * (NT / cols) lanes)
  if (RP == 1) {
    if (t < cols) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (atomic) { atomicAdd(out0 + c0 + e, s[e]); atomicAdd(out1 + c0 + e, q[e]); }
        else { out0[c0 + e] = s[e]; out1[c0 + e] = q[e]; }
      }
    }
    return;
  }
  __syncthreads();  // red may still be read by a previous call
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[0][t][e] = s[e]; red[1][t][e] = q[e]; }
  __syncthreads();
  int P = 1;
  while (P * 2 <= RP) P *= 2;
  if (P < RP) {  // fold the row-lanes beyond the largest power of two
    if (t < (RP - P) * cols) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { red[0][t][e] += red[0][t + P * cols][e]; red[1][t][e] += red[1][t + P * cols][e]; }
    }
    __syncthreads();
  }
  for (int h = P / 2; h >= 1; h >>= 1) {
    if (t < h * cols) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { red[0][t][e] += red[0][t + h * cols][e]; red[1][t][e] += red[1][t + h * cols][e]; }
    }
    __syncthreads();
  }
  if (t < cols) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (atomic) { atomicAdd(out0 + c0 + e, red[0][t][e]); atomicAdd(out1 + c0 + e, red[1][t][e]); }
      else { out0[c0 + e] = red[0][t][e]; out1[c0 + e] = red[1][t][e]; }
    }
  }
}

namespace dtm {
// BatchNorm finalize backward of one channel (bn_finalize_bwd_kernel's algebra): from dss = [dscale;
// dshift; dmean; drstd], ss = [scale; shift; mean; rstd] and gamma -> the statistics gradient
// (ds = d/dsum, dq = d/dsumsq, divided by the count) and the parameter gradients dg, db.
// training BatchNorm finalize of one channel from the batch sums: ss = [scale; shift; mean; rstd] (out[c],
// out[K+c], ...) and the moving averages (shared by stats_reduce_finalize and the conv epilogue's hand-off)
__device__ __forceinline__ void bn_fin_channel(float sum, float sq, int c, int K, const float* gamma, const float* beta,
                                               float* mov_mean, float* mov_var, float* out, float count, float eps,
                                               float decay, int update, int bessel) {
  const float mean = sum / count;
  const float var = fmaxf(sq / count - mean * mean, 0.f);
  const float rstd = rsqrtf(var + eps);
  const float sc = (gamma ? gamma[c] : 1.f) * rstd;
  out[c] = sc;
  out[K + c] = (beta ? beta[c] : 0.f) - mean * sc;
  out[2 * K + c] = mean;
  out[3 * K + c] = rstd;
  if (update) {
    const float uvar = (bessel && count > 1.f) ? var * count / (count - 1.f) : var;
    mov_mean[c] -= (mov_mean[c] - mean) * (1.f - decay);
    mov_var[c] -= (mov_var[c] - uvar) * (1.f - decay);
  }
}

__device__ __forceinline__ void fin_bwd_channel(const float* dss, const float* ss, const float* gamma, int C, int c,
                                                float count, float* ds, float* dq, float* dg, float* db) {
  const float scale = ss[c], mean = ss[2 * C + c], rstd = ss[3 * C + c];
  const float g = gamma ? gamma[c] : 1.f;
  const float dsc = dss[c], dsh = dss[C + c];
  const float dscale_tot = dsc - dsh * mean;
  const float dmean = dss[2 * C + c] - dsh * scale;
  const float drstd = dss[3 * C + c] + dscale_tot * g;
  const float dvar = drstd * (-0.5f) * rstd * rstd * rstd;
  *ds = dmean / count - dvar * 2.f * mean / count;
  *dq = dvar / count;
  *dg = dscale_tot * rstd;
  *db = dsh;
}
}  // namespace dtm
