// Device scratch arena for two-stage (contention-free) per-channel reductions.
//
// Reductions over B*H*W rows write one partial row per workgroup (plain stores, no atomics);
// `reduce_rows` then sums the rows with a handful of atomics per output.  (fp32 atomics from
// thousands of workgroups onto the same few hundred addresses serialise at the memory-side
// atomic units -- measured 10-100x slower on MI355X than this two-stage form.)
// The arena grows on first use (warm-up step, before any hipGraph capture) and is reused.
#include "common.h"

static float* g_ws = nullptr;
static size_t g_ws_floats = 0;

float* dtm_ws_get(size_t floats) {
  if (floats > g_ws_floats) {
    size_t n = floats < (16u << 20) ? (16u << 20) : floats;  // >= 64 MB
    if (g_ws) {
      hipDeviceSynchronize();
      hipFree(g_ws);
    }
    if (hipMalloc(&g_ws, n * sizeof(float)) != hipSuccess) {
      g_ws = nullptr;
      g_ws_floats = 0;
      return nullptr;
    }
    g_ws_floats = n;
  }
  return g_ws;
}

// out[j] (+)= sum_r ws[r*ld + j], j < width
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ ws, int rows, int width, int ld,
                                                          float* __restrict__ out, int chunks) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= width) return;
  float s = 0.f;
  for (int r = blockIdx.y; r < rows; r += chunks) s += ws[(size_t)r * ld + j];
  if (chunks == 1) out[j] += s;
  else atomicAdd(out + j, s);
}

void dtm_reduce_rows(const float* ws, int rows, int width, int ld, float* out, hipStream_t st) {
  int chunks = rows >= 512 ? 32 : (rows >= 64 ? 8 : 1);
  hipLaunchKernelGGL(reduce_rows_kernel, dim3((width + 255) / 256, chunks), dim3(256), 0, st, ws, rows, width, ld, out,
                     chunks);
}

DTM_API int dtm_ws_reserve(long floats) { return dtm_ws_get((size_t)floats) ? 0 : -1; }
