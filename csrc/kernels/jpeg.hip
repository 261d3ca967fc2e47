// Device stage of the split JPEG decode: dequantization + 8x8 inverse DCT of the
// host-entropy-decoded coefficient blocks (csrc/runtime/jpeg.cpp), then chroma upsampling + YCbCr -> RGB,
// for a whole batch of images in two launches.  Bit-exact with libjpeg(-turbo)'s default decompression
// (what tf.image.decode_jpeg in the reference, inception/image_processing.py:339-407, and PIL run): the
// accurate integer IDCT ("islow", jidctint.c) with its post-IDCT range-limit table, "fancy" triangular
// h2v1 / h2v2 / h1v2 upsampling with edge replication, and jdcolor.c's fixed-point tables.  The output is
// the packed HxWx3 uint8 ragged buffer that dtm_imagenet_prep (image.hip) consumes.
#include "common.h"

namespace dtm {

// one image of the batch (mirrored in data/jpeg.py JPEG_DESC_DT)
struct JpegDesc {
  long long coef_base;   // int16 offset of the image's coefficients in the batch coefficient buffer
  long long plane_base;  // byte offset of its component planes in the plane scratch
  long long rgb_off;     // byte offset of its HxWx3 output in the RGB buffer
  int width, height, ncomp, hmax, vmax;
  int h[3], v[3], bw[3], bh[3], coef_off[3];
  int nblocks;           // sum of bw * bh over the components
  int pad;
  unsigned short qt[3][64];
};

constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
              F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }
__device__ __forceinline__ unsigned idct_limit(int x) {  // libjpeg's post-IDCT range-limit table
  const int i = x & 1023;
  return i < 128 ? i + 128 : (i < 512 ? 255 : (i < 896 ? 0 : i - 896));
}

// 1-D islow butterfly over 8 values (even part from v0, v2, v4, v6; odd from v1, v3, v5, v7)
__device__ __forceinline__ void idct8(const int* v, int* o, int shift_even_in) {
  int z2 = v[2], z3 = v[6];
  int z1 = (z2 + z3) * F0541;
  int tmp2 = z1 + z3 * (-F1847), tmp3 = z1 + z2 * F0765;
  int tmp0 = (v[0] + v[4]) * (1 << CONST_BITS), tmp1 = (v[0] - v[4]) * (1 << CONST_BITS);
  const int t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
  tmp0 = v[7]; tmp1 = v[5]; tmp2 = v[3]; tmp3 = v[1];
  z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
  int z4 = tmp1 + tmp3;
  const int z5 = (z3 + z4) * F1175;
  tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
  z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
  z3 += z5; z4 += z5;
  tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
  o[0] = t10 + tmp3; o[7] = t10 - tmp3; o[1] = t11 + tmp2; o[6] = t11 - tmp2;
  o[2] = t12 + tmp1; o[5] = t12 - tmp1; o[3] = t13 + tmp0; o[4] = t13 - tmp0;
  (void)shift_even_in;
}

// IDCT: grid (ceil(max blocks per image / 32), images); 8 threads per 8x8 block, 32 blocks per workgroup.
// Thread t of a block: loads row t of the coefficients, does column t of pass 1 and row t of pass 2.
__global__ __launch_bounds__(256) void jpeg_idct_kernel(const short* __restrict__ coefs, const JpegDesc* __restrict__ descs,
                                                        unsigned char* __restrict__ planes) {
  __shared__ short s_in[32][64];
  __shared__ int s_ws[32][64];
  const JpegDesc& d = descs[blockIdx.y];
  const int lb = threadIdx.x >> 3, t = threadIdx.x & 7;
  const int b = blockIdx.x * 32 + lb;  // block index within the image (components back to back)
  const bool valid = b < d.nblocks;
  int c = 0, bi = b;
  if (valid) {
    while (c < d.ncomp - 1 && bi >= d.bw[c] * d.bh[c]) {
      bi -= d.bw[c] * d.bh[c];
      ++c;
    }
  }
  const short* blk = coefs + d.coef_base + d.coef_off[c] + (long long)bi * 64;
  if (valid) *(uint4*)&s_in[lb][t * 8] = *(const uint4*)(blk + t * 8);
  __syncthreads();
  if (valid) {
    // pass 1: column t (dequantized), DC-only shortcut as in jidctint.c
    const unsigned short* q = d.qt[c];
    int v[8], o[8];
    bool ac0 = true;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      v[r] = (int)s_in[lb][r * 8 + t] * (int)q[r * 8 + t];
      if (r) ac0 &= v[r] == 0;
    }
    if (ac0) {
#pragma unroll
      for (int r = 0; r < 8; ++r) s_ws[lb][r * 8 + t] = v[0] * (1 << PASS1_BITS);
    } else {
      idct8(v, o, 0);
#pragma unroll
      for (int r = 0; r < 8; ++r) s_ws[lb][r * 8 + t] = descale(o[r], CONST_BITS - PASS1_BITS);
    }
  }
  __syncthreads();
  if (valid) {
    // pass 2: row t -> 8 output samples
    int v[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s_ws[lb][t * 8 + k];
    idct8(v, o, 0);
    unsigned w0 = 0, w1 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w0 |= idct_limit(descale(o[k], CONST_BITS + PASS1_BITS + 3)) << (8 * k);
      w1 |= idct_limit(descale(o[k + 4], CONST_BITS + PASS1_BITS + 3)) << (8 * k);
    }
    // plane of component c: pitch bw*8, the block at (bi / bw, bi % bw)
    long long pbase = d.plane_base;
    for (int cc = 0; cc < c; ++cc) pbase += (long long)d.bw[cc] * 8 * d.bh[cc] * 8;
    const int pw = d.bw[c] * 8;
    const int by = bi / d.bw[c], bx = bi - by * d.bw[c];
    *(uint2*)(planes + pbase + (long long)(by * 8 + t) * pw + bx * 8) = make_uint2(w0, w1);
  }
}

// fancy upsampling of one chroma sample for full-resolution pixel (y, x) (see jpeg.cpp fancy())
__device__ __forceinline__ int fancy_up(const unsigned char* pl, int pw, int cw, int ch, int fx, int fy, int y, int x) {
  if (fx == 1 && fy == 1) return pl[y * pw + x];
  if (fy == 1) {
    const int i = x >> 1;
    const int c = pl[y * pw + i];
    if (x & 1) return i == cw - 1 ? c : (c * 3 + pl[y * pw + i + 1] + 2) >> 2;
    return i == 0 ? c : (c * 3 + pl[y * pw + i - 1] + 1) >> 2;
  }
  const int j = y >> 1;
  int jo = (y & 1) ? j + 1 : j - 1;
  jo = jo < 0 ? 0 : (jo > ch - 1 ? ch - 1 : jo);
  const unsigned char* r0 = pl + j * pw;
  const unsigned char* r1 = pl + jo * pw;
  if (fx == 1) return (r0[x] * 3 + r1[x] + 1 + (y & 1)) >> 2;
  const int i = x >> 1;
  const int cs = r0[i] * 3 + r1[i];
  if (x & 1) {
    if (i == cw - 1) return (cs * 4 + 7) >> 4;
    return (cs * 3 + r0[i + 1] * 3 + r1[i + 1] + 7) >> 4;
  }
  if (i == 0) return (cs * 4 + 8) >> 4;
  return (cs * 3 + r0[i - 1] * 3 + r1[i - 1] + 8) >> 4;
}

__device__ __forceinline__ unsigned clamp255(int v) { return v < 0 ? 0u : (v > 255 ? 255u : (unsigned)v); }

// colour: grid (ceil(max pixels per image / 1024), images), 4 consecutive pixels (12 bytes) per thread
__global__ __launch_bounds__(256) void jpeg_color_kernel(const JpegDesc* __restrict__ descs,
                                                         const unsigned char* __restrict__ planes,
                                                         unsigned char* __restrict__ rgb) {
  const JpegDesc& d = descs[blockIdx.y];
  const long long npix = (long long)d.width * d.height;
  const long long p0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (p0 >= npix) return;
  const unsigned char* pY = planes + d.plane_base;
  const int pw0 = d.bw[0] * 8;
  unsigned char* out = rgb + d.rgb_off;
  if (d.ncomp == 1) {
    for (int k = 0; k < 4 && p0 + k < npix; ++k) {
      const int y = (int)((p0 + k) / d.width), x = (int)((p0 + k) - (long long)y * d.width);
      const unsigned char g = pY[y * pw0 + x];
      unsigned char* o = out + (p0 + k) * 3;
      o[0] = o[1] = o[2] = g;
    }
    return;
  }
  const unsigned char* pCb = pY + (long long)pw0 * d.bh[0] * 8;
  const int pw1 = d.bw[1] * 8;
  const unsigned char* pCr = pCb + (long long)pw1 * d.bh[1] * 8;
  const int pw2 = d.bw[2] * 8;
  const int fx1 = d.hmax / d.h[1], fy1 = d.vmax / d.v[1], fx2 = d.hmax / d.h[2], fy2 = d.vmax / d.v[2];
  const int cw1 = (d.width * d.h[1] + d.hmax - 1) / d.hmax, ch1 = (d.height * d.v[1] + d.vmax - 1) / d.vmax;
  const int cw2 = (d.width * d.h[2] + d.hmax - 1) / d.hmax, ch2 = (d.height * d.v[2] + d.vmax - 1) / d.vmax;
  for (int k = 0; k < 4 && p0 + k < npix; ++k) {
    const int y = (int)((p0 + k) / d.width), x = (int)((p0 + k) - (long long)y * d.width);
    const int Y = pY[y * pw0 + x];
    const int cb = fancy_up(pCb, pw1, cw1, ch1, fx1, fy1, y, x) - 128;
    const int cr = fancy_up(pCr, pw2, cw2, ch2, fx2, fy2, y, x) - 128;
    unsigned char* o = out + (p0 + k) * 3;
    o[0] = (unsigned char)clamp255(Y + ((91881 * cr + 32768) >> 16));
    o[1] = (unsigned char)clamp255(Y + ((-22554 * cb - 46802 * cr + 32768) >> 16));
    o[2] = (unsigned char)clamp255(Y + ((116130 * cb + 32768) >> 16));
  }
}

}  // namespace dtm
using namespace dtm;

DTM_API int dtm_jpeg_desc_bytes() { return (int)sizeof(JpegDesc); }

// descs: device [n] JpegDesc; max_blocks / max_pixels: the largest nblocks / width*height in the batch
// (grid extents).  coefs int16, planes / rgb uint8 device buffers sized by the caller from the table.
DTM_API int dtm_jpeg_decode_gpu(const void* coefs, const void* descs, int n, int max_blocks, long max_pixels,
                                void* planes, void* rgb, void* stream) {
  if (n <= 0) return 0;
  if (n > 65535 || max_blocks <= 0 || max_pixels <= 0) return -1;
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((max_blocks + 31) / 32, n), dim3(256), 0, (hipStream_t)stream,
                     (const short*)coefs, (const JpegDesc*)descs, (unsigned char*)planes);
  const long gx = (max_pixels + 1023) / 1024;
  if (gx > 0x7fffffff) return -1;
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)gx, n), dim3(256), 0, (hipStream_t)stream,
                     (const JpegDesc*)descs, (const unsigned char*)planes, (unsigned char*)rgb);
  return 0;
}
