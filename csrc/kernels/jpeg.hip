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


// ---- entropy (Huffman) decode ----------------------------------------------------------------------------
// One workgroup per image decodes the unstuffed entropy-coded bytes (host: dtm_jpeg_scan, csrc/runtime/jpeg.cpp)
// into the zeroed [comp][bh][bw][64] int16 coefficient layout jpeg_idct_kernel reads - exactly what the host
// decoder (decode_scan) writes.
//  * restart interval > 0: every restart segment is an independent run with a known start (MCU s * RI, block 0,
//    coefficient 0, DC predictors 0): thread t decodes segments t, t + 256, ...
//  * no restart markers (the common case): the bit stream is cut into 256 subsequences of L bits.  Thread t decodes
//    from a start state S_t = (bit, block-in-MCU, coefficient) to the first codeword boundary past its end, giving
//    the exit state E_t, its block count and per-component DC-difference sums.  S_0 is exact; S_t starts as a guess
//    (bit t * L, block 0, coefficient 0) and is replaced by E_{t-1} until nothing changes - a fixed point that is
//    exact by induction (after pass j the first j + 1 starts are), and in practice reached in a few passes because a
//    Huffman decode started at a wrong bit falls back into step with the true one (see the measurements below).  Scans of
//    the counts and DC sums then place every thread's blocks and DC predictors, and a last pass writes them.
// Tables: each of the image's (<= 4) DHT tables becomes a 9..11-bit lookup in LDS (code length + symbol, or for
// short codes the code + magnitude bits -> the value, run and total length in one entry; the host decoder's
// fast_ac), longer codes walk the canonical maxcode table.
// Measured (tools/jpeg_gpu_bench.py, ImageNet-like 300-500 px q90 files): the fixed point takes 3-5 passes at
// 256 threads per image (a wrong-start decode regains bit sync within ~15-80 bits but the block-in-MCU / coefficient
// state only after ~800 bits median, ~6000 worst), ~430k images/s on the whole GPU with 3 images per CU; 256 images
// decoded under the ResNet-50 step cost it ~1 ms (6 %), which is why the full host decode stays the default
// wherever the host CPUs keep up (data/capacity.py).

// mirror of csrc/runtime/jpeg.cpp JpegScan
struct JpegScan {
  int nbytes, nseg, restart;
  int ncomp, bpm, mcux, nmcu, nslot;
  int bcomp[12], bdy[12], bdx[12];
  int h[3], v[3], bw[3], coef_off[3];
  int dc_slot[3], ac_slot[3];
  int slot_dc[4];
  unsigned char counts[4][16];
  unsigned char vals[4][256];
};

// one image of the batch (mirrored in data/jpeg.py HUFF_DESC_DT)
struct HuffDesc {
  long long stream_off;  // byte offset (4-aligned) of the image's unstuffed bytes in the batch stream buffer
  long long coef_base;   // int16 offset of its coefficients (JpegDesc.coef_base)
  int coef_count;        // int16 coefficients of the image (zeroed here first)
  int seg_off;           // its first restart segment in the batch segment table
  int min_bits;          // floor of the subsequence length L (0: 1024)
  int pad;
  JpegScan s;
};

// lookup entry, one per 11-bit prefix (0: a code longer than 11 bits - huff_slow_entry builds the same form):
//   bits 0-4   code length, or code + magnitude bits of a value entry
//   bit 5      value entry: bits 16-31 hold the signed coefficient (code + magnitude fit the 11 bits)
//   bit 6      the symbol places a coefficient (a DC difference, or an AC value of size > 0)
//   bit 7      invalid (no such code / DC category > 15): 1 bit is skipped, an AC block ends
//   bits 8-14  coefficient-index advance: run + 1 for a placed value (DC: 1), 16 for ZRL, 64 for EOB
//   bits 16-19 magnitude bit count of a symbol (non-value) entry
// so DC and AC symbols take one branch-light path.
constexpr unsigned HE_VAL = 32u, HE_PUT = 64u, HE_BAD = 128u;
// A subsequence pass reads its bits from LDS, staged in phases of HPW words per thread: the loads of phase j + 1
// are issued as phase j starts and written to LDS after it, so no refill waits on memory (a per-thread refill from
// global memory stalls the whole wave on the latest load of whichever lane refilled last).
constexpr int HPW = 16;

template <int NT, int LK>
struct HuffLds {
  static constexpr int kLook = LK;
  unsigned lut[4][1 << LK];
  int maxcode[4][18];
  int valoff[4][17];
  unsigned char vals[4][256];
  unsigned char zz[64];
  int bcomp[12], bdy[12], bdx[12], dcs[3], acs[3];
  int bctx[12];  // component | DC slot << 4 | AC slot << 8 of the b-th block of an MCU
  unsigned win[HPW + 4][NT];  // each thread's stream words of the current phase (+ a 4-word tail), thread-minor:
                              // lanes at similar offsets read distinct banks
  int ep[NT], eb[NT], ek[NT], cnt[NT], ds[3][NT];
  int flag[3], err, passes;
};

__constant__ unsigned char c_zigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                           12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                           35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                           58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

__device__ __forceinline__ int hextend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

// entry for symbol `sym` of code length len (dc: a DC table); bits: the 11-bit prefix (value entries read the
// magnitude bits that follow the code in it), or -1 (longer codes: no value entry)
template <int LK>
__device__ __forceinline__ unsigned huff_entry(int len, int sym, bool dc, int bits) {
  if (dc && sym > 15) return 1u | HE_BAD;  // (advance 0: the DC is retried one bit later)
  const int run = dc ? 0 : sym >> 4, size = dc ? sym : sym & 15;
  if (!dc && !size) return (unsigned)len | ((run == 15 ? 16u : 64u) << 8);  // ZRL / EOB
  const unsigned adv = (unsigned)(run + 1) << 8;
  if (bits >= 0 && len + size <= LK) {
    const int v = size ? hextend((bits >> (LK - len - size)) & ((1 << size) - 1), size) : 0;
    return (unsigned)(len + size) | HE_VAL | HE_PUT | adv | ((unsigned)v << 16);
  }
  return (unsigned)len | HE_PUT | adv | ((unsigned)size << 16);
}

// a code longer than LK bits (canonical maxcode walk over the next 16 bits)
template <int NT, int LK>
__device__ __forceinline__ unsigned huff_slow_entry(const HuffLds<NT, LK>& L, int slot, unsigned code16, bool dc) {
  constexpr int NL = 16 - LK;
  int m[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) m[i] = L.maxcode[slot][LK + 1 + i];
  int l = 0, c = 0;
#pragma unroll
  for (int i = NL - 1; i >= 0; --i) {  // the shortest matching length wins
    const int ci = (int)(code16 >> (16 - (LK + 1 + i)));
    if (ci <= m[i]) {
      l = LK + 1 + i;
      c = ci;
    }
  }
  if (!l) return 1u | HE_BAD | (dc ? 0u : 64u << 8);
  return huff_entry<LK>(l, L.vals[slot][(c + L.valoff[slot][l]) & 255], dc, -1);
}

// MSB-first bit reader over big-endian 32-bit words in global memory (restart segments: arbitrary starts and
// lengths); one word is always in flight
struct GReader {
  const unsigned* w;
  unsigned long long buf;
  int nb, wi, p;
  unsigned nxt;
  __device__ __forceinline__ void init(const unsigned* words, int pos) {
    w = words;
    wi = pos >> 5;
    const unsigned long long hi = __builtin_bswap32(w[wi]), lo = __builtin_bswap32(w[wi + 1]);
    buf = ((hi << 32) | lo) << (pos & 31);
    nb = 64 - (pos & 31);
    wi += 2;
    nxt = w[wi];  // (raw: swapped when used, so nothing waits for the load before the next refill)
    p = pos;
  }
  __device__ __forceinline__ void fill() {
    if (nb < 32) {
      buf |= (unsigned long long)__builtin_bswap32(nxt) << (32 - nb);
      nb += 32;
      nxt = w[++wi];
    }
  }
  __device__ __forceinline__ unsigned peek(int n) const { return (unsigned)(buf >> (64 - n)); }
  __device__ __forceinline__ void skip(int n) { buf <<= n; nb -= n; p += n; }
};

// the same over this thread's LDS phase window: win[i * stride] holds absolute word base + i
template <int NT>
struct LReader {
  const unsigned* win;
  int base;
  unsigned long long buf;
  int nb, wi, p;
  __device__ __forceinline__ unsigned word(int i) const { return __builtin_bswap32(win[(i - base) * NT]); }
  __device__ __forceinline__ void init(int pos) {
    wi = pos >> 5;
    buf = (((unsigned long long)word(wi) << 32) | word(wi + 1)) << (pos & 31);
    nb = 64 - (pos & 31);
    wi += 2;
    p = pos;
  }
  __device__ __forceinline__ void fill() {
    if (nb < 32) {
      buf |= (unsigned long long)word(wi) << (32 - nb);
      nb += 32;
      ++wi;
    }
  }
  __device__ __forceinline__ unsigned peek(int n) const { return (unsigned)(buf >> (64 - n)); }
  __device__ __forceinline__ void skip(int n) { buf <<= n; nb -= n; p += n; }
};

struct HuffState {
  int p, b, k;
};

template <class LDS>
__device__ __forceinline__ short* block_at(const LDS& L, const JpegScan& s, short* img, int g) {
  const int mcu = g / s.bpm, bb = g - mcu * s.bpm, my = mcu / s.mcux, mx = mcu - my * s.mcux, c = L.bcomp[bb];
  return img + s.coef_off[c] + ((long long)(my * s.v[c] + L.bdy[bb]) * s.bw[c] + mx * s.h[c] + L.bdx[bb]) * 64;
}

// decoder state that survives between phases
struct HuffDec {
  int b, k, ctx, g, nblk, err;
  int a0, a1, a2;  // count passes: DC-difference sums per component; output pass: the DC predictors (no array:
                   // a lane-indexed one goes to scratch)
  short* blk;
};

template <class LDS>
__device__ __forceinline__ void dec_start(HuffDec& d, const LDS& L, const JpegScan& s, short* img, HuffState st,
                                          int g, const int* acc, bool out, int total) {
  d.b = st.b;
  d.k = st.k;
  d.ctx = L.bctx[st.b];
  d.g = g;
  d.nblk = 0;
  d.err = 0;
  d.a0 = acc[0];
  d.a1 = acc[1];
  d.a2 = acc[2];
  d.blk = (out && st.k > 0 && g < total) ? block_at(L, s, img, g) : nullptr;
}

// Decode until the first codeword boundary at or past `stop` (or, with gstop >= 0, until block gstop would start).
// OUT = false: count blocks started (DC symbols) and sum the DC differences per component.  OUT = true: write the
// coefficients of blocks g < total.  A decode error in a block < total sets err (chains started from a wrong
// guess may hit them; only the exact, final pass reports).  Every iteration consumes >= 1 bit.
template <bool OUT, class R, class LDS>
__device__ __forceinline__ void huff_steps(const LDS& L, const JpegScan& s, R& br, HuffDec& d, int stop, int gstop, int total,
                           short* img) {
  int b = d.b, k = d.k, ctx = d.ctx, g = d.g, a0 = d.a0, a1 = d.a1, a2 = d.a2, nblk = d.nblk, err = d.err;
  short* blk = d.blk;
  while (br.p < stop) {
    if (gstop >= 0 && k == 0 && g >= gstop) break;
    br.fill();
    const int c = ctx & 15;
    const int slot = k == 0 ? (ctx >> 4) & 15 : ctx >> 8;
    unsigned e = L.lut[slot][br.peek(LDS::kLook)];
    if (!e) e = huff_slow_entry(L, slot, br.peek(16), k == 0);
    const int size = (e & HE_VAL) ? 0 : (e >> 16) & 15;
    const int used = (e & 31) + size;
    int val = (e & HE_VAL) ? (int)e >> 16 : (size ? hextend((int)(br.peek(used) & ((1u << size) - 1)), size) : 0);
    br.skip(used);
    const int adv = (e >> 8) & 127;
    if ((e & HE_BAD) && (!OUT || g < total)) err = 1;
    if (e & HE_PUT) {
      const int pos = k + adv - 1;
      if (k == 0) {
        const int a = (c == 0 ? a0 : c == 1 ? a1 : a2) + val;
        a0 = c == 0 ? a : a0;
        a1 = c == 1 ? a : a1;
        a2 = c == 2 ? a : a2;
        val = a;
        if (!OUT) ++nblk;
        else if (g < total) blk = block_at(L, s, img, g);
      }
      if (pos > 63) {
        if (!OUT || g < total) err = 1;
        k = 64;
      } else {
        if (OUT && g < total) blk[L.zz[pos]] = (short)val;
        k = pos + 1;
      }
    } else {
      k += adv;
    }
    if (k >= 64) {
      k = 0;
      b = b + 1 == s.bpm ? 0 : b + 1;
      ctx = L.bctx[b];
      if (OUT) ++g;
    }
  }
  d.b = b;
  d.k = k;
  d.ctx = ctx;
  d.g = g;
  d.blk = blk;
  d.a0 = a0;
  d.a1 = a1;
  d.a2 = a2;
  d.nblk = nblk;
  d.err = err;
}

template <int NT>
__device__ __forceinline__ int block_scan_excl(int* a, int v) {  // exclusive prefix sum over the NT threads
  const int t = threadIdx.x;
  a[t] = v;
  __syncthreads();
  for (int o = 1; o < NT; o <<= 1) {
    const int x = t >= o ? a[t - o] : 0;
    __syncthreads();
    a[t] += x;
    __syncthreads();
  }
  const int r = a[t] - v;
  __syncthreads();
  return r;
}

// the HPW + 4 words of phase j of a thread whose subsequence starts at word w0 (zeros past the image's stream)
__device__ __forceinline__ void stage_load(uint4 (&r)[(HPW + 4) / 4], const unsigned* words, int w0, int j, int nw) {
#pragma unroll
  for (int i = 0; i < (HPW + 4) / 4; ++i) {
    const int w = w0 + j * HPW + 4 * i;
    r[i] = w + 4 <= nw ? *(const uint4*)(words + w) : make_uint4(0, 0, 0, 0);
  }
}

// One subsequence pass over the LDS phases: every thread takes part in the staging barriers; `run` threads decode
// from st up to `stop`.  Returns the exit state (for OUT = false, with the counts in d).
template <bool OUT, int NT, int LK>
__device__ __forceinline__ HuffState huff_pass(HuffLds<NT, LK>& L, const JpegScan& s, const unsigned* words, int nw, int w0,
                               int nphase, bool run, HuffState st, int stop, int g, const int* acc, int total,
                               short* img, HuffDec& d) {
  const int t = threadIdx.x;
  uint4 r[(HPW + 4) / 4];
  if (run) stage_load(r, words, w0, 0, nw);
  dec_start(d, L, s, img, st, g, acc, OUT, total);
  LReader<NT> br;
  br.win = &L.win[0][t];
  br.base = w0;
  for (int j = 0; j < nphase; ++j) {
    if (run) {
#pragma unroll
      for (int i = 0; i < (HPW + 4) / 4; ++i) {
        L.win[4 * i][t] = r[i].x;
        L.win[4 * i + 1][t] = r[i].y;
        L.win[4 * i + 2][t] = r[i].z;
        L.win[4 * i + 3][t] = r[i].w;
      }
    }
    __syncthreads();
    if (run && j + 1 < nphase) stage_load(r, words, w0, j + 1, nw);  // (in flight during this phase)
    if (run) {
      br.base = w0 + j * HPW;
      if (j == 0) br.init(st.p);
      huff_steps<OUT>(L, s, br, d, min(stop, (w0 + (j + 1) * HPW) * 32), -1, total, img);
    }
    __syncthreads();
  }
  return HuffState{br.p, d.b, d.k};
}

template <int NT, int LK>
__global__ __launch_bounds__(NT) void jpeg_huff_kernel(const unsigned char* __restrict__ stream,
                                                       const int* __restrict__ segs, const HuffDesc* __restrict__ descs,
                                                       short* __restrict__ coefs, int* __restrict__ status) {
  __shared__ HuffLds<NT, LK> L;
  const HuffDesc& d = descs[blockIdx.x];
  const JpegScan& s = d.s;
  const int t = threadIdx.x;
  short* img = coefs + d.coef_base;
  {
    uint4* z = (uint4*)img;  // (coef_base and every image's capacity are 8-int16 aligned)
    for (int i = t; i < (d.coef_count + 7) / 8; i += NT) z[i] = make_uint4(0, 0, 0, 0);
  }
  // tables
  if (t < s.nslot) {
    int code = 0, kk = 0;
    for (int len = 1; len <= 16; ++len) {
      const int n = s.counts[t][len - 1];
      L.valoff[t][len] = kk - code;
      code += n;
      kk += n;
      L.maxcode[t][len] = n ? code - 1 : -1;
      code <<= 1;
    }
    L.maxcode[t][17] = 0x7fffffff;
  }
  for (int i = t; i < 4 * 256; i += NT) (&L.vals[0][0])[i] = (&s.vals[0][0])[i];
  if (t < 64) L.zz[t] = c_zigzag[t];
  if (t < 12) {
    L.bcomp[t] = s.bcomp[t];
    L.bdy[t] = s.bdy[t];
    L.bdx[t] = s.bdx[t];
    const int c = s.bcomp[t];
    L.bctx[t] = c | (s.dc_slot[c] << 4) | (s.ac_slot[c] << 8);
  }
  if (t == 0) {
    L.err = 0;
    L.flag[0] = L.flag[1] = L.flag[2] = 0;
  }
  __syncthreads();
  for (int i = t; i < s.nslot << LK; i += NT) {
    const int slot = i >> LK, f = i & ((1 << LK) - 1);
    unsigned e = 0;
    for (int len = 1; len <= LK; ++len) {
      const int code = f >> (LK - len);
      if (code <= L.maxcode[slot][len]) {
        e = huff_entry<LK>(len, L.vals[slot][(code + L.valoff[slot][len]) & 255], s.slot_dc[slot] != 0, f);
        break;
      }
    }
    L.lut[slot][f] = e;
  }
  __threadfence_block();
  __syncthreads();

  const unsigned* words = (const unsigned*)(stream + d.stream_off);
  const int nbits = s.nbytes * 8, total = s.nmcu * s.bpm, nw = (s.nbytes + 32) / 4;
  int err = 0;
  if (s.restart > 0) {
    // independent restart segments, read straight from global memory
    const int per = s.restart * s.bpm;
    for (int sg = t; sg < s.nseg; sg += NT) {
      GReader br;
      br.init(words, segs[d.seg_off + sg] * 8);
      HuffDec dd;
      const int zero[3] = {0, 0, 0};
      dec_start(dd, L, s, img, HuffState{br.p, 0, 0}, sg * per, zero, true, total);
      const int gstop = min(sg * per + per, total);
      huff_steps<true>(L, s, br, dd, nbits + 64, gstop, total, img);
      if (dd.err || dd.g < gstop) err = 1;  // (g < gstop: ran out of data)
    }
    if (t == 0) L.passes = 0;
  } else {
    // subsequences of Lb bits (a multiple of 128: 16-byte aligned phase loads)
    int Lb = d.min_bits > 0 ? d.min_bits : 1024;
    Lb = max(Lb, (nbits + NT - 1) / NT);
    Lb = (Lb + 127) & ~127;
    const int nact = (nbits + Lb - 1) / Lb;
    const int stop = min((t + 1) * Lb, nbits), w0 = t * Lb / 32;
    const int nphase = (Lb + HPW * 32 - 1) / (HPW * 32);
    HuffState st{t * Lb, 0, 0};
    const int zero[3] = {0, 0, 0};
    bool dirty = t < nact;
    int pass = 0;
    for (; pass <= NT; ++pass) {
      HuffDec dd;
      const HuffState e = huff_pass<false>(L, s, words, nw, w0, nphase, dirty, st, stop, 0, zero, total, img, dd);
      if (dirty) {
        L.ep[t] = e.p;
        L.eb[t] = e.b;
        L.ek[t] = e.k;
        L.cnt[t] = dd.nblk;
        L.ds[0][t] = dd.a0;
        L.ds[1][t] = dd.a1;
        L.ds[2][t] = dd.a2;
      }
      if (t == 0) L.flag[(pass + 1) % 3] = 0;  // (3 flags: a slow thread may still read the previous pass's)
      __syncthreads();
      dirty = false;
      if (t >= 1 && t < nact && (L.ep[t - 1] != st.p || L.eb[t - 1] != st.b || L.ek[t - 1] != st.k)) {
        st = HuffState{L.ep[t - 1], L.eb[t - 1], L.ek[t - 1]};
        dirty = true;
        L.flag[pass % 3] = 1;
      }
      __syncthreads();
      if (!L.flag[pass % 3]) break;
    }
    const bool act = t < nact;
    const int nb = act ? L.cnt[t] : 0;
    const int d0 = act ? L.ds[0][t] : 0, d1 = act ? L.ds[1][t] : 0, d2 = act ? L.ds[2][t] : 0;
    __syncthreads();
    const int G = block_scan_excl<NT>(L.cnt, nb);
    int pred[3];
    pred[0] = block_scan_excl<NT>(L.ds[0], d0);
    pred[1] = block_scan_excl<NT>(L.ds[1], d1);
    pred[2] = block_scan_excl<NT>(L.ds[2], d2);
    if (t == NT - 1 && G + nb < total) L.err = 1;  // the stream ended before the last block
    HuffDec dd;
    huff_pass<true>(L, s, words, nw, w0, nphase, act, st, stop, st.k > 0 ? G - 1 : G, pred, total, img, dd);
    if (act && dd.err) err = 1;
    if (t == 0) L.passes = pass + 1;
  }
  if (err) L.err = 1;
  __syncthreads();
  if (t == 0) status[blockIdx.x] = L.err ? -1 : L.passes;
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

DTM_API int dtm_jpeg_huff_desc_bytes() { return (int)sizeof(HuffDesc); }

// Entropy-decode a batch: stream = the images' unstuffed bytes (each 4-aligned, 32 zero bytes after), segs = the
// restart segment table, descs = device [n] HuffDesc.  coefs receives every image's zero-filled coefficients;
// status[i] = passes of the subsequence fixed point (0: restart segments), -1: the image's data is corrupt.
// threads per image (64 / 128 / 256) and lookup bits (9 / 10 / 11) of the entropy decoder.  256 x 10 measured
// fastest on ImageNet-like files, alone and co-running with the ResNet-50 step (profiles/r6/r6_s23_jpeg_bench*.log,
// r6_s24_decode_overlap.log): fewer threads per image sync in fewer passes but leave the CU latency-bound; an
// 11-bit lookup costs LDS occupancy.
static int g_huff_nt = getenv("DTM_JPEG_NT") ? atoi(getenv("DTM_JPEG_NT")) : 256;
static int g_huff_lk = getenv("DTM_JPEG_LOOK") ? atoi(getenv("DTM_JPEG_LOOK")) : 10;
DTM_API void dtm_jpeg_set_huff(int nt, int lk) {
  g_huff_nt = nt;
  g_huff_lk = lk;
}

DTM_API int dtm_jpeg_huff_gpu(const void* stream, const void* segs, const void* descs, int n, void* coefs,
                              void* status, void* st) {
  if (n <= 0) return 0;
  const int nt = g_huff_nt, lk = g_huff_lk;
#define DTM_HUFF(NT_, LK_)                                                                                         \
  if (nt == NT_ && lk == LK_) {                                                                                    \
    hipLaunchKernelGGL((jpeg_huff_kernel<NT_, LK_>), dim3(n), dim3(NT_), 0, (hipStream_t)st,                        \
                       (const unsigned char*)stream, (const int*)segs, (const HuffDesc*)descs, (short*)coefs,      \
                       (int*)status);                                                                              \
    return 0;                                                                                                      \
  }
  DTM_HUFF(256, 11) DTM_HUFF(256, 10) DTM_HUFF(256, 9) DTM_HUFF(128, 11) DTM_HUFF(128, 10) DTM_HUFF(128, 9)
  DTM_HUFF(64, 11) DTM_HUFF(64, 10) DTM_HUFF(64, 9)
#undef DTM_HUFF
  return -2;
}
