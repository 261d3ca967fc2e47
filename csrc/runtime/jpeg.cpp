// Baseline JPEG entropy decoder for the GPU ImageNet pipeline.
//
// The reference decodes every JPEG on the host (tf.image.decode_jpeg, inception/image_processing.py:
// 339-407).  Here the decoder processes do only the serial, branchy part - marker parsing and Huffman
// decoding into quantized DCT coefficients - and the data-parallel rest (dequantization, the 8x8
// inverse DCT, chroma upsampling, YCbCr -> RGB) runs on the GPU (csrc/kernels/jpeg.hip), which turns a
// ~2 ms/image host decode into a ~0.4 ms/image one.  The GPU stage reproduces libjpeg(-turbo)'s default
// decompression bit for bit: the accurate integer IDCT (jidctint "islow"), "fancy" triangular chroma
// upsampling (h2v1 / h2v2) with edge replication, and the fixed-point YCbCr -> RGB tables.  The same math
// is here on the CPU (dtm_jpeg_pixels) as the oracle of that kernel and as the host fallback.
//
// Scope: 8-bit baseline / extended-sequential Huffman JPEGs with one interleaved scan (the encoder default:
// every ImageNet / PIL / libjpeg image of that kind), 1 or 3 components, sampling factors 1 or 2 with
// luma at the maximum.  Anything else (progressive, arithmetic, 12-bit, multi-scan, CMYK, exotic
// sampling) returns a negative code and the caller decodes that image with PIL.
#include <cstdint>
#include <cstring>

#define API extern "C" __attribute__((visibility("default")))

namespace {

// natural-order index of the k-th coefficient in zigzag order
const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

constexpr int LOOK = 11;  // bits resolved by one table lookup

struct Huff {
  bool defined = false;
  // fast table: (code length << 8) | symbol for every LOOK-bit prefix; 0 = longer code
  uint16_t fast[1 << LOOK];
  // AC fast path (code + magnitude bits within LOOK): (value << 8) | (run << 4) | total bits; 0 = slow path
  int32_t fast_ac[1 << LOOK];
  int32_t maxcode[18];  // largest code of each length (-1: none), maxcode[17] sentinel
  int32_t valoff[17];   // symbol index offset per length
  uint8_t vals[256];
};

bool build_huff(Huff& h, const uint8_t* counts, const uint8_t* symbols, int nsym) {
  if (nsym > 256) return false;
  memcpy(h.vals, symbols, nsym);
  memset(h.fast, 0, sizeof(h.fast));
  int code = 0, k = 0;
  for (int len = 1; len <= 16; ++len) {
    const int n = counts[len - 1];
    h.valoff[len] = k - code;
    if (n) {
      for (int i = 0; i < n; ++i, ++k, ++code) {
        if (len <= LOOK) {
          const int shift = LOOK - len;
          for (int f = code << shift; f < (code + 1) << shift; ++f) h.fast[f] = (uint16_t)((len << 8) | h.vals[k]);
        }
      }
      h.maxcode[len] = code - 1;
    } else {
      h.maxcode[len] = -1;
    }
    if (code > (1 << len)) return false;  // over-subscribed table
    code <<= 1;
  }
  h.maxcode[17] = 0x7fffffff;
  // combined AC entries: symbol (run, size) whose code length + size fit in LOOK bits -> the value too
  for (int f = 0; f < (1 << LOOK); ++f) {
    h.fast_ac[f] = 0;
    const uint16_t e = h.fast[f];
    if (!e) continue;
    const int len = e >> 8, rs = e & 0xFF, run = rs >> 4, size = rs & 15;
    if (size && len + size <= LOOK) {
      const int bits = (f >> (LOOK - len - size)) & ((1 << size) - 1);
      const int v = bits < (1 << (size - 1)) ? bits - (1 << size) + 1 : bits;
      h.fast_ac[f] = (v * 256) | (run << 4) | (len + size);
    }
  }
  h.defined = true;
  return true;
}

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

// a DHT table as transmitted (code-length counts + symbols): what the GPU entropy decoder builds its tables from
struct RawHuff {
  bool defined = false;
  uint8_t counts[16];
  uint8_t vals[256];
};

// canonical-code sanity of a DHT table (build_huff's over-subscription check without building anything)
bool check_huff(const uint8_t* counts, int nsym) {
  if (nsym > 256) return false;
  int code = 0;
  for (int len = 1; len <= 16; ++len) {
    code += counts[len - 1];
    if (code > (1 << len)) return false;
    code <<= 1;
  }
  return true;
}

struct Comp {
  int id, h, v, tq, td, ta;
};

}  // namespace

// Header + layout of one image, filled by dtm_jpeg_decode (mirrored in data/jpeg.py)
struct JpegInfo {
  int32_t width, height, ncomp;
  int32_t hmax, vmax, mcux, mcuy;     // max sampling factors, MCUs per row / column
  int32_t h[3], v[3];                 // per component sampling factors
  int32_t bw[3], bh[3];               // blocks per row / column of each component (MCU-padded)
  int32_t coef_off[3];                // int16 offset of each component's [bh][bw][64] coefficients
  int32_t coef_count;                 // total int16 coefficients
  uint16_t qt[3][64];                 // quantization table of each component, natural order
};

// The entropy-coded segment of one interleaved scan -> coefficient blocks.  The bit buffer lives in
// locals (registers) for the whole scan; refills are inlined, 4 bytes at a time when no 0xFF is near.
__attribute__((noinline)) static int decode_scan(const uint8_t* p, const uint8_t* end, const JpegInfo* info,
                                                 const Comp* comp, int ncomp, const Huff* dc, const Huff* ac,
                                                 int restart_interval, int16_t* coefs) {
  uint64_t buf = 0;
  int nbits = 0;
  bool marker = false;
  auto refill = [&]() __attribute__((always_inline)) {
    while (nbits <= 32 && !marker && p + 4 <= end) {
      uint32_t w;
      memcpy(&w, p, 4);
      if ((((~w) - 0x01010101u) & w & 0x80808080u) != 0) break;  // some byte is 0xFF: byte path
      buf |= (uint64_t)__builtin_bswap32(w) << (32 - nbits);
      nbits += 32;
      p += 4;
    }
    while (nbits <= 56) {
      uint32_t byte = 0;
      if (!marker && p < end) {
        byte = *p++;
        if (byte == 0xFF) {
          uint32_t nxt = p < end ? *p : 0;
          while (nxt == 0xFF && p + 1 < end) nxt = *++p;
          if (nxt == 0) {
            ++p;
          } else {
            marker = true;  // p stays on the marker's 0xFF; zeros are fed in from here
            --p;
            byte = 0;
          }
        }
      }
      buf |= (uint64_t)byte << (56 - nbits);
      nbits += 8;
    }
  };
  // one Huffman symbol (>= 16 bits must be buffered)
  auto sym = [&](const Huff& h) __attribute__((always_inline)) -> int {
    const uint16_t f = h.fast[buf >> (64 - LOOK)];
    if (f) {
      buf <<= (f >> 8);
      nbits -= f >> 8;
      return f & 0xFF;
    }
    const uint32_t code = (uint32_t)(buf >> 48);
    for (int len = LOOK + 1; len <= 16; ++len) {
      const int32_t c = (int32_t)(code >> (16 - len));
      if (c <= h.maxcode[len]) {
        buf <<= len;
        nbits -= len;
        return h.vals[c + h.valoff[len]];
      }
    }
    return -1;
  };
  int pred[3] = {0, 0, 0};
  const long nmcu = (long)info->mcux * info->mcuy;
  int todo = restart_interval;
  for (long m = 0; m < nmcu; ++m) {
    if (restart_interval) {
      if (todo == 0) {  // RSTn: byte-align, skip the marker, reset the DC predictors
        buf = 0;
        nbits = 0;
        while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
        if (p + 1 >= end) return -1;
        p += 2;
        marker = false;
        pred[0] = pred[1] = pred[2] = 0;
        todo = restart_interval;
      }
      --todo;
    }
    const int my = (int)(m / info->mcux), mx = (int)(m % info->mcux);
    for (int c = 0; c < ncomp; ++c) {
      const Huff& hd = dc[comp[c].td];
      const Huff& ha = ac[comp[c].ta];
      const int cv = info->v[c], ch = info->h[c];
      for (int by = 0; by < cv; ++by)
        for (int bx = 0; bx < ch; ++bx) {
          const long brow = (long)my * cv + by, bcol = (long)mx * ch + bx;
          int16_t* blk = coefs + info->coef_off[c] + (brow * info->bw[c] + bcol) * 64;
          memset(blk, 0, 128);
          if (nbits < 32) refill();
          const int t = sym(hd);
          if (t < 0 || t > 15) return -1;
          int diff = 0;
          if (t) {
            const int v = (int)(buf >> (64 - t));
            buf <<= t;
            nbits -= t;
            diff = extend(v, t);
          }
          pred[c] += diff;
          blk[0] = (int16_t)pred[c];
          for (int k = 1; k < 64;) {
            if (nbits < 32) refill();
            const int32_t fa = ha.fast_ac[buf >> (64 - LOOK)];
            if (fa) {
              k += (fa >> 4) & 15;
              if (k > 63) return -1;
              buf <<= (fa & 15);
              nbits -= fa & 15;
              blk[kZigzag[k]] = (int16_t)(fa >> 8);
              ++k;
              continue;
            }
            const int rs = sym(ha);  // (>= 32 bits buffered: code <= 16 + magnitude <= 15 bits)
            if (rs < 0) return -1;
            const int r = rs >> 4, sz = rs & 15;
            if (sz) {
              k += r;
              if (k > 63) return -1;
              const int v = (int)(buf >> (64 - sz));
              buf <<= sz;
              nbits -= sz;
              blk[kZigzag[k]] = (int16_t)extend(v, sz);
              ++k;
            } else {
              if (r != 15) break;
              k += 16;
            }
          }
        }
    }
  }
  return 0;
}

namespace {
// Everything the marker parser hands to an entropy decoder: the components and their table selectors, the
// restart interval, the entropy-coded segment [scan, end) and the tables - built for the host decoder (dc/ac,
// when asked for) and raw (for the GPU one).
struct Parsed {
  Comp comp[3];
  int ncomp = 0, restart = 0;
  const uint8_t* scan = nullptr;
  const uint8_t* end = nullptr;
  RawHuff rdc[4], rac[4];
};

// Marker parse up to the (single, interleaved) scan: fills info's layout and ps.  Returns 0, -1 corrupt,
// -2 unsupported.  dc / ac: host decode tables to build (nullptr: only the raw tables are kept).
int parse_jpeg(const uint8_t* data, long n, JpegInfo* info, Parsed& ps, Huff* dc, Huff* ac) {
  memset(info, 0, sizeof(*info));
  if (n < 4 || data[0] != 0xFF || data[1] != 0xD8) return -1;
  const uint8_t* p = data + 2;
  const uint8_t* end = data + n;
  uint16_t qtab[4][64];
  bool qdef[4] = {false, false, false, false};
  if (dc)
    for (int i = 0; i < 4; ++i) dc[i].defined = ac[i].defined = false;
  for (int i = 0; i < 4; ++i) ps.rdc[i].defined = ps.rac[i].defined = false;
  ps.ncomp = ps.restart = 0;
  ps.scan = ps.end = nullptr;
  Comp* comp = ps.comp;
  int& ncomp = ps.ncomp;
  int& restart_interval = ps.restart;
  bool have_frame = false;
  while (p + 4 <= end) {
    if (p[0] != 0xFF) return -1;
    const int marker = p[1];
    if (marker == 0xFF) {  // fill byte
      ++p;
      continue;
    }
    p += 2;
    if (marker == 0xD8 || (marker >= 0xD0 && marker <= 0xD7) || marker == 0x01) continue;
    if (marker == 0xD9) return -1;  // EOI before a scan
    if (p + 2 > end) return -1;
    const int len = (p[0] << 8) | p[1];
    if (len < 2 || p + len > end) return -1;
    const uint8_t* seg = p + 2;
    const uint8_t* segend = p + len;
    p += len;
    switch (marker) {
      case 0xDB:  // DQT
        while (seg < segend) {
          const int pq = seg[0] >> 4, tq = seg[0] & 15;
          ++seg;
          if (tq > 3) return -1;
          for (int k = 0; k < 64; ++k) {
            if (pq) {
              if (seg + 2 > segend) return -1;
              qtab[tq][kZigzag[k]] = (uint16_t)((seg[0] << 8) | seg[1]);
              seg += 2;
            } else {
              if (seg >= segend) return -1;
              qtab[tq][kZigzag[k]] = seg[0];
              ++seg;
            }
          }
          qdef[tq] = true;
        }
        break;
      case 0xC4:  // DHT
        while (seg < segend) {
          if (seg + 17 > segend) return -1;
          const int tc = seg[0] >> 4, th = seg[0] & 15;
          if (tc > 1 || th > 3) return -1;
          const uint8_t* counts = seg + 1;
          int nsym = 0;
          for (int i = 0; i < 16; ++i) nsym += counts[i];
          if (seg + 17 + nsym > segend) return -1;
          if (dc) {
            if (!build_huff(tc ? ac[th] : dc[th], counts, seg + 17, nsym)) return -1;
          } else if (!check_huff(counts, nsym)) {
            return -1;
          }
          RawHuff& r = tc ? ps.rac[th] : ps.rdc[th];
          memcpy(r.counts, counts, 16);
          memset(r.vals, 0, sizeof(r.vals));
          memcpy(r.vals, seg + 17, nsym);
          r.defined = true;
          seg += 17 + nsym;
        }
        break;
      case 0xDD:  // DRI
        if (len < 4) return -1;
        restart_interval = (seg[0] << 8) | seg[1];
        break;
      case 0xC0:
      case 0xC1: {  // SOF0 baseline / SOF1 extended sequential (Huffman)
        if (len < 8 || seg[0] != 8) return -2;  // 8-bit samples only
        info->height = (seg[1] << 8) | seg[2];
        info->width = (seg[3] << 8) | seg[4];
        ncomp = seg[5];
        if ((ncomp != 1 && ncomp != 3) || len < 8 + 3 * ncomp || info->width <= 0 || info->height <= 0) return -2;
        for (int c = 0; c < ncomp; ++c) {
          comp[c].id = seg[6 + 3 * c];
          comp[c].h = seg[7 + 3 * c] >> 4;
          comp[c].v = seg[7 + 3 * c] & 15;
          comp[c].tq = seg[8 + 3 * c];
          if (comp[c].h < 1 || comp[c].h > 2 || comp[c].v < 1 || comp[c].v > 2 || comp[c].tq > 3) return -2;
        }
        have_frame = true;
        break;
      }
      case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB: case 0xCD:
      case 0xCE: case 0xCF:
        return -2;  // progressive / lossless / hierarchical / arithmetic
      case 0xDA: {  // SOS: decode the (single, interleaved) scan
        if (!have_frame) return -1;
        const int ns = seg[0];
        if (ns != ncomp || len < 6 + 2 * ns) return -2;  // non-interleaved multi-scan files: PIL
        for (int i = 0; i < ns; ++i) {
          const int cid = seg[1 + 2 * i];
          int c = -1;
          for (int j = 0; j < ncomp; ++j)
            if (comp[j].id == cid) c = j;
          if (c != i) return -2;
          comp[c].td = seg[2 + 2 * i] >> 4;
          comp[c].ta = seg[2 + 2 * i] & 15;
          if (comp[c].td > 3 || comp[c].ta > 3 || !ps.rdc[comp[c].td].defined || !ps.rac[comp[c].ta].defined) return -1;
        }
        const int ss = seg[1 + 2 * ns], se = seg[2 + 2 * ns], ahal = seg[3 + 2 * ns];
        if (ss != 0 || se != 63 || ahal != 0) return -2;
        // layout
        int hmax = 1, vmax = 1;
        for (int c = 0; c < ncomp; ++c) {
          hmax = comp[c].h > hmax ? comp[c].h : hmax;
          vmax = comp[c].v > vmax ? comp[c].v : vmax;
          if (!qdef[comp[c].tq]) return -1;
        }
        if (ncomp == 3 && (comp[0].h != hmax || comp[0].v != vmax)) return -2;  // luma must be full resolution
        if (ncomp == 1) hmax = vmax = comp[0].h = comp[0].v = 1;  // single-component scans are not interleaved
        info->ncomp = ncomp;
        info->hmax = hmax;
        info->vmax = vmax;
        info->mcux = (info->width + 8 * hmax - 1) / (8 * hmax);
        info->mcuy = (info->height + 8 * vmax - 1) / (8 * vmax);
        long total = 0;
        for (int c = 0; c < ncomp; ++c) {
          info->h[c] = comp[c].h;
          info->v[c] = comp[c].v;
          info->bw[c] = info->mcux * comp[c].h;
          info->bh[c] = info->mcuy * comp[c].v;
          info->coef_off[c] = (int32_t)total;
          total += (long)info->bw[c] * info->bh[c] * 64;
          memcpy(info->qt[c], qtab[comp[c].tq], sizeof(info->qt[c]));
        }
        if (total > (1l << 30)) return -2;
        info->coef_count = (int32_t)total;
        ps.scan = segend;
        ps.end = end;
        return 0;
      }
      default:  // APPn, COM, DNL, ...: skip
        break;
    }
  }
  return -1;
}
}  // namespace

// Parse + Huffman-decode `data` into `coefs` (int16, natural order, [comp][bh][bw][64]) of capacity
// `cap` int16.  Returns 0, or: -1 corrupt, -2 unsupported (caller falls back to PIL), -3 capacity too
// small (info is filled: info->coef_count is the need).
API int dtm_jpeg_decode(const uint8_t* data, long n, JpegInfo* info, int16_t* coefs, long cap) {
  static thread_local Huff dc[4], ac[4];
  static thread_local Parsed ps;
  const int rc = parse_jpeg(data, n, info, ps, dc, ac);
  if (rc) return rc;
  if (info->coef_count > cap) return -3;
  return decode_scan(ps.scan, ps.end, info, ps.comp, ps.ncomp, dc, ac, ps.restart, coefs);
}

API int dtm_jpeg_info_bytes() { return (int)sizeof(JpegInfo); }

// ---- host share of the GPU entropy decode (csrc/kernels/jpeg.hip jpeg_huff_kernel) ----------------------
// What the device needs to Huffman-decode one image: the MCU layout, up to 4 distinct tables as transmitted and
// the restart segments of the unstuffed entropy-coded bytes (mirrored in jpeg.hip JpegScan and data/jpeg.py).
struct JpegScan {
  int32_t nbytes;             // unstuffed entropy-coded bytes (0xFF00 -> 0xFF, RSTn removed), 32 zero bytes follow
  int32_t nseg;               // restart segments (restart interval > 0), else 0
  int32_t restart;            // restart interval in MCUs (0: none)
  int32_t ncomp, bpm, mcux, nmcu, nslot;  // blocks per MCU, MCUs per row, MCUs, distinct tables
  int32_t bcomp[12], bdy[12], bdx[12];    // component of the b-th block of an MCU, its block row / column in the MCU
  int32_t h[3], v[3], bw[3], coef_off[3];
  int32_t dc_slot[3], ac_slot[3];         // table slot of each component's DC / AC table
  int32_t slot_dc[4];                     // 1: the slot holds a DC table
  uint8_t counts[4][16];
  uint8_t vals[4][256];
};

// Marker parse + byte unstuffing of `data` for the GPU entropy decoder: the host work per image is a header walk
// and a memchr/memcpy pass over the scan (no bit-level work).  `stream` (capacity cap >= n + 32 bytes) receives the
// unstuffed entropy-coded bytes and 32 zero bytes; `segs` (capacity seg_cap) the byte offset of every restart
// segment in it.  Returns 0, -1 corrupt, -2 unsupported (the caller decodes on the host / with PIL), -3 capacity
// (scan->nseg holds the segment need).
API int dtm_jpeg_scan(const uint8_t* data, long n, JpegInfo* info, JpegScan* scan, uint8_t* stream, long cap,
                      int32_t* segs, long seg_cap) {
  static thread_local Parsed ps;
  memset(scan, 0, sizeof(*scan));
  const int rc = parse_jpeg(data, n, info, ps, nullptr, nullptr);
  if (rc) return rc;
  JpegScan& d = *scan;
  d.ncomp = info->ncomp;
  d.mcux = info->mcux;
  d.nmcu = info->mcux * info->mcuy;
  d.restart = ps.restart;
  int bpm = 0;
  for (int c = 0; c < info->ncomp; ++c) {
    d.h[c] = info->h[c];
    d.v[c] = info->v[c];
    d.bw[c] = info->bw[c];
    d.coef_off[c] = info->coef_off[c];
    for (int by = 0; by < info->v[c]; ++by)
      for (int bx = 0; bx < info->h[c]; ++bx) {
        if (bpm >= 12) return -2;
        d.bcomp[bpm] = c;
        d.bdy[bpm] = by;
        d.bdx[bpm] = bx;
        ++bpm;
      }
  }
  d.bpm = bpm;
  // distinct (class, id) tables -> slots
  int key[4], ns = 0;
  auto slot = [&](int cls, int id) -> int {
    const int k = cls * 4 + id;
    for (int i = 0; i < ns; ++i)
      if (key[i] == k) return i;
    if (ns == 4) return -1;
    const RawHuff& r = cls ? ps.rac[id] : ps.rdc[id];
    key[ns] = k;
    d.slot_dc[ns] = cls ? 0 : 1;
    memcpy(d.counts[ns], r.counts, 16);
    memcpy(d.vals[ns], r.vals, 256);
    return ns++;
  };
  for (int c = 0; c < info->ncomp; ++c) {
    d.dc_slot[c] = slot(0, ps.comp[c].td);
    d.ac_slot[c] = slot(1, ps.comp[c].ta);
    if (d.dc_slot[c] < 0 || d.ac_slot[c] < 0) return -2;
  }
  d.nslot = ns;
  const long need_seg = ps.restart ? (d.nmcu + ps.restart - 1) / ps.restart : 0;
  d.nseg = (int32_t)need_seg;
  if (cap < (ps.end - ps.scan) + 32 || seg_cap < need_seg || (ps.end - ps.scan) >= (1l << 28)) return -3;
  // unstuff: 0xFF 0x00 -> 0xFF, fill bytes dropped, RSTn -> a segment boundary, any other marker ends the scan
  const uint8_t* p = ps.scan;
  const uint8_t* end = ps.end;
  uint8_t* o = stream;
  long nseg = 0;
  if (ps.restart) segs[nseg++] = 0;
  while (p < end) {
    const uint8_t* q = (const uint8_t*)memchr(p, 0xFF, end - p);
    if (!q) {
      memcpy(o, p, end - p);
      o += end - p;
      break;
    }
    memcpy(o, p, q - p);
    o += q - p;
    p = q + 1;
    while (p < end && *p == 0xFF) ++p;
    if (p >= end) break;
    if (*p == 0) {
      *o++ = 0xFF;
      ++p;
      continue;
    }
    if (ps.restart && *p >= 0xD0 && *p <= 0xD7) {
      ++p;
      if (nseg < need_seg) segs[nseg++] = (int32_t)(o - stream);
      continue;
    }
    break;
  }
  if (nseg < need_seg) return -1;  // missing restart markers (the host decoder fails such a file the same way)
  d.nbytes = (int32_t)(o - stream);
  memset(o, 0, 32);
  return 0;
}

API int dtm_jpeg_scan_bytes() { return (int)sizeof(JpegScan); }

// ---- CPU reference of the GPU stage (libjpeg's islow IDCT + fancy upsampling + YCbCr->RGB) ------------
namespace {

constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                  F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;

inline int32_t descale(int32_t x, int n) { return (x + (1 << (n - 1))) >> n; }

// post-IDCT range limit: libjpeg's sample_range_limit + CENTERJSAMPLE table indexed by (x & 1023)
inline uint8_t idct_limit(int32_t x) {
  const int i = x & 1023;
  if (i < 128) return (uint8_t)(i + 128);
  if (i < 512) return 255;
  if (i < 896) return 0;
  return (uint8_t)(i - 896);
}

void idct_islow(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
  int32_t ws[64];
  for (int c = 0; c < 8; ++c) {
    const int16_t* ip = in + c;
    const uint16_t* qp = q + c;
    if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
      const int32_t dc = ((int32_t)ip[0] * qp[0]) * (1 << PASS1_BITS);
      for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
      continue;
    }
    int32_t z2 = ip[16] * qp[16], z3 = ip[48] * qp[48];
    int32_t z1 = (z2 + z3) * F0541;
    int32_t tmp2 = z1 + z3 * (-F1847), tmp3 = z1 + z2 * F0765;
    z2 = ip[0] * qp[0];
    z3 = ip[32] * qp[32];
    int32_t tmp0 = (z2 + z3) * (1 << CONST_BITS), tmp1 = (z2 - z3) * (1 << CONST_BITS);
    const int32_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = ip[56] * qp[56];
    tmp1 = ip[40] * qp[40];
    tmp2 = ip[24] * qp[24];
    tmp3 = ip[8] * qp[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int32_t z4 = tmp1 + tmp3;
    const int32_t z5 = (z3 + z4) * F1175;
    tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    const int n = CONST_BITS - PASS1_BITS;
    ws[0 * 8 + c] = descale(t10 + tmp3, n);
    ws[7 * 8 + c] = descale(t10 - tmp3, n);
    ws[1 * 8 + c] = descale(t11 + tmp2, n);
    ws[6 * 8 + c] = descale(t11 - tmp2, n);
    ws[2 * 8 + c] = descale(t12 + tmp1, n);
    ws[5 * 8 + c] = descale(t12 - tmp1, n);
    ws[3 * 8 + c] = descale(t13 + tmp0, n);
    ws[4 * 8 + c] = descale(t13 - tmp0, n);
  }
  for (int r = 0; r < 8; ++r) {
    const int32_t* w = ws + r * 8;
    uint8_t* o = out + r * stride;
    // (libjpeg-turbo's C islow has no zero-row shortcut in pass 2 by default: the general path is exact)
    int32_t z2 = w[2], z3 = w[6];
    int32_t z1 = (z2 + z3) * F0541;
    int32_t tmp2 = z1 + z3 * (-F1847), tmp3 = z1 + z2 * F0765;
    int32_t tmp0 = (w[0] + w[4]) * (1 << CONST_BITS), tmp1 = (w[0] - w[4]) * (1 << CONST_BITS);
    const int32_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
    int32_t z4 = tmp1 + tmp3;
    const int32_t z5 = (z3 + z4) * F1175;
    tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    const int n = CONST_BITS + PASS1_BITS + 3;
    o[0] = idct_limit(descale(t10 + tmp3, n));
    o[7] = idct_limit(descale(t10 - tmp3, n));
    o[1] = idct_limit(descale(t11 + tmp2, n));
    o[6] = idct_limit(descale(t11 - tmp2, n));
    o[2] = idct_limit(descale(t12 + tmp1, n));
    o[5] = idct_limit(descale(t12 - tmp1, n));
    o[3] = idct_limit(descale(t13 + tmp0, n));
    o[4] = idct_limit(descale(t13 - tmp0, n));
  }
}

inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// chroma sample of full-resolution pixel (y, x) with libjpeg's fancy upsampling of a plane of
// real size cw x ch (pitch pw), factors fx, fy in {1, 2}
inline int fancy(const uint8_t* pl, int pw, int cw, int ch, int fx, int fy, int y, int x) {
  if (fx == 1 && fy == 1) return pl[y * pw + x];
  if (fy == 1) {  // h2v1
    const int i = x >> 1;
    const int c = pl[y * pw + i];
    if (x & 1) {
      if (i == cw - 1) return c;
      return (c * 3 + pl[y * pw + i + 1] + 2) >> 2;
    }
    if (i == 0) return c;
    return (c * 3 + pl[y * pw + i - 1] + 1) >> 2;
  }
  // h2v2 (fx == 2): rows: nearest = y/2, other = y/2 -1 (even y) or +1 (odd y), replicated at the edges
  // (h1v2 is rare: handled as h2v2 with the horizontal pass skipped)
  const int j = y >> 1;
  int jo = (y & 1) ? j + 1 : j - 1;
  if (jo < 0) jo = 0;
  if (jo > ch - 1) jo = ch - 1;
  const uint8_t* r0 = pl + j * pw;
  const uint8_t* r1 = pl + jo * pw;
  if (fx == 1) return (r0[x] * 3 + r1[x] + 1 + (y & 1)) >> 2;  // libjpeg-turbo h1v2: bias 1 / 2
  const int i = x >> 1;
  const int cs = r0[i] * 3 + r1[i];
  if (x & 1) {
    if (i == cw - 1) return (cs * 4 + 7) >> 4;
    const int ns = r0[i + 1] * 3 + r1[i + 1];
    return (cs * 3 + ns + 7) >> 4;
  }
  if (i == 0) return (cs * 4 + 8) >> 4;
  const int ls = r0[i - 1] * 3 + r1[i - 1];
  return (cs * 3 + ls + 8) >> 4;
}

}  // namespace

// Decoded coefficients -> RGB (H x W x 3 uint8), the CPU form of the GPU stage.  `scratch` holds the
// component planes: at least sum_c bw*8 * bh*8 bytes.  Returns 0.
API int dtm_jpeg_pixels(const int16_t* coefs, const JpegInfo* info, uint8_t* scratch, uint8_t* rgb) {
  uint8_t* planes[3];
  int pw[3];
  long off = 0;
  for (int c = 0; c < info->ncomp; ++c) {
    planes[c] = scratch + off;
    pw[c] = info->bw[c] * 8;
    off += (long)pw[c] * info->bh[c] * 8;
    for (int by = 0; by < info->bh[c]; ++by)
      for (int bx = 0; bx < info->bw[c]; ++bx)
        idct_islow(coefs + info->coef_off[c] + ((long)by * info->bw[c] + bx) * 64, info->qt[c],
                   planes[c] + (long)by * 8 * pw[c] + bx * 8, pw[c]);
  }
  const int W = info->width, H = info->height;
  if (info->ncomp == 1) {
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x) {
        const uint8_t g = planes[0][y * pw[0] + x];
        uint8_t* o = rgb + ((long)y * W + x) * 3;
        o[0] = o[1] = o[2] = g;
      }
    return 0;
  }
  int fx[3], fy[3], cw[3], chh[3];
  for (int c = 1; c < 3; ++c) {
    fx[c] = info->hmax / info->h[c];
    fy[c] = info->vmax / info->v[c];
    cw[c] = (W * info->h[c] + info->hmax - 1) / info->hmax;  // downsampled_width (jdinput.c)
    chh[c] = (H * info->v[c] + info->vmax - 1) / info->vmax;
  }
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const int Y = planes[0][y * pw[0] + x];
      const int cb = fancy(planes[1], pw[1], cw[1], chh[1], fx[1], fy[1], y, x) - 128;
      const int cr = fancy(planes[2], pw[2], cw[2], chh[2], fx[2], fy[2], y, x) - 128;
      // jdcolor.c ycc_rgb_convert, SCALEBITS 16
      const int r = Y + ((91881 * cr + 32768) >> 16);
      const int g = Y + ((-22554 * cb - 46802 * cr + 32768) >> 16);
      const int b = Y + ((116130 * cb + 32768) >> 16);
      uint8_t* o = rgb + ((long)y * W + x) * 3;
      o[0] = clamp255(r);
      o[1] = clamp255(g);
      o[2] = clamp255(b);
    }
  return 0;
}
