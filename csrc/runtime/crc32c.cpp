// Table-driven (slicing-by-8) CRC-32C.  Uses the SSE4.2 crc32 instruction when the host has it.
#include "crc32c.h"

#include <cstring>
#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

namespace dtmrt {
namespace {
uint32_t T[8][256];
bool init_tables() {
  const uint32_t poly = 0x82f63b78u;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
    T[0][i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t i = 0; i < 256; ++i) T[t][i] = (T[t - 1][i] >> 8) ^ T[0][T[t - 1][i] & 0xff];
  return true;
}
const bool g_init = init_tables();

#if defined(__x86_64__)
bool have_sse42() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  return (c & bit_SSE4_2) != 0;
}
const bool g_sse42 = have_sse42();

__attribute__((target("sse4.2"))) uint32_t crc_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc ^ 0xffffffffu;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32 ^ 0xffffffffu;
}
#endif

uint32_t crc_sw(uint32_t crc, const uint8_t* p, size_t n) {
  (void)g_init;
  uint32_t c = crc ^ 0xffffffffu;
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = T[7][lo & 0xff] ^ T[6][(lo >> 8) & 0xff] ^ T[5][(lo >> 16) & 0xff] ^ T[4][lo >> 24] ^ T[3][hi & 0xff] ^
        T[2][(hi >> 8) & 0xff] ^ T[1][(hi >> 16) & 0xff] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = T[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return c ^ 0xffffffffu;
}
}  // namespace

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
#if defined(__x86_64__)
  if (g_sse42) return crc_hw(crc, p, n);
#endif
  return crc_sw(crc, p, n);
}
}  // namespace dtmrt

extern "C" __attribute__((visibility("default"))) uint32_t dtm_crc32c(const void* data, size_t n) {
  return dtmrt::crc32c(data, n);
}
extern "C" __attribute__((visibility("default"))) uint32_t dtm_crc32c_masked(const void* data, size_t n) {
  return dtmrt::crc_mask(dtmrt::crc32c(data, n));
}
