// CRC-32C (Castagnoli) with TensorFlow/LevelDB masking (used by TensorBundle .index blocks,
// BundleEntryProto checksums and TFRecord framing).
#pragma once
#include <cstddef>
#include <cstdint>

namespace dtmrt {
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
inline uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }
inline uint32_t crc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
inline uint32_t crc_unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return ((rot >> 17) | (rot << 15));
}
}  // namespace dtmrt
