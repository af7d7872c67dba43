// Record codecs for Ray Data file formats: CRC32C (Castagnoli) and TFRecord framing.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace ray_amd {

// CRC32C of data[0..n) continuing from `crc` (0 to start). SSE4.2 crc32 instructions
// when the host has them, slice-by-8 tables otherwise.
uint32_t crc32c(const uint8_t* data, size_t n, uint32_t crc = 0);

// TFRecord's masked CRC: rotate right 15, add a constant (tensorflow/core/lib/hash/crc32c.h)
inline uint32_t crc_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}

// (offset, length) of every record payload in a TFRecord byte stream. Throws
// std::runtime_error on truncation or (verify) a length / data CRC mismatch.
std::vector<std::pair<uint64_t, uint64_t>> tfrecord_index(const uint8_t* buf, size_t n,
                                                          bool verify);

// Appends the framed record (length, masked CRC of length, payload, masked CRC of payload).
void tfrecord_append(std::string* out, const uint8_t* rec, size_t n);

}  // namespace ray_amd
