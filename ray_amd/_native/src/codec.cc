#include "codec.h"

#include <cstring>
#include <stdexcept>

namespace ray_amd {
namespace {

struct Tables {
  uint32_t t[8][256];
  Tables() {
    const uint32_t poly = 0x82f63b78u;  // reflected Castagnoli polynomial
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};

const Tables& tables() {
  static const Tables tb;
  return tb;
}

uint32_t crc_sw(const uint8_t* p, size_t n, uint32_t c) {
  const Tables& tb = tables();
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    v ^= c;
    c = tb.t[7][v & 0xff] ^ tb.t[6][(v >> 8) & 0xff] ^ tb.t[5][(v >> 16) & 0xff] ^
        tb.t[4][(v >> 24) & 0xff] ^ tb.t[3][(v >> 32) & 0xff] ^ tb.t[2][(v >> 40) & 0xff] ^
        tb.t[1][(v >> 48) & 0xff] ^ tb.t[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = tb.t[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return c;
}

__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, size_t n, uint32_t c) {
  uint64_t c64 = c;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c64 = __builtin_ia32_crc32di(c64, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c64;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}

const bool kHaveSse42 = __builtin_cpu_supports("sse4.2");

uint64_t load_u64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);  // little-endian host (x86-64), as the format
  return v;
}

uint32_t load_u32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

}  // namespace

uint32_t crc32c(const uint8_t* data, size_t n, uint32_t crc) {
  const uint32_t c = ~crc;
  return ~(kHaveSse42 ? crc_hw(data, n, c) : crc_sw(data, n, c));
}

std::vector<std::pair<uint64_t, uint64_t>> tfrecord_index(const uint8_t* buf, size_t n,
                                                          bool verify) {
  std::vector<std::pair<uint64_t, uint64_t>> out;
  size_t pos = 0;
  while (pos < n) {
    if (n - pos < 12) throw std::runtime_error("truncated TFRecord header");
    const uint64_t len = load_u64(buf + pos);
    if (verify && crc_mask(crc32c(buf + pos, 8)) != load_u32(buf + pos + 8))
      throw std::runtime_error("TFRecord length CRC mismatch");
    const size_t data = pos + 12;
    if (len > n - data || n - data - len < 4) throw std::runtime_error("truncated TFRecord");
    if (verify && crc_mask(crc32c(buf + data, len)) != load_u32(buf + data + len))
      throw std::runtime_error("TFRecord data CRC mismatch");
    out.emplace_back(data, len);
    pos = data + len + 4;
  }
  return out;
}

void tfrecord_append(std::string* out, const uint8_t* rec, size_t n) {
  uint8_t hdr[12];
  const uint64_t len = n;
  memcpy(hdr, &len, 8);
  const uint32_t lc = crc_mask(crc32c(hdr, 8));
  memcpy(hdr + 8, &lc, 4);
  out->append(reinterpret_cast<const char*>(hdr), 12);
  out->append(reinterpret_cast<const char*>(rec), n);
  const uint32_t dc = crc_mask(crc32c(rec, n));
  out->append(reinterpret_cast<const char*>(&dc), 4);
}

}  // namespace ray_amd
