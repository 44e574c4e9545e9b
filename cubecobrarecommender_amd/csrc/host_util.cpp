// Host utilities exported through the C ABI (no device code): CRC32C for the TF tensor-bundle
// checkpoint layout of ml_files/ (BundleEntryProto.crc32c and the index table's block trailers).
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "ccrec.h"

namespace {
uint32_t g_table[256];
bool g_init = false;

void init_table() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    g_table[i] = c;
  }
  g_init = true;
}

__attribute__((target("sse4.2"))) uint32_t crc_hw(uint32_t crc, const unsigned char *p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}

uint32_t crc_sw(uint32_t crc, const unsigned char *p, size_t n) {
  if (!g_init) init_table();
  while (n--) crc = g_table[(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return crc;
}
}  // namespace

// Extends a CRC32C (Castagnoli) over [data, data+n); start with crc = 0.
extern "C" uint32_t cc_crc32c(uint32_t crc, const void *data, size_t n) {
  const unsigned char *p = static_cast<const unsigned char *>(data);
  uint32_t c = ~crc;
  c = __builtin_cpu_supports("sse4.2") ? crc_hw(c, p, n) : crc_sw(c, p, n);
  return ~c;
}
