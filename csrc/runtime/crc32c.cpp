// CRC32-C (Castagnoli) with the SSE4.2 crc32 instruction (slice-by-8 software fallback).
// Used by the TF-V2-bundle-compatible checkpoint writer/reader (tensor payload checksums and the
// SSTable block trailers: masked crc32c, /root/reference/mnist_python_m.py:235-253 Supervisor/Saver).
#include <stdint.h>
#include <stddef.h>
#if defined(__x86_64__)
#include <cpuid.h>
#include <nmmintrin.h>
#endif

namespace tfd {

static uint32_t table8[8][256];
static bool table_ready = false;

static void init_table() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
    table8[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) table8[t][i] = (table8[t - 1][i] >> 8) ^ table8[0][table8[t - 1][i] & 0xFF];
  table_ready = true;
}

static uint32_t crc_sw(uint32_t crc, const uint8_t* p, size_t n) {
  if (!table_ready) init_table();
  while (n >= 8) {
    const uint32_t lo = crc ^ (uint32_t)(p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24);
    const uint32_t hi = (uint32_t)(p[4] | p[5] << 8 | p[6] << 16 | (uint32_t)p[7] << 24);
    crc = table8[7][lo & 0xFF] ^ table8[6][(lo >> 8) & 0xFF] ^ table8[5][(lo >> 16) & 0xFF] ^ table8[4][lo >> 24] ^
          table8[3][hi & 0xFF] ^ table8[2][(hi >> 8) & 0xFF] ^ table8[1][(hi >> 16) & 0xFF] ^ table8[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = table8[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return crc;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) static uint32_t crc_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}
static bool have_sse42() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  return (c & bit_SSE4_2) != 0;
}
#endif

// Extend a crc32c value (pass 0 to start).
uint32_t crc32c_extend(uint32_t init, const void* data, size_t n) {
  uint32_t crc = ~init;
#if defined(__x86_64__)
  static const bool hw = have_sse42();
  crc = hw ? crc_hw(crc, (const uint8_t*)data, n) : crc_sw(crc, (const uint8_t*)data, n);
#else
  crc = crc_sw(crc, (const uint8_t*)data, n);
#endif
  return ~crc;
}

}  // namespace tfd
