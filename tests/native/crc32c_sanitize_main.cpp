// Host-side sanitizer harness: built with -fsanitize=address,undefined by
// tests/test_native_sanitize_cpu.py. Includes the runtime source directly so the static
// software (slice-by-8) and SSE4.2 paths can both be checked, on every length and misalignment.
#include "../../csrc/runtime/crc32c.cpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static uint32_t crc_bitwise(const uint8_t* p, size_t n) {
  uint32_t c = ~0u;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
  }
  return ~c;
}

int main() {
  const char* v = "123456789";
  if (tfd::crc32c_extend(0, v, 9) != 0xE3069283u) { std::puts("check vector failed"); return 1; }
  std::vector<uint8_t> buf(4096 + 16);
  uint32_t s = 12345;
  for (auto& b : buf) { s = s * 1103515245u + 12345u; b = (uint8_t)(s >> 16); }
  int bad = 0;
  for (size_t off = 0; off < 8; ++off)
    for (size_t n = 0; n <= 4096; n += (n < 64 ? 1 : 61)) {
      // exact-size heap copy: any over-read past n is an ASan error
      uint8_t* p = (uint8_t*)std::malloc(n ? n : 1);
      std::memcpy(p, buf.data() + off, n);
      const uint32_t want = crc_bitwise(p, n);
      const uint32_t sw = ~tfd::crc_sw(~0u, p, n);
      const uint32_t api = tfd::crc32c_extend(0, p, n);
      // extend in two pieces == one shot
      const size_t h = n / 3;
      const uint32_t two = tfd::crc32c_extend(tfd::crc32c_extend(0, p, h), p + h, n - h);
      bad += (sw != want) + (api != want) + (two != want);
      std::free(p);
    }
  std::printf("crc32c sanitize harness: %s\n", bad ? "MISMATCH" : "ok");
  return bad ? 1 : 0;
}
