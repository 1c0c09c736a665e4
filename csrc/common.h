// Shared device-side helpers for the gfx950 (CDNA4) kernel library.
// Wave = 64 lanes; MFMA operand/accumulator vector types; bf16 helpers; Philox RNG.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tfd {

constexpr int kWave = 64;

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;   // A/B operand of mfma_f32_16x16x32_bf16
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;     // C/D of mfma_f32_16x16x32_bf16
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ float bf2f(bf16 h) { return (float)h; }
// Round-to-nearest-even f32->bf16 via the hardware cvt (keeps NaN a NaN on gfx950).
__device__ __forceinline__ uint16_t f2bf_bits(float f) {
  bf16 b = (bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return (uint32_t)f2bf_bits(lo) | ((uint32_t)f2bf_bits(hi) << 16);
}

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ---- wave / block reductions (64-wide) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// x[c] += x[c] of the DPP source lane (masked-off lanes add 0), N independent values interleaved
template <int CTRL, int RMASK, int BMASK, int N>
__device__ __forceinline__ void dpp_add(float (&x)[N]) {
#pragma unroll
  for (int c = 0; c < N; ++c)
    x[c] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x[c]), CTRL, RMASK, BMASK, true));
}
// N wave sums at once by DPP (quad swaps, row shifts, row broadcasts: no LDS round trips, unlike
// the shuffle-based wave_sum); the wave's totals land in lane 63
template <int N>
__device__ __forceinline__ void wave_sums_to_lane63(float (&x)[N]) {
  dpp_add<0xB1, 0xF, 0xF>(x);   // quad_perm [1,0,3,2]
  dpp_add<0x4E, 0xF, 0xF>(x);   // quad_perm [2,3,0,1]
  dpp_add<0x114, 0xF, 0xE>(x);  // row_shr:4, banks 1-3
  dpp_add<0x118, 0xF, 0xC>(x);  // row_shr:8, banks 2-3
  dpp_add<0x142, 0xA, 0xF>(x);  // row_bcast:15 into rows 1, 3
  dpp_add<0x143, 0xC, 0xF>(x);  // row_bcast:31 into rows 2, 3
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- Philox4x32-10 counter-based RNG (dropout masks keyed by seed/step/rank/element) ----
struct Philox4 {
  uint32_t v[4];
};
__device__ __forceinline__ Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += W0; k1 += W1;
  }
  Philox4 o; o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}
// uniform in [0,1) with 24 bits
__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

}  // namespace tfd
