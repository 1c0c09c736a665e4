// Forward batch-norm affine constants of one channel: out = relu?(y * sc + sh) with sc = invstd * gamma,
// sh = beta - mean * sc (one explicit fma). Every kernel that forms a BN output or re-derives its relu
// mask -- norm.hip's apply and backward passes, the conv loaders that apply their input's BN while
// staging it (csrc/kernels/conv_nhwc.hip BnRelu), the dgrad BN-statistics epilogue -- takes these exact
// values and the same fmaf(y, sc, sh), so a mask recomputed from y matches the relu the consumer
// applied bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>


namespace tfd {

__device__ __forceinline__ void bn_affine(float mean, float invstd, float gamma, float beta, float& sc, float& sh) {
  sc = invstd * gamma;
  sh = fmaf(-mean, sc, beta);
}

// relu(y * sc + sh) of two bf16 values packed in a dword (low half = the lower channel): two fmas
// (one v_pk_fma_f32 where the build allows packed fp32; this library's build does not, see
// docs/DESIGN.md §6), one v_cvt_pk_bf16_f32 (RNE), and the relu as v_pk_max_i16 against 0 on the
// rounded bf16 bits (a negative bf16 is a negative int16; -0 -> +0) -- equal to rounding fmaxf(z, 0)
// for every non-NaN z. bn_apply_kernel and the folded conv loaders both use it, so the two forms
// of a relu BN output agree bit for bit.
typedef float bn_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bn_bf16x2 __attribute__((ext_vector_type(2)));
typedef short bn_s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t bn_relu2(uint32_t w, bn_f32x2 sc, bn_f32x2 sh) {
  const bn_f32x2 y = {__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u)};
  const bn_f32x2 z = __builtin_elementwise_fma(y, sc, sh);
  bn_s16x2 b = __builtin_bit_cast(bn_s16x2, __builtin_convertvector(z, bn_bf16x2));
  b = __builtin_elementwise_max(b, (bn_s16x2){0, 0});
  return __builtin_bit_cast(uint32_t, b);
}

// A statistics-partials destination as a kernel argument: the [rows][2][N] buffer and its mode
// (bn_slots(), see conv_kernels.h) fixed at launch -- so a captured graph keeps the mode it was built
// with, and every device of a process follows the host setting (there is no device-side copy).
struct BnPart {
  float* p = nullptr;
  int slots = 0;  // 0: row mode (plain stores into row `row`); S > 0: fp32 atomics into slot row % S
};
// Row of the buffer that producer row block `row` writes: the block itself (row mode), or row % S.
__device__ __forceinline__ int bn_part_row(const BnPart& part, int row) {
  return part.slots > 0 ? row % part.slots : row;
}
// One producer block's column sums (a, b) of channel n: a plain store into its row, or fp32 atomic
// adds into its slot of a zeroed buffer.
__device__ __forceinline__ void put_bn_part(const BnPart& part, int row, int N, int n, float a, float b) {
  float* p = part.p + (size_t)bn_part_row(part, row) * 2 * N;
  if (part.slots > 0) {
    atomicAdd(p + n, a);
    atomicAdd(p + N + n, b);
  } else {
    p[n] = a;
    p[N + n] = b;
  }
}

}  // namespace tfd
