// Forward batch-norm affine constants of one channel: out = relu?(y * sc + sh) with sc = invstd * gamma,
// sh = beta - mean * sc (one explicit fma). Every kernel that forms a BN output or re-derives its relu
// mask -- norm.hip's apply and backward passes, the conv loaders that apply their input's BN while
// staging it (csrc/kernels/conv_nhwc.hip BnRelu), the dgrad BN-statistics epilogue -- takes these exact
// values and the same fmaf(y, sc, sh), so a mask recomputed from y matches the relu the consumer
// applied bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "conv_kernels.h"  // TFD_BN_SLOTS

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

// The statistics-partials mode (bn_slots(), see conv_kernels.h) as each kernel TU's own device copy:
// internal linkage, so conv_nhwc.hip and norm.hip each hold one, uploaded by set_bn_slots.
static __device__ int g_bn_slots_dev = TFD_BN_SLOTS;
static inline hipError_t bn_slots_upload(int s) { return hipMemcpyToSymbol(HIP_SYMBOL(g_bn_slots_dev), &s, sizeof(int)); }

// Row of a [rows][2][N] statistics-partials buffer that producer row block `row` writes: the block
// itself (row mode), or slot row % S (slot mode).
__device__ __forceinline__ int bn_part_row(int row) {
  const int sl = g_bn_slots_dev;
  return sl > 0 ? row % sl : row;
}
// One producer block's column sums (a, b) of channel n: a plain store into its row, or fp32 atomic
// adds into its slot of a zeroed buffer.
__device__ __forceinline__ void put_bn_part(float* part, int row, int N, int n, float a, float b) {
  float* p = part + (size_t)bn_part_row(row) * 2 * N;
  if (g_bn_slots_dev > 0) {
    atomicAdd(p + n, a);
    atomicAdd(p + N + n, b);
  } else {
    p[n] = a;
    p[N + n] = b;
  }
}

}  // namespace tfd
