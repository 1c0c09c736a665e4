// Forward batch-norm affine constants of one channel: out = relu?(y * sc + sh) with sc = invstd * gamma,
// sh = beta - mean * sc (one explicit fma). Every kernel that forms a BN output or re-derives its relu
// mask -- norm.hip's apply and backward passes, the conv loaders that apply their input's BN while
// staging it (csrc/kernels/conv_nhwc.hip BnRelu), the dgrad BN-statistics epilogue -- takes these exact
// values and the same fmaf(y, sc, sh), so a mask recomputed from y matches the relu the consumer
// applied bit for bit.
#pragma once
#include <hip/hip_runtime.h>

namespace tfd {

__device__ __forceinline__ void bn_affine(float mean, float invstd, float gamma, float beta, float& sc, float& sh) {
  sc = invstd * gamma;
  sh = fmaf(-mean, sc, beta);
}

}  // namespace tfd
