// fp32 LDS-staged MFMA GEMM core for gfx950: the reference-precision (--dtype fp32) path.
//
// Same shape as csrc/gemm.h (loader functors, epilogue functors, one workgroup = BM x BN tile,
// double-buffered LDS), but operands stay fp32 end to end and the matrix core runs
// v_mfma_f32_16x16x4_f32: lane l supplies A[m = l & 15][k = l >> 4] and B[k = l >> 4][n = l & 15]
// (one float each), and receives C rows 4 (l >> 4) .. +3 of column l & 15 (the same C layout as the
// bf16 core, so the pooled / unpooled epilogues are shared in spirit).
//
//   Loader::KC = true : operator()(mn, k) returns float4 {X[mn][k..k+3]}  -> LDS [MN][BK + 4]
//   Loader::KC = false: operator()(mn, k) returns float4 {X[mn..mn+3][k]} -> LDS [BK][MN + 4]
// Padding 4: with BK = 32 the k-major rows are 36 floats apart, so the 16 row-lanes x 4 k-lanes of
// a fragment read hit 64 distinct banks; the mn-major rows are read along mn (consecutive lanes).
#pragma once
#include "common.h"

namespace tfd {

__device__ __forceinline__ f32x4 mfma16x16x4f32(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 zero_f4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

template <int MN, int BK, bool KC>
struct LdsTileF {
  static constexpr int ROW = KC ? (BK + 4) : (MN + 4);
  static constexpr int ELEMS = KC ? MN * ROW : BK * ROW;
  static constexpr int CH_PER_ROW = KC ? BK / 4 : MN / 4;  // float4 chunks per LDS row
  static constexpr int CHUNKS = MN * BK / 4;
};

template <int BM, int BN, int BK, class LA, class LB>
struct GemmSmemF {
  static constexpr int BYTES = 2 * (LdsTileF<BM, BK, LA::KC>::ELEMS + LdsTileF<BN, BK, LB::KC>::ELEMS) * 4;
};

template <int MN, int BK, bool KC>
__device__ __forceinline__ float read_frag_f(const float* lds, int r0, int kk, int lane) {
  using L = LdsTileF<MN, BK, KC>;
  const int i = lane & 15, k = kk + (lane >> 4);
  if constexpr (KC) return lds[(r0 + i) * L::ROW + k];
  else return lds[k * L::ROW + r0 + i];
}

// C tile (m0, n0) over k in [kbeg, kend); WM x WN waves; epilogue epi(m4, n, f32x4 rows m4..m4+3).
// RS = register stages: RS = 2 issues the global loads of K-tile t+2 while tile t+1 still waits in
// registers (two K-iterations of latency cover instead of one): 268 -> 190 us/step for the fp32 MNIST
// step; 3-4 stages no better (profiles/mnist_fp32_gemm_ab_r2.log).
template <int BM, int BN, int BK, int WM, int WN, class LA, class LB, class EPI, int RS = 2>
__device__ __forceinline__ void gemm_block_f32(const LA& la, const LB& lb, const EPI& epi, int m0, int n0, int kbeg,
                                               int kend, float* smem) {
  constexpr int NT = 64 * WM * WN;
  using TA = LdsTileF<BM, BK, LA::KC>;
  using TB = LdsTileF<BN, BK, LB::KC>;
  static_assert(BK % 4 == 0 && BM % (16 * WM) == 0 && BN % (16 * WN) == 0, "tile shape");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int CA = (TA::CHUNKS + NT - 1) / NT;
  constexpr int CB = (TB::CHUNKS + NT - 1) / NT;
  float* As[2] = {smem, smem + TA::ELEMS};
  float* Bs[2] = {smem + 2 * TA::ELEMS, smem + 2 * TA::ELEMS + TB::ELEMS};
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  static_assert(RS >= 1 && RS <= 6, "register stages");
  f32x4 ra[RS][CA], rb[RS][CB];
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero_f4();

  auto gload = [&](int k0, f32x4 (&xa)[CA], f32x4 (&xb)[CB]) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (CA * NT == TA::CHUNKS || idx < TA::CHUNKS) {
        const int row = idx / TA::CH_PER_ROW, col = (idx % TA::CH_PER_ROW) * 4;
        if constexpr (LA::KC) xa[c] = la(m0 + row, k0 + col);
        else xa[c] = la(m0 + col, k0 + row);
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (CB * NT == TB::CHUNKS || idx < TB::CHUNKS) {
        const int row = idx / TB::CH_PER_ROW, col = (idx % TB::CH_PER_ROW) * 4;
        if constexpr (LB::KC) xb[c] = lb(n0 + row, k0 + col);
        else xb[c] = lb(n0 + col, k0 + row);
      }
    }
  };
  auto sstore = [&](float* A, float* Bt, const f32x4 (&xa)[CA], const f32x4 (&xb)[CB]) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (CA * NT == TA::CHUNKS || idx < TA::CHUNKS) {
        const int row = idx / TA::CH_PER_ROW, col = (idx % TA::CH_PER_ROW) * 4;
        *reinterpret_cast<f32x4*>(A + row * TA::ROW + col) = xa[c];
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (CB * NT == TB::CHUNKS || idx < TB::CHUNKS) {
        const int row = idx / TB::CH_PER_ROW, col = (idx % TB::CH_PER_ROW) * 4;
        *reinterpret_cast<f32x4*>(Bt + row * TB::ROW + col) = xb[c];
      }
    }
  };
  auto compute = [&](const float* A, const float* Bt) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = read_frag_f<BM, BK, LA::KC>(A, wm * WTM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = read_frag_f<BN, BK, LB::KC>(Bt, wn * WTN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x4f32(a[i], b[j], acc[i][j]);
    }
  };
  const int nk = (kend - kbeg + BK - 1) / BK;
  if constexpr (RS == 1) {
    if (nk > 0) {
      gload(kbeg, ra[0], rb[0]);
      sstore(As[0], Bs[0], ra[0], rb[0]);
      __syncthreads();
      for (int t = 0; t < nk; ++t) {
        const int cur = t & 1;
        if (t + 1 < nk) gload(kbeg + (t + 1) * BK, ra[0], rb[0]);
        compute(As[cur], Bs[cur]);
        if (t + 1 < nk) sstore(As[cur ^ 1], Bs[cur ^ 1], ra[0], rb[0]);
        __syncthreads();
      }
    }
  } else if constexpr (RS > 2) {
    // register ring: set u = t % RS holds tile t until it is written to LDS at step t-1, then is
    // refilled with tile t+RS (RS tiles of loads in flight behind the MFMAs)
    if (nk > 0) {
#pragma unroll
      for (int u = 0; u < RS; ++u)
        if (u < nk) gload(kbeg + u * BK, ra[u], rb[u]);
      sstore(As[0], Bs[0], ra[0], rb[0]);
      __syncthreads();
      for (int t0 = 0; t0 < nk; t0 += RS) {
#pragma unroll
        for (int u = 0; u < RS; ++u) {
          const int t = t0 + u;
          if (t < nk) {
            if (t + RS < nk) gload(kbeg + (t + RS) * BK, ra[u], rb[u]);
            compute(As[t & 1], Bs[t & 1]);
            if (t + 1 < nk) sstore(As[(t + 1) & 1], Bs[(t + 1) & 1], ra[(u + 1) % RS], rb[(u + 1) % RS]);
            __syncthreads();
          }
        }
      }
    }
  } else {
    // LDS[t&1] holds tile t; register set (t+1)&1 holds tile t+1; tile t+2 loads into set t&1
    if (nk > 0) {
      gload(kbeg, ra[0], rb[0]);
      if (nk > 1) gload(kbeg + BK, ra[1], rb[1]);
      sstore(As[0], Bs[0], ra[0], rb[0]);
      __syncthreads();
      for (int t = 0; t < nk; t += 2) {
        if (t + 2 < nk) gload(kbeg + (t + 2) * BK, ra[0], rb[0]);
        compute(As[0], Bs[0]);
        if (t + 1 < nk) sstore(As[1], Bs[1], ra[1], rb[1]);
        __syncthreads();
        if (t + 1 >= nk) break;
        if (t + 3 < nk) gload(kbeg + (t + 3) * BK, ra[1], rb[1]);
        compute(As[1], Bs[1]);
        if (t + 2 < nk) sstore(As[0], Bs[0], ra[0], rb[0]);
        __syncthreads();
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      epi(m0 + wm * WTM + 16 * i + 4 * (lane >> 4), n0 + wn * WTN + 16 * j + (lane & 15), acc[i][j]);
}

// Row-major fp32 X[rows][ld]: KC: (mn, k) = X[mn][k]; !KC: (mn, k) = X[k][mn]. Zero past bounds.
template <bool KC_>
struct DenseLoaderF {
  static constexpr bool KC = KC_;
  const float* __restrict__ x;
  int ld, mn_lim, k_lim;
  __device__ __forceinline__ f32x4 operator()(int mn, int k) const {
    if constexpr (KC) {
      if (mn >= mn_lim || k >= k_lim) return zero_f4();
      if (k + 4 <= k_lim) return *reinterpret_cast<const f32x4*>(x + (size_t)mn * ld + k);
      f32x4 t;
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = (k + j < k_lim) ? x[(size_t)mn * ld + k + j] : 0.f;
      return t;
    } else {
      if (k >= k_lim || mn >= mn_lim) return zero_f4();
      if (mn + 4 <= mn_lim) return *reinterpret_cast<const f32x4*>(x + (size_t)k * ld + mn);
      f32x4 t;
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = (mn + j < mn_lim) ? x[(size_t)k * ld + mn + j] : 0.f;
      return t;
    }
  }
};

}  // namespace tfd
