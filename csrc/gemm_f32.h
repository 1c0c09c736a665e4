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
// Padding 4 keeps every fragment read conflict-free (read_frag4_f); a KC row stays 16-B aligned.
#pragma once
#include "common.h"
#include "gemm.h"  // buf_ld

#include <type_traits>

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

// Four K-steps of one operand fragment per read, K permuted inside each 16-deep group: lane group
// g = lane >> 4 holds k = kq + 4g .. kq + 4g + 3, and MFMA s of the group takes component s, so MFMA s
// sums k = kq + s + {0, 4, 8, 12} and the four MFMAs together cover the group exactly once (A and B
// use the same map). KC tiles: one ds_read_b128 per lane ([MN][BK + 4] rows are 144 B apart: the 16
// rows of a lane group hit 64 distinct banks). !KC tiles: four ds_read_b32 from rows 4 apart; with a
// row of MN + 4 floats, 4 rows = 16 banks mod 64, so the four lane groups are conflict-free too.
template <int MN, int BK, bool KC>
__device__ __forceinline__ f32x4 read_frag4_f(const float* lds, int r0, int kq, int lane) {
  using L = LdsTileF<MN, BK, KC>;
  const int i = lane & 15, k = kq + 4 * (lane >> 4);
  if constexpr (KC) {
    return *reinterpret_cast<const f32x4*>(lds + (r0 + i) * L::ROW + k);
  } else {
    const float* p = lds + k * L::ROW + r0 + i;
    return f32x4{p[0], p[L::ROW], p[2 * L::ROW], p[3 * L::ROW]};
  }
}

// Branch-free float4 operand load (raw buffer load; an out-of-range chunk gets an offset past the
// descriptor, which the hardware range check returns as zeros): no exec-masked branch per load, so the
// register pipeline keeps the next K-tiles' loads in flight.
__device__ __forceinline__ f32x4 buf_ld_f4(const float* base, uint32_t nbytes, uint32_t elem_off, bool ok) {
  const uint4 u = buf_ld(reinterpret_cast<const uint16_t*>(base), nbytes, elem_off * 2u, ok);
  return f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
}

// An epilogue with `static constexpr bool STAGED = true` gets the whole C tile through LDS instead of
// fragment by fragment: the accumulators go to a [BM][BN + 4] float image (the operand tiles' LDS,
// dead after the last K-step), then epi.tile<BM, BN, NT>(img, BN + 4, m0, n0) stores whole 16-B
// chunks of rows -- a wave instruction writes 1 KiB of row bytes instead of 4-B scalars in 64-B row
// pieces (the bf16 step's fc epilogues, docs/DESIGN.md §4c).
template <class E, class = void>
struct EpiStaged { static constexpr bool value = false; };
template <class E>
struct EpiStaged<E, std::void_t<decltype(E::STAGED)>> { static constexpr bool value = E::STAGED; };

// C tile (m0, n0) over k in [kbeg, kend); WM x WN waves; epilogue epi(m4, n, f32x4 rows m4..m4+3).
// Two register stages: the global loads of K-tile t+2 are issued while tile t+1 still waits in
// registers (two K-iterations of latency cover; 268 -> 190 us/step for the fp32 MNIST step, 3-4 stages
// no better, profiles/mnist_fp32_gemm_ab_r2.log). The loop body is the pair (t, t+1) with one exit, and
// the loads are unconditional (loaders zero or range-check past their bounds; loads past kend are
// never stored): a mid-body exit or per-tile load guards made the compiler shuttle the accumulators
// between AGPRs and VGPRs every iteration and drain vmcnt before each load batch.
template <int BM, int BN, int BK, int WM, int WN, class LA, class LB, class EPI>
__device__ __forceinline__ void gemm_block_f32(const LA& la, const LB& lb, const EPI& epi, int m0, int n0, int kbeg,
                                               int kend, float* smem) {
  constexpr int NT = 64 * WM * WN;
  using TA = LdsTileF<BM, BK, LA::KC>;
  using TB = LdsTileF<BN, BK, LB::KC>;
  static_assert(BK % 16 == 0 && BM % (16 * WM) == 0 && BN % (16 * WN) == 0, "tile shape");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int CA = (TA::CHUNKS + NT - 1) / NT;
  constexpr int CB = (TB::CHUNKS + NT - 1) / NT;
  float* const A0 = smem;
  float* const A1 = smem + TA::ELEMS;
  float* const B0 = smem + 2 * TA::ELEMS;
  float* const B1 = smem + 2 * TA::ELEMS + TB::ELEMS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  f32x4 ra0[CA], rb0[CB], ra1[CA], rb1[CB];
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
  // every fragment of the K-tile is read before the first MFMA (the scheduler otherwise interleaves
  // each read with a wait right before its MFMAs), and the next loads are pinned at the top of each
  // half-iteration (sunk below the compute they got one K-tile of latency cover instead of two)
  auto compute = [&](const float* A, const float* Bt) {
    constexpr int KQ = BK / 16;
    f32x4 a[KQ][TM], b[KQ][TN];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
#pragma unroll
      for (int i = 0; i < TM; ++i) a[q][i] = read_frag4_f<BM, BK, LA::KC>(A, wm * WTM + 16 * i, 16 * q, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[q][j] = read_frag4_f<BN, BK, LB::KC>(Bt, wn * WTN + 16 * j, 16 * q, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < KQ; ++q)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x4f32(a[q][i][s], b[q][j][s], acc[i][j]);
  };
  const int nk = (kend - kbeg + BK - 1) / BK;
  // LDS buffer 0 holds even tiles, 1 odd tiles; register set 0 even tiles, set 1 odd tiles
  gload(kbeg, ra0, rb0);
  gload(kbeg + BK, ra1, rb1);
  sstore(A0, B0, ra0, rb0);
  __syncthreads();
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    gload(kbeg + (t + 2) * BK, ra0, rb0);
    __builtin_amdgcn_sched_barrier(0);
    compute(A0, B0);
    sstore(A1, B1, ra1, rb1);
    __syncthreads();
    gload(kbeg + (t + 3) * BK, ra1, rb1);
    __builtin_amdgcn_sched_barrier(0);
    compute(A1, B1);
    if (t + 2 < nk) sstore(A0, B0, ra0, rb0);
    __syncthreads();
  }
  if (t < nk) compute(A0, B0);
  if constexpr (EpiStaged<EPI>::value) {
    constexpr int P = BN + 4;
    static_assert(BM * P <= 2 * (TA::ELEMS + TB::ELEMS), "the C image fits the operand tiles' LDS");
    __syncthreads();  // every wave's last fragment reads are done
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          smem[(wm * WTM + 16 * i + 4 * (lane >> 4) + r) * P + wn * WTN + 16 * j + (lane & 15)] = acc[i][j][r];
    __syncthreads();
    epi.template tile<BM, BN, NT>(smem, P, m0, n0);
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        epi(m0 + wm * WTM + 16 * i + 4 * (lane >> 4), n0 + wn * WTN + 16 * j + (lane & 15), acc[i][j]);
  }
}

// Row-major fp32 X[rows][ld]: KC: (mn, k) = X[mn][k]; !KC: (mn, k) = X[k][mn]. A chunk is all in or
// all out (zeros): the caller keeps ld and the chunked bound (k_lim for KC, mn_lim for !KC) multiples
// of 4.
template <bool KC_>
struct DenseLoaderF {
  static constexpr bool KC = KC_;
  const float* __restrict__ x;
  int ld, mn_lim, k_lim;
  __device__ __forceinline__ f32x4 operator()(int mn, int k) const {
    const bool ok = mn < mn_lim && k < k_lim;
    if constexpr (KC) return buf_ld_f4(x, (uint32_t)mn_lim * (uint32_t)ld * 4u, (uint32_t)mn * (uint32_t)ld + (uint32_t)k, ok);
    else return buf_ld_f4(x, (uint32_t)k_lim * (uint32_t)ld * 4u, (uint32_t)k * (uint32_t)ld + (uint32_t)mn, ok);
  }
};

}  // namespace tfd
