// Generic LDS-staged MFMA GEMM core for gfx950 (bf16 in, fp32 accumulate).
//
// C[m][n] = sum_k A[m][k] * B[k][n], computed per workgroup tile BM x BN, K stepped by BK.
// Operands are produced by *loader functors* so the same core serves plain GEMMs, implicit-GEMM
// convolutions (im2col gather in the loader) and transposed operands:
//
//   struct Loader { static constexpr bool KC = ...;           // k-contiguous chunks?
//                   __device__ uint4 operator()(int mn, int k) const; };
//   KC = true : returns 8 bf16 {X[mn][k..k+7]}   -> LDS image [MN][BK+8], fragments by ds_read_b128
//   KC = false: returns 8 bf16 {X[mn..mn+7][k]}  -> LDS image [BK][MN+16], fragments by two
//               ds_read_b64_tr_b16 (hardware transpose read; no separate transposed weight copies)
//   Loaders zero-fill out-of-range elements.
//
// Epilogue functor: epi(m4, n, f32x4 v) receives rows m4..m4+3 (m4 % 4 == 0) of column n: the
// mfma_f32_16x16x32 C layout (row = 4*(lane>>4)+r, col = lane&15) gives each lane 4 consecutive
// rows, which the fused pool epilogue uses as one 2x2 window.
//
// Pipeline: register-staged double-buffered LDS (global loads of tile t+1 are issued before the
// MFMAs on tile t and written after them), one barrier per K-tile.
#pragma once
#include <type_traits>

#include "common.h"

namespace tfd {

// Epilogues that declare `static constexpr bool WANTS_IJ = true` are called as
// epi(m4, n, v, i, j) with the compile-time (after unrolling) tile indices of the lane's
// accumulator, so they can consume per-tile values they prefetched before the K loop.
template <class E, class = void>
struct EpiWantsIJ : std::false_type {};
template <class E>
struct EpiWantsIJ<E, std::void_t<decltype(E::WANTS_IJ)>> : std::integral_constant<bool, E::WANTS_IJ> {};
template <class EPI>
__device__ __forceinline__ void epi_call(const EPI& epi, int m4, int n, const f32x4& v, int i, int j) {
  if constexpr (EpiWantsIJ<EPI>::value) epi(m4, n, v, i, j);
  else epi(m4, n, v);
}

// LDS images (MI355X LDS: 64 banks x 4 B; ds_read_b128 in 4 groups of 16 lanes, ds_read_b64_tr_b16
// in 2 groups of 32, tools/debug/lds_banks.py):
//  KC = true : [MN][BK + 16] -- the 16 rows of a b128 fragment read land 8 banks apart per row
//              (pad 8 put rows r and r + 8 on the same banks: 2-way on every read);
//  KC = false: [BK][MN] with the 16-B chunk index of row k XORed by swz_chunk(k) (no pad): the 8
//              rows k = kk + 8g + q (g < 2, q < 4) of one tr-read lane group cover 8 disjoint 8-bank
//              windows (pad 16 mapped rows k and k + 8 to the same banks: 2-way on every read).
// (measured: ResNet-50 -0.6 %, the MNIST step neutral -- profiles/ab_gemm_lds_swz_r3.log)
template <int CPR>
__device__ __forceinline__ int swz_chunk(int k) {
  if constexpr ((CPR & (CPR - 1)) != 0 || CPR < 4) return 0;
  else if constexpr (CPR >= 16) return (2 * (k & 1) + 4 * ((k >> 1) & 1) + 8 * ((k >> 3) & 1)) & (CPR - 1);
  else if constexpr (CPR == 8) return 2 * ((k >> 1) & 1) + 4 * ((k >> 3) & 1);
  else return 2 * ((k >> 3) & 1);
}
template <int MN, int BK, bool KC>
struct LdsTile {
  static constexpr int CH_PER_ROW = KC ? BK / 8 : MN / 8; // 16-byte chunks per LDS row
  static constexpr bool SWZ = !KC && (CH_PER_ROW & (CH_PER_ROW - 1)) == 0 && CH_PER_ROW >= 4;
  static constexpr int PAD = KC ? 16 : (SWZ ? 0 : 16);  // elements
  static constexpr int ROW = KC ? (BK + PAD) : (MN + PAD);
  static constexpr int ELEMS = KC ? MN * ROW : BK * ROW;
  static constexpr int CHUNKS = MN * BK / 8;
  // element offset of (LDS row, column col) -- col a multiple of 4 inside one 16-B chunk
  static __device__ __forceinline__ int at(int row, int col) {
    if constexpr (SWZ) return row * ROW + (((col >> 3) ^ swz_chunk<CH_PER_ROW>(row)) << 3) + (col & 7);
    else return row * ROW + col;
  }
};

typedef __attribute__((ext_vector_type(8))) short s16x8;

template <int MN, int BK, bool KC>
__device__ __forceinline__ bf16x8 read_frag(const bf16* lds, int r0, int kk, int lane) {
  using L = LdsTile<MN, BK, KC>;
  if constexpr (KC) {
    const bf16* p = lds + (r0 + (lane & 15)) * L::ROW + kk + 8 * (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p4 = i & 3;
    const bf16* p0 = lds + L::at(kk + 8 * g + q, r0 + 4 * p4);
    const bf16* p1 = lds + L::at(kk + 8 * g + q + 4, r0 + 4 * p4);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p1));
    s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
  }
}

// Transposed operand fragment (mfma_f32_16x16x32_bf16 A or B) from an LDS image stored with
// rows = k and columns = m/n (m/n contiguous, 16-B aligned rows). For lane l (g = l >> 4,
// q = (l & 15) >> 2, p4 = l & 3) the caller passes p0 = &image[row(8g + q)][c0 + 4 p4] and
// p1 = &image[row(8g + q + 4)][c0 + 4 p4]; rows may be arbitrary per lane (im2col gathers), the
// result holds {X[k = 8g + j][c0 + (l & 15)] : j = 0..7}. EXEC must be all ones.
__device__ __forceinline__ bf16x8 frag_tr16(const bf16* p0, const bf16* p1) {
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p1));
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// Operand transforms: a loader that declares `static constexpr int XF_BYTES` still travels
// global -> registers -> LDS, but gload keeps a per-chunk tag (v = ld.load(mn, k, tag)) and before
// the LDS store ld.xform(v[], tag[], table) rewrites the thread's chunks of the K-tile in place;
// ld.stage(table) fills the loader's XF_BYTES-byte LDS table (placed after the operand images) once
// per block, before the first store. Used by the
// conv loaders that apply the producing layer's batch norm + relu while staging their input
// (csrc/kernels/conv_nhwc.hip BnRelu).
template <class L, class = void>
struct LoaderXF {
  static constexpr int BYTES = 0;
};
template <class L>
struct LoaderXF<L, std::void_t<decltype(L::XF_BYTES)>> {
  static constexpr int BYTES = L::XF_BYTES;
};

template <int BM, int BN, int BK, class LA, class LB>
struct GemmSmem {
  using TA = LdsTile<BM, BK, LA::KC>;
  using TB = LdsTile<BN, BK, LB::KC>;
  static constexpr int BYTES = 2 * (TA::ELEMS + TB::ELEMS) * 2 + LoaderXF<LA>::BYTES + LoaderXF<LB>::BYTES;
};

// One workgroup computes the BM x BN tile at (m0, n0) over k in [kbeg, kend).
// WM x WN waves (64*WM*WN threads). kend - kbeg should be a multiple of BK except at the global
// K tail (loaders zero-fill past K).
// RS = register stages: with RS = 2 the global loads of tile t+2 are issued while tile t+1 still
// sits in registers, so every load has ~2 K-iterations of latency cover (twice the bytes in flight
// per CU -- these small GEMMs are bound by bytes-in-flight / memory latency, not by MFMA rate).
// gemm_mainloop: the K loop only, accumulating into the caller's acc[TM][TN] (TM = BM/WM/16,
// TN = BN/WN/16); gemm_block = mainloop + per-fragment epilogue calls. Kernels with a block-wide
// epilogue (LDS-staged stores, csrc/kernels/conv_nhwc.hip) call the mainloop directly. The loop
// ends with a barrier, so the operand LDS images are dead when it returns.
template <int BM, int BN, int BK, int WM, int WN, class LA, class LB, int RS = 1>
__device__ __forceinline__ void gemm_mainloop(const LA& la, const LB& lb, int m0, int n0, int kbeg, int kend,
                                              bf16* smem, f32x4 (&acc)[BM / WM / 16][BN / WN / 16]) {
  constexpr int NT = 64 * WM * WN;
  using TA = LdsTile<BM, BK, LA::KC>;
  using TB = LdsTile<BN, BK, LB::KC>;
  static_assert(BK % 32 == 0, "BK multiple of 32");
  static_assert(BM % (16 * WM) == 0 && BN % (16 * WN) == 0, "tile/wave mismatch");
  static_assert(RS >= 1 && RS <= 8, "register stages");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int CA = (TA::CHUNKS + NT - 1) / NT;
  constexpr int CB = (TB::CHUNKS + NT - 1) / NT;
  constexpr bool XA = LoaderXF<LA>::BYTES > 0, XB = LoaderXF<LB>::BYTES > 0;
  bf16* As0 = smem;
  bf16* As1 = smem + TA::ELEMS;
  bf16* Bs0 = smem + 2 * TA::ELEMS;
  bf16* Bs1 = Bs0 + TB::ELEMS;
  char* xtab_a = reinterpret_cast<char*>(smem + 2 * (TA::ELEMS + TB::ELEMS));
  char* xtab_b = xtab_a + LoaderXF<LA>::BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  uint4 ra[RS][CA], rb[RS][CB];
  [[maybe_unused]] int ta[RS][CA], tb[RS][CB];  // transform tags (XA / XB loaders only)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto gload = [&](int k0, uint4 (&xa)[CA], uint4 (&xb)[CB], int (&ga)[CA], int (&gb)[CB]) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (CA * NT == TA::CHUNKS || idx < TA::CHUNKS) {
        const int row = idx / TA::CH_PER_ROW, col = (idx % TA::CH_PER_ROW) * 8;
        const int mn = LA::KC ? m0 + row : m0 + col, k = LA::KC ? k0 + col : k0 + row;
        if constexpr (XA) xa[c] = la.load(mn, k, ga[c]);
        else xa[c] = la(mn, k);
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (CB * NT == TB::CHUNKS || idx < TB::CHUNKS) {
        const int row = idx / TB::CH_PER_ROW, col = (idx % TB::CH_PER_ROW) * 8;
        const int mn = LB::KC ? n0 + row : n0 + col, k = LB::KC ? k0 + col : k0 + row;
        if constexpr (XB) xb[c] = lb.load(mn, k, gb[c]);
        else xb[c] = lb(mn, k);
      }
    }
  };
  // a transform sees all of the thread's chunks at once: they share the LDS column `col` (the asserts),
  // so a per-channel transform looks its constants up once per K-tile
  static_assert(!XA || (CA * NT == TA::CHUNKS && NT % TA::CH_PER_ROW == 0), "XF layout (A)");
  static_assert(!XB || (CB * NT == TB::CHUNKS && NT % TB::CH_PER_ROW == 0), "XF layout (B)");
  auto sstore = [&](bf16* As, bf16* Bs, const uint4 (&xa)[CA], const uint4 (&xb)[CB], const int (&ga)[CA],
                    const int (&gb)[CB]) {
    uint4 va[CA], vb[CB];
#pragma unroll
    for (int c = 0; c < CA; ++c) va[c] = xa[c];
#pragma unroll
    for (int c = 0; c < CB; ++c) vb[c] = xb[c];
    if constexpr (XA) la.xform(va, ga, xtab_a);
    if constexpr (XB) lb.xform(vb, gb, xtab_b);
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (CA * NT == TA::CHUNKS || idx < TA::CHUNKS) {
        const int row = idx / TA::CH_PER_ROW, col = (idx % TA::CH_PER_ROW) * 8;
        *reinterpret_cast<uint4*>(As + TA::at(row, col)) = va[c];
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (CB * NT == TB::CHUNKS || idx < TB::CHUNKS) {
        const int row = idx / TB::CH_PER_ROW, col = (idx % TB::CH_PER_ROW) * 8;
        *reinterpret_cast<uint4*>(Bs + TB::at(row, col)) = vb[c];
      }
    }
  };
  // transform tables: built while the first tiles' loads are in flight, visible before the first store
  auto stage_tables = [&]() {
    if constexpr (XA || XB) {
      if constexpr (XA) la.stage(xtab_a);
      if constexpr (XB) lb.stage(xtab_b);
      __syncthreads();
    }
  };
  auto compute = [&](const bf16* As, const bf16* Bs) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = read_frag<BM, BK, LA::KC>(As, wm * WTM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = read_frag<BN, BK, LB::KC>(Bs, wn * WTN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
    }
  };

  const int nk = (kend - kbeg + BK - 1) / BK;
  if constexpr (RS == 1) {
    if (nk > 0) {
      gload(kbeg, ra[0], rb[0], ta[0], tb[0]);
      stage_tables();
      sstore(As0, Bs0, ra[0], rb[0], ta[0], tb[0]);
      __syncthreads();
      for (int t = 0; t < nk; ++t) {
        const bool odd = t & 1;
        if (t + 1 < nk) gload(kbeg + (t + 1) * BK, ra[0], rb[0], ta[0], tb[0]);
        compute(odd ? As1 : As0, odd ? Bs1 : Bs0);
        if (t + 1 < nk) sstore(odd ? As0 : As1, odd ? Bs0 : Bs1, ra[0], rb[0], ta[0], tb[0]);
        __syncthreads();
      }
    }
  } else if constexpr (RS > 2) {
    // Register ring: set u = t % RS holds tile t until it is written to LDS at step t-1, then is
    // refilled with tile t+RS -- RS tiles of loads in flight behind the MFMAs (long-K blocks).
    if (nk > 0) {
#pragma unroll
      for (int u = 0; u < RS; ++u)
        if (u < nk) gload(kbeg + u * BK, ra[u], rb[u], ta[u], tb[u]);
      stage_tables();
      sstore(As0, Bs0, ra[0], rb[0], ta[0], tb[0]);
      __syncthreads();
      for (int t0 = 0; t0 < nk; t0 += RS) {
#pragma unroll
        for (int u = 0; u < RS; ++u) {
          const int t = t0 + u;
          if (t < nk) {
            if (t + RS < nk) gload(kbeg + (t + RS) * BK, ra[u], rb[u], ta[u], tb[u]);
            compute((t & 1) ? As1 : As0, (t & 1) ? Bs1 : Bs0);
            if (t + 1 < nk)
              sstore((t & 1) ? As0 : As1, (t & 1) ? Bs0 : Bs1, ra[(u + 1) % RS], rb[(u + 1) % RS], ta[(u + 1) % RS],
                     tb[(u + 1) % RS]);
            __syncthreads();
          }
        }
      }
    }
  } else {
    // LDS[t&1] holds tile t; register set (t+1)&1 holds tile t+1; tile t+2 loads into set t&1.
    if (nk > 0) {
      gload(kbeg, ra[0], rb[0], ta[0], tb[0]);
      if (nk > 1) gload(kbeg + BK, ra[1], rb[1], ta[1], tb[1]);
      stage_tables();
      sstore(As0, Bs0, ra[0], rb[0], ta[0], tb[0]);
      __syncthreads();
      for (int t = 0; t < nk; t += 2) {
        // even step: compute LDS0 (tile t), regs1 = tile t+1, refill regs0 with tile t+2
        if (t + 2 < nk) gload(kbeg + (t + 2) * BK, ra[0], rb[0], ta[0], tb[0]);
        compute(As0, Bs0);
        if (t + 1 < nk) sstore(As1, Bs1, ra[1], rb[1], ta[1], tb[1]);
        __syncthreads();
        if (t + 1 >= nk) break;
        // odd step: compute LDS1 (tile t+1), regs0 = tile t+2, refill regs1 with tile t+3
        if (t + 3 < nk) gload(kbeg + (t + 3) * BK, ra[1], rb[1], ta[1], tb[1]);
        compute(As1, Bs1);
        if (t + 2 < nk) sstore(As0, Bs0, ra[0], rb[0], ta[0], tb[0]);
        __syncthreads();
      }
    }
  }
}

template <int BM, int BN, int BK, int WM, int WN, class LA, class LB, class EPI, int RS = 1>
__device__ __forceinline__ void gemm_block(const LA& la, const LB& lb, const EPI& epi, int m0, int n0,
                                           int kbeg, int kend, bf16* smem) {
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  f32x4 acc[TM][TN];
  gemm_mainloop<BM, BN, BK, WM, WN, LA, LB, RS>(la, lb, m0, n0, kbeg, kend, smem, acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid / WN, wn = wid % WN;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      epi_call(epi, m0 + wm * WTM + 16 * i + 4 * (lane >> 4), n0 + wn * WTN + 16 * j + (lane & 15), acc[i][j], i, j);
}

// Whole-K variant for short, latency-bound K ranges (split-K slabs): the global loads of ALL NKT
// K-tiles are issued back to back (NKT x (CA + CB) x 16 B per lane in flight), each tile is written
// to its own LDS slot as soon as its loads land (in-order vmcnt), then ONE barrier and the MFMA
// sweep. Replaces the NKT-deep load -> barrier chain of gemm_block by a single memory round trip.
// LDS: NKT x GemmSmem/2 bytes; K range [kbeg, kbeg + NKT*BK) (loaders zero-fill past K).
template <int BM, int BN, int BK, int NKT, class LA, class LB>
struct GemmSmemOneshot {
  static constexpr int BYTES = NKT * (LdsTile<BM, BK, LA::KC>::ELEMS + LdsTile<BN, BK, LB::KC>::ELEMS) * 2;
};
template <int BM, int BN, int BK, int NKT, int WM, int WN, class LA, class LB, class EPI>
__device__ __forceinline__ void gemm_block_oneshot(const LA& la, const LB& lb, const EPI& epi, int m0, int n0,
                                                   int kbeg, bf16* smem) {
  constexpr int NT = 64 * WM * WN;
  using TA = LdsTile<BM, BK, LA::KC>;
  using TB = LdsTile<BN, BK, LB::KC>;
  static_assert(BK % 32 == 0 && BM % (16 * WM) == 0 && BN % (16 * WN) == 0, "tile shape");
  static_assert(LoaderXF<LA>::BYTES == 0 && LoaderXF<LB>::BYTES == 0, "operand transforms: gemm_mainloop only");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int CA = (TA::CHUNKS + NT - 1) / NT;
  constexpr int CB = (TB::CHUNKS + NT - 1) / NT;
  bf16* As = smem;
  bf16* Bs = smem + NKT * TA::ELEMS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  uint4 ra[NKT][CA], rb[NKT][CB];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    const int k0 = kbeg + t * BK;
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (CA * NT == TA::CHUNKS || idx < TA::CHUNKS) {
        const int row = idx / TA::CH_PER_ROW, col = (idx % TA::CH_PER_ROW) * 8;
        if constexpr (LA::KC) ra[t][c] = la(m0 + row, k0 + col);
        else ra[t][c] = la(m0 + col, k0 + row);
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (CB * NT == TB::CHUNKS || idx < TB::CHUNKS) {
        const int row = idx / TB::CH_PER_ROW, col = (idx % TB::CH_PER_ROW) * 8;
        if constexpr (LB::KC) rb[t][c] = lb(n0 + row, k0 + col);
        else rb[t][c] = lb(n0 + col, k0 + row);
      }
    }
  }
  // every load is issued before the first LDS store: without this fence the scheduler interleaves
  // them (to save registers) and the staging becomes several round trips
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (CA * NT == TA::CHUNKS || idx < TA::CHUNKS) {
        const int row = idx / TA::CH_PER_ROW, col = (idx % TA::CH_PER_ROW) * 8;
        *reinterpret_cast<uint4*>(As + t * TA::ELEMS + TA::at(row, col)) = ra[t][c];
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (CB * NT == TB::CHUNKS || idx < TB::CHUNKS) {
        const int row = idx / TB::CH_PER_ROW, col = (idx % TB::CH_PER_ROW) * 8;
        *reinterpret_cast<uint4*>(Bs + t * TB::ELEMS + TB::at(row, col)) = rb[t][c];
      }
    }
  }
  __syncthreads();
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NKT; ++t)
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = read_frag<BM, BK, LA::KC>(As + t * TA::ELEMS, wm * WTM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = read_frag<BN, BK, LB::KC>(Bs + t * TB::ELEMS, wn * WTN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
    }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      epi(m0 + wm * WTM + 16 * i + 4 * (lane >> 4), n0 + wn * WTN + 16 * j + (lane & 15), acc[i][j]);
}

// ---------------- common loaders ----------------
__device__ __forceinline__ uint4 zero4() { return make_uint4(0u, 0u, 0u, 0u); }

// Branch-free 16-B operand load: a raw buffer load through a descriptor over [base, base + nbytes)
// (built from kernel arguments, so scalar); an out-of-range chunk (ok == false) gets an offset past
// the range, which the hardware range check returns as zeros. No exec-masked branch around the
// load, so the compiler can count loads in flight (register pipelines, RS > 1). nbytes < 2 GiB.
typedef int i32x4v __attribute__((ext_vector_type(4)));
constexpr uint32_t kBufOOB = 0xFFFFFFF0u;
// one byte (relu / mask bits), branch-free: an exec-masked byte load is waited for inside its branch
__device__ __forceinline__ uint32_t buf_ld_u8(const uint8_t* base, uint32_t nbytes, uint32_t off, bool ok) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nbytes, 0x00020000);
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, ok ? off : kBufOOB, 0, 0);
}
__device__ __forceinline__ uint4 buf_ld(const uint16_t* base, uint32_t nbytes, uint32_t elem_off, bool ok) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nbytes, 0x00020000);
  const i32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? elem_off * 2u : kBufOOB, 0, 0);
  return make_uint4((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]);
}

// Row-major X[rows][ld] bf16; chunk runs along the contiguous (column) dimension.
//  KC=true : operand index (mn, k) = X[mn][k]   (A as [M][K] or B as [N][K])
//  KC=false: operand index (mn, k) = X[k][mn]   (A as [K][M] or B as [K][N])
template <bool KC_>
struct DenseLoader {
  static constexpr bool KC = KC_;
  const uint16_t* __restrict__ x;
  int ld, mn_lim, k_lim;  // logical bounds (mn < mn_lim, k < k_lim)
  __device__ __forceinline__ uint4 operator()(int mn, int k) const {
    if constexpr (KC) {
      if (mn >= mn_lim || k >= k_lim) return zero4();
      if (k + 8 <= k_lim) return *reinterpret_cast<const uint4*>(x + (size_t)mn * ld + k);
      uint16_t t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = (k + j < k_lim) ? x[(size_t)mn * ld + k + j] : 0;
      return *reinterpret_cast<uint4*>(t);
    } else {
      if (k >= k_lim || mn >= mn_lim) return zero4();
      if (mn + 8 <= mn_lim) return *reinterpret_cast<const uint4*>(x + (size_t)k * ld + mn);
      uint16_t t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = (mn + j < mn_lim) ? x[(size_t)k * ld + mn + j] : 0;
      return *reinterpret_cast<uint4*>(t);
    }
  }
};

// DenseLoader for shapes whose chunked dimension is a multiple of 8 (k_lim for KC, mn_lim for !KC),
// so a chunk is all in or all out: one raw buffer load per chunk, out-of-range chunks read as zeros
// by the hardware range check. No branch: DenseLoader's exec-masked loads merged by a phi made the
// compiler copy a loaded register (and so drain vmcnt) in the middle of a prologue's load batch.
template <bool KC_>
struct DenseLoaderX {
  static constexpr bool KC = KC_;
  const uint16_t* __restrict__ x;
  int ld, mn_lim, k_lim;
  __device__ __forceinline__ uint4 operator()(int mn, int k) const {
    const bool ok = mn < mn_lim && k < k_lim;
    if constexpr (KC) return buf_ld(x, (uint32_t)mn_lim * (uint32_t)ld * 2u, (uint32_t)mn * (uint32_t)ld + (uint32_t)k, ok);
    else return buf_ld(x, (uint32_t)k_lim * (uint32_t)ld * 2u, (uint32_t)k * (uint32_t)ld + (uint32_t)mn, ok);
  }
};

}  // namespace tfd
