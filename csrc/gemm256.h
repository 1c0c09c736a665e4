// 256-row MFMA GEMM core for gfx950: 8 waves, v_mfma_f32_32x32x16_bf16, operands staged global -> LDS
// by the buffer-load-to-LDS DMA (`buffer_load_dwordx4 ... lds`: no VGPR round trip, no ds_write pass),
// two LDS stages, one barrier per 64-deep K step. Block tile 256 x BN (BN = 256 / 128 / 64).
//
// Why this shape (csrc/gemm.h is the 128 x 128, 4-wave, 16x16x32, register-staged core):
//  * 256 x 256 with 8 waves (a 128 x 64 output per wave) doubles the FLOP per staged byte of a
//    128 x 128 tile -- the LDS image is read 4x less per MFMA;
//  * the 32x32x16 MFMA reads 8 bf16 of A and of B per lane for 32 x 32 x 16 MACs: half the LDS
//    fragment bytes per FLOP of 16x16x32;
//  * the DMA staging frees the VGPRs the register pipeline needed and issues 4x fewer instructions.
// Dense 4096^3: 1025 TF/s against 735 for the 128 x 128 core and 1106 for hipBLASLt on the same GPU
// (profiles/gemm256_dense_r4.txt).
//
// Operand SOURCES map a 16-B chunk to a byte offset inside their buffer descriptor, or past its range
// when the chunk is out of bounds (M / N / K tails, convolution halos), which the hardware range check
// turns into zeros -- implicit-GEMM gathers ride the same DMA path:
//   struct Src { __device__ __amdgpu_buffer_rsrc_t rsrc() const;   // from kernel arguments: scalar
//                __device__ uint32_t off(int mn, int k) const; };
// KC ("k-contiguous") operands: chunk (mn, k) = X[mn][k .. k+7];
// MNC ("mn-contiguous") operands: chunk (mn, k) = X[k][mn .. mn+7] (weight-gradient operands, HWIO
// weights), read back transposed by ds_read_b64_tr_b16.
//
// LDS images (one operand, one stage). The DMA writes lane-linear (one wave instruction = 1 KiB), so
// every bank swizzle is applied to the per-lane SOURCE chunk:
//  KC  [rows][64 bf16] (128-B rows): slot s of row r holds chunk s ^ ((r >> 1) & 7). A fragment read
//      (lane l: row l & 31, chunk 2 ks + (l >> 5)) hits 16 distinct bank quads per 16-lane group.
//  MNC [64 k][W mn] (2W-B rows): slot s of row k holds chunk s ^ sw(k), sw = 4 (k & 3) for W >= 128,
//      4 ((k >> 1) & 1) for W = 64. A transposed fragment read covers 4 rows x 4 chunks per 32-lane
//      half; the swizzle spreads them over the 16 bank quads of a 256-B bank row.
#pragma once
#include "common.h"
#include "gemm.h"  // kBufOOB, frag_tr16

namespace tfd {

__device__ __forceinline__ f32x16 mfma32x32x16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nbytes, 0x00020000);
}

// BN: block columns; WM: waves along M (8 / WM along N); AKC / BKC: operand kinds
template <int BN_ = 256, int WM_ = 2, bool AKC_ = true, bool BKC_ = true>
struct G256 {
  static constexpr int BM = 256, BN = BN_, BK = 64, NT = 512, WM = WM_, WN = 8 / WM_;
  static constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  static constexpr bool AKC = AKC_, BKC = BKC_;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int SMEM = 2 * STAGE_BYTES;
  static_assert(WM * WN == 8 && TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "wave layout");
  static_assert(BN == 64 || BN == 128 || BN == 256, "block columns");
};

__device__ __forceinline__ int kc_slot(int row, int ch) { return ch ^ ((row >> 1) & 7); }
template <int W>
__device__ __forceinline__ int mnc_slot(int k, int ch) {
  return W >= 128 ? ch ^ (4 * (k & 3)) : ch ^ (4 * ((k >> 1) & 1));
}

// DMA one operand tile into `img`: R rows (KC: rows = mn, 64 k each) or W = R columns (MNC: 64 rows = k).
// Either way R / 8 wave instructions of 1 KiB, R / 64 per wave.
template <int R, bool KC, class SRC>
__device__ __forceinline__ void g256_stage_op(const SRC& src, char* img, int mn0, int k0, int w, int l) {
  constexpr int PER_WAVE = R / 64;
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int ins = w * PER_WAVE + i;
    uint32_t off;
    if constexpr (KC) {
      const int row = ins * 8 + (l >> 3);
      off = src.off(mn0 + row, k0 + kc_slot(row, l & 7) * 8);
    } else {
      constexpr int CPR = R / 8, RPI = 64 / CPR;  // chunks per row, rows per instruction
      const int k = ins * RPI + l / CPR;
      off = src.off(mn0 + mnc_slot<R>(k, l % CPR) * 8, k0 + k);
    }
#if defined(__HIP_DEVICE_COMPILE__)  // the DMA builtin exists only for the device pass; a kernel template
    // instantiated from a host-side generic lambda is otherwise rejected by hipcc's host pass
    __builtin_amdgcn_raw_ptr_buffer_load_lds(src.rsrc(), (__attribute__((address_space(3))) void*)(img + ins * 1024), 16,
                                             off, 0, 0, 0);
#else
    (void)off;
#endif
  }
}

// Fragment (8 bf16 along k) of the 32-wide tile starting at row / column t0 for k-sub-step ks.
template <int R, bool KC>
__device__ __forceinline__ bf16x8 g256_frag(const char* img, int t0, int ks, int l) {
  if constexpr (KC) {
    const int row = t0 + (l & 31), ch = 2 * ks + (l >> 5);
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + (kc_slot(row, ch) << 4));
  } else {
    const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
    const int k = ks * 16 + 8 * (g >> 1) + q;
    const int ch = (t0 >> 3) + 2 * (g & 1) + (p >> 1);
    const char* p0 = img + k * (2 * R) + (mnc_slot<R>(k, ch) << 4) + (p & 1) * 8;
    const char* p1 = p0 + 4 * (2 * R);  // row k + 4: same swizzle (k & 3 unchanged)
    return frag_tr16(reinterpret_cast<const bf16*>(p0), reinterpret_cast<const bf16*>(p1));
  }
}

// One 64-deep K step of the wave's WTM x WTN output from the staged images. The fragments of k-sub-step
// ks + 1 are read while ks's MFMAs run (two fragment register sets).
template <class C>
__device__ __forceinline__ void g256_frags(const char* As, const char* Bs, int ks, int wm, int wn, int l,
                                           bf16x8 (&a)[C::TM], bf16x8 (&b)[C::TN]) {
#pragma unroll
  for (int i = 0; i < C::TM; ++i) a[i] = g256_frag<C::BM, C::AKC>(As, wm * C::WTM + i * 32, ks, l);
#pragma unroll
  for (int j = 0; j < C::TN; ++j) b[j] = g256_frag<C::BN, C::BKC>(Bs, wn * C::WTN + j * 32, ks, l);
}
template <class C>
__device__ __forceinline__ void g256_compute(const char* As, const char* Bs, f32x16 (&acc)[C::TM][C::TN], int wm, int wn,
                                             int l) {
  bf16x8 a0[C::TM], b0[C::TN], a1[C::TM], b1[C::TN];
  g256_frags<C>(As, Bs, 0, wm, wn, l, a0, b0);
#pragma unroll
  for (int ks = 0; ks < C::BK / 16; ks += 2) {
    g256_frags<C>(As, Bs, ks + 1, wm, wn, l, a1, b1);
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j) acc[i][j] = mfma32x32x16(a0[i], b0[j], acc[i][j]);
    if (ks + 2 < C::BK / 16) g256_frags<C>(As, Bs, ks + 2, wm, wn, l, a0, b0);
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j) acc[i][j] = mfma32x32x16(a1[i], b1[j], acc[i][j]);
  }
}

// The K loop over [kbeg, kend) (sources zero-fill past their K). Stage t + 1's DMA is issued before
// stage t's MFMAs and retired (vmcnt(0) + barrier) after them.
template <class C, class SA, class SB>
__device__ __forceinline__ void g256_mainloop(const SA& sa, const SB& sb, int m0, int n0, int kbeg, int kend, char* smem,
                                              f32x16 (&acc)[C::TM][C::TN]) {
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, wm = w / C::WN, wn = w % C::WN;
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (kend - kbeg + C::BK - 1) / C::BK;
  if (nk <= 0) return;
  g256_stage_op<C::BM, C::AKC>(sa, smem, m0, kbeg, w, l);
  g256_stage_op<C::BN, C::BKC>(sb, smem + C::A_BYTES, n0, kbeg, w, l);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * C::STAGE_BYTES;
    if (t + 1 < nk) {
      char* nxt = smem + ((t + 1) & 1) * C::STAGE_BYTES;
      const int k1 = kbeg + (t + 1) * C::BK;
      g256_stage_op<C::BM, C::AKC>(sa, nxt, m0, k1, w, l);
      g256_stage_op<C::BN, C::BKC>(sb, nxt + C::A_BYTES, n0, k1, w, l);
    }
    g256_compute<C>(cur, cur + C::A_BYTES, acc, wm, wn, l);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// Tile index of workgroup `bid` of a tiles_m x tiles_n grid: XCD-aware (the 8 XCDs take workgroups
// round-robin; the bijective remap gives each XCD a contiguous range of tile ids), then grouped by
// GROUP row tiles so the tiles one XCD runs at a time share A and B panels in its L2.
__device__ __forceinline__ void g256_tile(int bid, int nwg, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  constexpr int GROUP = 4;
  const int per_group = GROUP * tiles_n, g = id / per_group, first = g * GROUP;
  const int gsize = min(tiles_m - first, GROUP), in = id - g * per_group;
  tm = first + in % gsize;
  tn = in / gsize;
}

// Accumulator element r of tile (i, j) of wave (wm, wn), lane l: row / column inside the block tile
template <class C>
__device__ __forceinline__ int g256_row(int wm, int i, int r, int l) {
  return wm * C::WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
}
template <class C>
__device__ __forceinline__ int g256_col(int wn, int j, int l) { return wn * C::WTN + j * 32 + (l & 31); }

// ---------------- sources ----------------
// Dense row-major X[rows][ld] bf16 (ld, lims multiples of 8):
//  KC : chunk (mn, k) = X[mn][k .. k+7]     (rows = mn)
//  MNC: chunk (mn, k) = X[k][mn .. mn+7]    (rows = k)
template <bool KC>
struct DenseSrc {
  const uint16_t* x;
  int ld, mn_lim, k_lim;
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return make_rsrc(x, (uint32_t)(KC ? mn_lim : k_lim) * (uint32_t)ld * 2u);
  }
  __device__ __forceinline__ uint32_t off(int mn, int k) const {
    if (!(mn < mn_lim && k < k_lim)) return kBufOOB;
    return KC ? ((uint32_t)mn * (uint32_t)ld + (uint32_t)k) * 2u : ((uint32_t)k * (uint32_t)ld + (uint32_t)mn) * 2u;
  }
};
using DenseKC = DenseSrc<true>;

}  // namespace tfd
