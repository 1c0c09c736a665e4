// 256 x 256 MFMA GEMM core for gfx950: 8 waves, v_mfma_f32_32x32x16_bf16, operands staged global ->
// LDS by the buffer-load-to-LDS DMA (`buffer_load_dwordx4 ... lds`: no VGPR round trip, no ds_write
// pass), two LDS stages (128 KiB), one barrier per 64-deep K step.
//
// Why this shape (csrc/gemm.h is the 128 x 128, 4-wave, 16x16x32, register-staged core):
//  * 256 x 256 with 8 waves (2 x 4, a 128 x 64 output per wave) doubles the FLOP per staged byte of
//    a 128 x 128 tile (128 FLOP/B) -- the LDS image is read 4x less per MFMA;
//  * the 32x32x16 MFMA reads 8 bf16 of A and of B per lane for 32 x 32 x 16 MACs: half the LDS
//    fragment bytes per FLOP of 16x16x32;
//  * the DMA staging frees the VGPRs the register pipeline needed and issues 4x fewer instructions.
//
// Operands are k-contiguous ("KC"): 16-B chunks (mn, k .. k+7). An operand SOURCE maps (mn, k) to a
// byte offset inside its buffer descriptor, or past the descriptor's range when the chunk is out of
// bounds (M / N / K tails, convolution halos), which the hardware range check turns into zeros --
// that is how implicit-GEMM gathers ride the same DMA path:
//   struct Src { __device__ __amdgpu_buffer_rsrc_t rsrc() const;   // from kernel arguments: scalar
//                __device__ uint32_t off(int mn, int k) const; };
//
// LDS image per operand and stage: [256 rows][64 bf16] (128-B rows). The DMA writes lane-linear (one
// wave instruction = 1 KiB = 8 rows), so the bank swizzle is applied to the per-lane SOURCE: 16-B
// slot s of row r holds chunk s ^ ((r >> 1) & 7). A 32x32x16 fragment read (lane l: row l & 31, chunk
// 2 ks + (l >> 5)) then hits 16 distinct bank quads per 16-lane ds_read_b128 group: rows r, r + 1
// differ in the 128-B half of the 256-B bank row, rows r, r + 2, ..., r + 14 in the slot.
#pragma once
#include "common.h"
#include "gemm.h"  // kBufOOB

namespace tfd {

__device__ __forceinline__ f32x16 mfma32x32x16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nbytes, 0x00020000);
}

struct G256 {
  static constexpr int BM = 256, BN = 256, BK = 64, NT = 512, WM = 2, WN = 4;
  static constexpr int OP_BYTES = 256 * BK * 2;       // one operand, one stage: 32 KiB
  static constexpr int STAGE_BYTES = 2 * OP_BYTES;    // A + B
  static constexpr int SMEM = 2 * STAGE_BYTES;        // two stages: 128 KiB
  static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;  // 4 x 2 tiles of 32 x 32 per wave
};

__device__ __forceinline__ int g256_slot(int row, int ch) { return ch ^ ((row >> 1) & 7); }

// DMA one 256-row operand tile (rows mn0 .., k0 .. k0 + 63) into `img`: wave w owns the 8-row groups
// 4w .. 4w + 3, lane l row 8 g + (l >> 3), slot l & 7 (= chunk slot ^ swizzle).
template <class SRC>
__device__ __forceinline__ void g256_stage_op(const SRC& src, char* img, int mn0, int k0, int w, int l) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int grp = w * 4 + i, row = grp * 8 + (l >> 3);
    const int ch = g256_slot(row, l & 7);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(src.rsrc(), (__attribute__((address_space(3))) void*)(img + grp * 1024), 16,
                                             src.off(mn0 + row, k0 + ch * 8), 0, 0, 0);
  }
}

// One 64-deep K step of the wave's 128 x 64 output from the staged images. The fragments of k-sub-step
// ks + 1 are read while ks's 8 MFMAs run (two fragment register sets): with one set the compiler
// waited lgkmcnt(0) before every MFMA pair -- one LDS round trip per 64 MFMA cycles.
__device__ __forceinline__ void g256_frags(const char* As, const char* Bs, int ks, int wm, int wn, int l,
                                           bf16x8 (&a)[G256::TM], bf16x8 (&b)[G256::TN]) {
  const int ch = 2 * ks + (l >> 5);
#pragma unroll
  for (int i = 0; i < G256::TM; ++i) {
    const int row = wm * 128 + i * 32 + (l & 31);
    a[i] = *reinterpret_cast<const bf16x8*>(As + row * 128 + (g256_slot(row, ch) << 4));
  }
#pragma unroll
  for (int j = 0; j < G256::TN; ++j) {
    const int row = wn * 64 + j * 32 + (l & 31);
    b[j] = *reinterpret_cast<const bf16x8*>(Bs + row * 128 + (g256_slot(row, ch) << 4));
  }
}
__device__ __forceinline__ void g256_compute(const char* As, const char* Bs, f32x16 (&acc)[G256::TM][G256::TN], int wm,
                                             int wn, int l) {
  bf16x8 a0[G256::TM], b0[G256::TN], a1[G256::TM], b1[G256::TN];
  g256_frags(As, Bs, 0, wm, wn, l, a0, b0);
#pragma unroll
  for (int ks = 0; ks < G256::BK / 16; ks += 2) {
    g256_frags(As, Bs, ks + 1, wm, wn, l, a1, b1);
#pragma unroll
    for (int i = 0; i < G256::TM; ++i)
#pragma unroll
      for (int j = 0; j < G256::TN; ++j) acc[i][j] = mfma32x32x16(a0[i], b0[j], acc[i][j]);
    if (ks + 2 < G256::BK / 16) g256_frags(As, Bs, ks + 2, wm, wn, l, a0, b0);
#pragma unroll
    for (int i = 0; i < G256::TM; ++i)
#pragma unroll
      for (int j = 0; j < G256::TN; ++j) acc[i][j] = mfma32x32x16(a1[i], b1[j], acc[i][j]);
  }
}

// The K loop over [kbeg, kend) (multiple of 64; sources zero-fill past their K). Stage t + 1's DMA
// is issued before stage t's MFMAs and retired (vmcnt(0) + barrier) after them.
template <class SA, class SB>
__device__ __forceinline__ void g256_mainloop(const SA& sa, const SB& sb, int m0, int n0, int kbeg, int kend, char* smem,
                                              f32x16 (&acc)[G256::TM][G256::TN]) {
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, wm = w / G256::WN, wn = w % G256::WN;
#pragma unroll
  for (int i = 0; i < G256::TM; ++i)
#pragma unroll
    for (int j = 0; j < G256::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = (kend - kbeg + G256::BK - 1) / G256::BK;
  if (nk <= 0) return;
  g256_stage_op(sa, smem, m0, kbeg, w, l);
  g256_stage_op(sb, smem + G256::OP_BYTES, n0, kbeg, w, l);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * G256::STAGE_BYTES;
    if (t + 1 < nk) {
      char* nxt = smem + ((t + 1) & 1) * G256::STAGE_BYTES;
      const int k1 = kbeg + (t + 1) * G256::BK;
      g256_stage_op(sa, nxt, m0, k1, w, l);
      g256_stage_op(sb, nxt + G256::OP_BYTES, n0, k1, w, l);
    }
    g256_compute(cur, cur + G256::OP_BYTES, acc, wm, wn, l);
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

// Accumulator element r of tile (i, j) of wave (wm, wn), lane l: row / column inside the 256 x 256 tile
__device__ __forceinline__ int g256_row(int wm, int i, int r, int l) { return wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }
__device__ __forceinline__ int g256_col(int wn, int j, int l) { return wn * 64 + j * 32 + (l & 31); }

// ---------------- sources ----------------
// Dense row-major X[rows][ld] bf16, chunk (mn, k) = X[mn][k .. k+7] (ld, k_lim multiples of 8)
struct DenseKC {
  const uint16_t* x;
  int ld, mn_lim, k_lim;
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return make_rsrc(x, (uint32_t)mn_lim * (uint32_t)ld * 2u);
  }
  __device__ __forceinline__ uint32_t off(int mn, int k) const {
    return (mn < mn_lim && k < k_lim) ? ((uint32_t)mn * (uint32_t)ld + (uint32_t)k) * 2u : kBufOOB;
  }
};

}  // namespace tfd
