// 3x3 stride-1 pad-1 convolutions (forward, and the stride-1 input gradient, which is the same
// convolution of dY with the 180-degree-rotated, channel-transposed filter) as implicit GEMMs whose A
// operand is staged ONCE per block as an LDS halo tile instead of gathered per K-tile.
//
// The im2col loaders (conv_nhwc.hip FwdA / DgradA) fetch every input element once per tap -- nine
// global (L2) loads and a div/mod address chain per 16-B chunk per K-tile. Here a block owns an
// 8 x 16 output-pixel tile of one image and BN output channels: per 64-channel chunk of the input it
// loads the (8+2) x (16+2) halo once (1440 16-B slots, ~1.4x the tile instead of 9x) into an LDS image
// laid out channel-chunk-major, [8 planes of 8 channels][10 rows][18 cols] x 16 B, and all nine taps'
// A fragments are single ds_read_b128s at (py + r, px + s) of that image: the 16 lanes of a
// fragment's row group are 16 consecutive pixels of one image row, i.e. 16 consecutive 16-B slots of
// one plane (conflict-free). The B operand (weights, one tap x 64 channels x BN per K-step) goes
// through the generic core's LDS tiles (csrc/gemm.h LdsTile / read_frag). The halo of chunk c + 1 is
// loaded at the chunk's first tap and stored at its last, so its latency hides behind eight K-steps.
// The epilogue is the generic LDS-staged one (bf16 out, BN statistics, residual add, BN-backward
// statistics) with a row map from tile rows to output pixels (pixels past the image edge: kNoRow).
//
// Included by csrc/kernels/conv_nhwc.hip inside its anonymous namespace (uses its LdsTile, AddSrc,
// lds_epilogue, rsrc_ld, boff).
#pragma once

struct HaloGeo {
  int N, H, W, Cin, Cout;  // input [N][H][W][Cin] -> output [N][H][W][Cout] (3x3, stride 1, pad 1)
  int tx, ty;              // tiles per image along W and H
  int mtiles;              // N * tx * ty
  uint32_t xbytes, wbytes, ybytes;
};
constexpr int HL_TH = 8, HL_TW = 16;                          // output tile (pixels)
constexpr int HL_HH = HL_TH + 2, HL_HW = HL_TW + 2;           // halo rows / cols
constexpr int HL_PLANE = HL_HH * HL_HW;                       // 180 16-B slots per 8-channel plane
constexpr int HL_CK = 64, HL_NPL = HL_CK / 8;                 // channels per K chunk, planes
constexpr int HL_SLOTS = HL_NPL * HL_PLANE;                   // 1440 slots = 23,040 B per halo image
static_assert(HL_TH * HL_TW == 128, "one 128-row GEMM tile");

__device__ __forceinline__ void halo_tile(const HaloGeo& g, int tile, int& img, int& y0, int& x0) {
  const int per = g.tx * g.ty;
  img = tile / per;
  const int r = tile - img * per, ty = r / g.tx;
  y0 = ty * HL_TH;
  x0 = (r - ty * g.tx) * HL_TW;
}

// GEMM row m = tile * 128 + py * 16 + px -> output pixel row (n, y0 + py, x0 + px), or kNoRow past the
// image edge (the epilogue then neither stores nor sums it)
struct HaloRows {
  HaloGeo g;
  __device__ __forceinline__ uint32_t operator()(int m) const {
    const int tile = m >> 7, lr = m & 127;
    int img, y0, x0;
    halo_tile(g, tile, img, y0, x0);
    const int y = y0 + (lr >> 4), x = x0 + (lr & 15);
    return (y < g.H && x < g.W) ? (uint32_t)((img * g.H + y) * g.W + x) : kNoRow;
  }
};

template <int BN>
struct HaloSmem {
  static constexpr int BYTES_MAIN = 2 * HL_SLOTS * 16 + 2 * LdsTile<BN, HL_CK, false>::ELEMS * 2;
  static constexpr int BYTES_MAIN_KC = 2 * HL_SLOTS * 16 + 2 * LdsTile<BN, HL_CK, true>::ELEMS * 2;
  static constexpr int EPI = LdsEpi<128, BN, 2, 2>::BYTES;
  static constexpr int BYTES = (BYTES_MAIN > BYTES_MAIN_KC ? BYTES_MAIN : BYTES_MAIN_KC) > EPI
                                   ? (BYTES_MAIN > BYTES_MAIN_KC ? BYTES_MAIN : BYTES_MAIN_KC)
                                   : EPI;
};

// DG = false: forward, x = X [N][H][W][Cin], w = HWIO [3][3][Cin][Cout]; B[k][n] = w[tap][k][n] (rows
//             k, n contiguous: the transposed-read LDS tile).
// DG = true : stride-1 input gradient, x = dY [N][H][W][Cin = the conv's K], w = the conv's HWIO filter
//             [3][3][Cout = the conv's C][Cin]; B[k][n] = w[8 - tap][n][k] (k contiguous).
template <int BN, bool DG, bool ADD, bool STATS, class BS>
__global__ __launch_bounds__(256) void conv3x3_halo_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                           uint16_t* __restrict__ y, HaloGeo g, AddSrc add,
                                                           BnPart part, BS bs) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  constexpr int BK = HL_CK, WM = 2, WN = 2, WTN = BN / WN, TM = 4, TN = WTN / 16;
  using TB = LdsTile<BN, BK, DG>;
  static_assert(TB::CHUNKS % 256 == 0, "whole B chunks per thread");
  constexpr int CB = TB::CHUNKS / 256;
  constexpr int HC = (HL_SLOTS + 255) / 256;  // 6 halo slots per thread (the last partly)
  bf16* H0 = reinterpret_cast<bf16*>(smem_raw);
  bf16* H1 = H0 + HL_SLOTS * 8;
  bf16* B0 = H1 + HL_SLOTS * 8;
  bf16* B1 = B0 + TB::ELEMS;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int tile = blockIdx.y, n0 = blockIdx.x * BN;
  int img, y0, x0;
  halo_tile(g, tile, img, y0, x0);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(x, g.xbytes), wr = make_rsrc(w, g.wbytes);

  // this thread's halo slots (plane p, halo pixel (hy, hx)): element offset at channel chunk 0
  uint32_t hoff[HC];
  bool hok[HC];
#pragma unroll
  for (int j = 0; j < HC; ++j) {
    const int i = tid + 256 * j, p = i / HL_PLANE, q = i - p * HL_PLANE, hy = q / HL_HW, hx = q - hy * HL_HW;
    const int gy = y0 - 1 + hy, gx = x0 - 1 + hx;
    hok[j] = i < HL_SLOTS && (unsigned)gy < (unsigned)g.H && (unsigned)gx < (unsigned)g.W;
    hoff[j] = hok[j] ? (uint32_t)((img * g.H + gy) * g.W + gx) * (uint32_t)g.Cin + (uint32_t)(8 * p) : 0u;
  }
  auto hload = [&](int ch, uint4 (&v)[HC]) {
#pragma unroll
    for (int j = 0; j < HC; ++j) v[j] = rsrc_ld(xr, boff(hoff[j] + (uint32_t)(ch * HL_CK), hok[j]));
  };
  auto hstore = [&](bf16* Hs, const uint4 (&v)[HC]) {
#pragma unroll
    for (int j = 0; j < HC; ++j) {
      const int i = tid + 256 * j;
      if (HC * 256 == HL_SLOTS || i < HL_SLOTS) *reinterpret_cast<uint4*>(Hs + i * 8) = v[j];
    }
  };
  auto bload = [&](int step, uint4 (&v)[CB]) {
    const int ch = step / 9, tap = step - ch * 9;
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + 256 * c, row = idx / TB::CH_PER_ROW, col = (idx % TB::CH_PER_ROW) * 8;
      uint32_t e;
      if constexpr (DG) {  // row = n (output channel = the conv's C), col = k
        e = ((uint32_t)(8 - tap) * (uint32_t)g.Cout + (uint32_t)(n0 + row)) * (uint32_t)g.Cin + (uint32_t)(ch * BK + col);
      } else {  // row = k (input channel), col = n
        e = ((uint32_t)tap * (uint32_t)g.Cin + (uint32_t)(ch * BK + row)) * (uint32_t)g.Cout + (uint32_t)(n0 + col);
      }
      v[c] = rsrc_ld(wr, e * 2u);
    }
  };
  auto bstore = [&](bf16* Bs, const uint4 (&v)[CB]) {
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + 256 * c, row = idx / TB::CH_PER_ROW, col = (idx % TB::CH_PER_ROW) * 8;
      *reinterpret_cast<uint4*>(Bs + TB::at(row, col)) = v[c];
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int px = lane & 15, kg = lane >> 4;
  auto compute = [&](const bf16* Hs, const bf16* Bs, int tap) {
    const int r = tap / 3, s = tap - 3 * r;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int slot = (kk / 8 + kg) * HL_PLANE + (4 * wm + i + r) * HL_HW + px + s;
        a[i] = *reinterpret_cast<const bf16x8*>(Hs + slot * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = read_frag<BN, BK, DG>(Bs, wn * WTN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
    }
  };

  const int nch = g.Cin / HL_CK, nsteps = nch * 9;
  uint4 hv[HC], bv[CB];
  hload(0, hv);
  bload(0, bv);
  hstore(H0, hv);
  bstore(B0, bv);
  __syncthreads();
  for (int t = 0; t < nsteps; ++t) {
    const int ch = t / 9, tap = t - ch * 9;
    const bool more = ch + 1 < nch;
    if (t + 1 < nsteps) bload(t + 1, bv);
    if (tap == 0 && more) hload(ch + 1, hv);  // the next chunk's halo rides behind this chunk's 9 taps
    compute((ch & 1) ? H1 : H0, (t & 1) ? B1 : B0, tap);
    if (t + 1 < nsteps) bstore((t & 1) ? B0 : B1, bv);
    if (tap == 8 && more) hstore((ch & 1) ? H0 : H1, hv);
    __syncthreads();
  }
  lds_epilogue<128, BN, WM, WN, ADD, STATS, HaloRows, BS>(acc, smem_raw, y, add, g.mtiles * 128, g.Cout, tile * 128, n0,
                                                          part, HaloRows{g}, g.ybytes, bs);
}
