// Fused CDNA4 kernels for one training step of the reference MNIST CNN
// (conv5x5(32)+relu -> maxpool2 -> conv5x5(64)+relu -> maxpool2 -> FC1024+relu -> dropout -> FC10,
//  softmax-xent mean loss; /root/reference/mnist_python_m.py:93-128, :205).
//
// Kernel map:
//   conv12_fwd_lds   K1+K3+K2+K3 (+K18 batch gather): per (image, conv2 channel half) block, conv1
//                    on the matrix core from a bf16 "5-wide row" x image, bias+relu+2x2 pool+argmax
//                    in registers into a zero-bordered LDS image, then conv2 as a whole-image
//                    implicit GEMM from LDS with the same pooled epilogue.
//   fc1_fwd          K4 (split-K MFMA GEMM, each split's K range in one memory round trip; fp32
//                    slabs, reduced by the head kernel).
//   head_kernel      K4 finish + K5 dropout (Philox) + K6 + K7 + K8(dX) + K9 fused per batch row.
//   fc1_bwd          K8 dW/db + K10 dW (+ bias row) and dX with the MaxPoolGrad + ReluGrad unpool
//                    epilogue (K11), one launch.
//   conv2_bwd_lds    K14 (+K12 bias row) wgrad slabs and K13 dgrad with conv1's relu/pool-mask
//                    epilogue, one launch; the dgrad blocks' tail is K15 (+K12) conv1 wgrad on MFMA.
//   reduce_conv_grads / mnist_adam_kernel  deterministic slab reduction (+ the next batch's gather,
//                    the step bump) / K16 ApplyAdam (one-GPU: with the slab reduction fused).
//   fc_grad_sfb      DP: the fc gradients from all-gathered sufficient factors.
// Each kernel's configuration constants won their A/B on one MI355X (logs: profiles/ab_*.log,
// docs/DESIGN.md); losing arms and timing-only experiments are not kept in the source.
#include "../common.h"

#include "../gemm.h"
#include "../gemm256.h"  // kc_slot, make_rsrc, DenseSrc (the fc1 dX DMA ring)
#include "../mnist_layout.h"
#include "../tfd_kernels.h"

#include <algorithm>
#include <stdexcept>

// Compile-time configuration of the kernels below (each value won its A/B on one MI355X; the losing
// arms and the timing-only experiment switches were removed, logs in profiles/ab_*.log):
constexpr int GEMM_RS = 2;       // register stages of the LDS-staged GEMM core (csrc/gemm.h)
constexpr int FDX_BK_ = 128;     // fc1 dX K-tile
constexpr int FDW_BK_ = 64;      // fc1 dW K-tile
// fc-region Adam: strides per lane with all loads issued up front (1: -0.5 us/step against 2 with the
// round-6 kernels, 4: +0.6; profiles/mnist_conv2_wgrad_grouping_r6.log)
constexpr int ADAM_U = 1;
constexpr int FC1_BK_ = 32;      // one-shot fc1: 14 K-tiles of 32 (140 KiB LDS), 0.6 us/step faster than 7 of 64

namespace tfd {
using namespace mnist;

namespace {

__device__ __forceinline__ int data_row(const int* perm, const int64_t* step, int n_data, int B, int b) {
  if (!perm) return b;
  const int64_t s = *step;
  return perm[(int)((s * (int64_t)B + b) % (int64_t)n_data)];
}
// the batch row b of this step: the prefetched rows[b] when their tag matches the step (the tag, the
// row and the step are three independent loads), else the step -> perm chain
__device__ __forceinline__ int data_row(const MnistStepArgs& a, int b) {
  if (!a.perm) return b;
  if (a.rows) {
    const int tag = a.rows[a.B], r = a.rows[b];
    const int64_t s = *a.step;
    if (tag == (int)s) return r;
    return a.perm[(int)((s * (int64_t)a.B + b) % (int64_t)a.n_data)];
  }
  return data_row(a.perm, a.step, a.n_data, a.B, b);
}
// data_row split in two: the three independent loads (step, tag, prefetched row) issued early, the
// choice (and, on a prefetch miss, the dependent perm load) made where the row is used, so the chain
// costs no wait of its own where it is consumed
struct RowPre {
  int64_t step;
  int tag, row;
};
__device__ __forceinline__ RowPre data_row_pre(const MnistStepArgs& a, int b) {
  RowPre r{0, -1, b};
  if (a.perm) {
    r.step = *a.step;
    if (a.rows) { r.tag = a.rows[a.B]; r.row = a.rows[b]; }
  }
  return r;
}
__device__ __forceinline__ int data_row_use(const MnistStepArgs& a, const RowPre& r, int b) {
  if (!a.perm) return b;
  if (a.rows && r.tag == (int)r.step) return r.row;
  return a.perm[(int)((r.step * (int64_t)a.B + b) % (int64_t)a.n_data)];
}
// gather block b: the batch row b of step `next` into rows / xpre / ypre; block 0 also writes the
// tag (visibility to the next kernel is the kernel boundary)
__device__ __forceinline__ void gather_next(const MnistStepArgs& a, int64_t next, int b) {
  const int row = a.perm[(int)((next * (int64_t)a.B + b) % (int64_t)a.n_data)];
  const f32x4* src = reinterpret_cast<const f32x4*>(a.data + (size_t)row * 784);
  f32x4* dst = reinterpret_cast<f32x4*>(a.xpre + (size_t)b * 784);
  for (int i = threadIdx.x; i < 196; i += blockDim.x) dst[i] = src[i];
  if (threadIdx.x == 0) {
    a.rows[b] = row;
    a.ypre[b] = a.labels[row];
    if (b == 0) a.rows[a.B] = (int)next;
  }
}
__device__ __forceinline__ int gather_blocks(const MnistStepArgs& a) { return (a.perm && a.xpre) ? a.B : 0; }
// the prefetched label of batch row b (speculative load beside the tag and the step)
__device__ __forceinline__ int batch_label(const MnistStepArgs& a, int b) {
  if (a.perm && a.xpre) {
    const int tag = a.rows[a.B], y = a.ypre[b];
    const int64_t s = *a.step;
    if (tag == (int)s) return y;
  }
  return a.labels[data_row(a, b)];
}


// ---------------- K2 layout: conv2 as a whole-image implicit GEMM from LDS ----------------
// Per (image b, output-channel half nh) block, 512 threads (8 waves): 2B blocks (256 at B = 128,
// every CU busy). The image's 14x14x32 bf16 activations sit in a zero-bordered,
// channel-chunk-major LDS image [4 chunks][18 rows][24 cols] x 16 B and the block's half of W2
// as [800 k][32 n + 16] rows; every im2col A fragment is then one ds_read_b128 at
// (pixel(m) + tap offset) -- no global re-reads of the 25x-expanded im2col matrix. Row stride
// 24 px = 8 (mod 16) 16-B slots and 256-B-multiple chunk planes make the pool-window-ordered A
// reads of a 16-lane group hit 16 distinct slots. M = 196 rows in pool-window-major order
// (13 tiles), N = 32 (2 tiles), K = 800 (25 taps x 32 ci = one MFMA k-step per tap). Wave w owns
// M-tiles {w, w + 8} and both N-tiles: per tap 2 B + <= 2 A fragment reads feed <= 4 MFMAs.
// Each lane's 4 accumulator rows are one 2x2 pool window, so bias + relu + maxpool + argmax
// happen in registers. (The per-image block of 64 channels used only 128 CUs at B = 128 and
// staged 129 KB per CU; this split stages 78 KB per CU on all 256.)
constexpr int C2F_W = 24, C2F_PLANE = 18 * C2F_W, C2F_WLD = 48;
// LDS weight rows r = tap*32 + ci (32 bf16 each): groups of 8 rows 384 elements apart, rows 32
// apart inside a group, odd groups shifted by 16 elements. A B-fragment ds_read_b64_tr_b16 has the
// lanes of K-chunks g = 0, 1 reading rows 8g + q (q < 4; the second read q + 4): with a plain
// 96-B pitch rows r and r + 8 share banks (2-way, 3.2 K of the conv2 loop's 5.7 K LDS cycles per
// block); with this layout the 8 rows cover 64 distinct banks (tools/debug/lds_banks.py). Same
// footprint as the plain [800][48] layout.
__device__ __forceinline__ int c2f_wrow(int r) { return (r >> 3) * 384 + (r & 7) * 32 + ((r >> 3) & 1) * 16; }
constexpr int C2F_WTAP = 4 * 384;  // one tap = 32 rows = 4 groups
constexpr int C2F_WR4 = 4 * 32;    // + 4 rows inside a group
static_assert(C2F_WTAP == 32 * C2F_WLD, "the layout keeps the [800][48] footprint");
constexpr int C2L_FWD_SMEM = (4 * C2F_PLANE * 8 + 800 * C2F_WLD) * 2;  // 104448 B
// conv2 forward main loop over the 25 taps: two M-tiles (rows base[0], base[1] of the LDS image) x
// two 16-channel N-tiles. Every wave runs both M-tiles (a second tile past row 196 reads row 0's
// valid LDS address; the epilogue drops it) so there is no exec-masked branch in the loop, and
// tap t + 1's fragments are read while tap t's MFMAs run: with a branch per tile the compiler
// waited lgkmcnt(0) twice per tap, 25 serial LDS round trips (6.2 K cycles of the 24 K-cycle
// conv12 block, s_memtime stamps).
__device__ __forceinline__ void conv2_taps(const bf16* img, const bf16* wcol, const int base[2], f32x4 acc[2][2]) {
  bf16x8 a[2][2], b[2][2];
  auto load = [&](int tap, int slot) {
    const int kh = tap / 5, kw = tap - 5 * kh, toff = (kh * C2F_W + kw) * 8;
    const bf16* wr = wcol + tap * C2F_WTAP;
    b[slot][0] = frag_tr16(wr, wr + C2F_WR4);
    b[slot][1] = frag_tr16(wr + 16, wr + 16 + C2F_WR4);
    a[slot][0] = *reinterpret_cast<const bf16x8*>(img + base[0] + toff);
    a[slot][1] = *reinterpret_cast<const bf16x8*>(img + base[1] + toff);
  };
  load(0, 0);
#pragma unroll
  for (int tap = 0; tap < 25; ++tap) {
    const int cur = tap & 1;
    if (tap + 1 < 25) load(tap + 1, cur ^ 1);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      acc[j][0] = mfma16x16x32(a[cur][j], b[cur][0], acc[j][0]);
      acc[j][1] = mfma16x16x32(a[cur][j], b[cur][1], acc[j][1]);
    }
  }
}
static_assert(C2F_PLANE * 16 % 256 == 0, "chunk planes must be bank-row aligned");

// ---------------- K1+K3+K2+K3 fused: conv1 -> pool -> conv2 -> pool per image, p1 in LDS ----------------
// Block = (image b, conv2 output-channel half nh), 512 threads. conv2 needs all 32 conv1 channels
// of the image, so each half recomputes conv1 (on the matrix core, step 3 below) straight into the
// zero-bordered, channel-chunk-major LDS image conv2 reads; p1 / idx1 still go to global (half 0
// only) for the backward. The conv2 weight half's loads are issued FIRST and stay in flight behind
// the conv1 arithmetic; they are written to LDS after it. One launch and no activation round trip
// between the two convolutions (a separate conv1 kernel + conv2 kernel measured slower).
// LDS: p1 image 27 KiB + W2 half 75 KiB + x / W1 staging + the bf16 "5-wide row" x image.
constexpr int C12_XS = 36;                                  // x image row stride (floats): fewer bank conflicts than 32
constexpr int C12_XR = 60;                                   // rows: 32 (zero-bordered 28 x 28) + 28 zero rows
constexpr int C12_XOFF = C2L_FWD_SMEM;                       // fp32 [C12_XR][C12_XS] x image
constexpr int C12_WOFF = C12_XOFF + C12_XR * C12_XS * 4;     // fp32 [25][32] W1 + [32] bias
constexpr int C12_IOFF = C12_WOFF + (KTAPS * C1 + C1) * 4;   // uint8 [196][32] conv1 argmax
constexpr int C12_X8P = 40;                                  // X8 row pitch (16-B entries): rows oh, oh + 1 of a
                                                             // 16-lane read group land 8 slots apart mod 16 (no overlap)
constexpr int C12_X8OFF = C12_IOFF + 196 * 32;               // bf16x8 [32][C12_X8P] = x[r][c..c+4], 0, 0, 0
constexpr int C12_SMEM = C12_X8OFF + 32 * C12_X8P * 16;     // 143,424 B
static_assert(C12_X8OFF % 16 == 0 && C12_SMEM <= 160 * 1024, "conv12 LDS carve");
static_assert(C12_IOFF % 16 == 0, "LDS carve alignment");
#ifndef TFD_STAMP
#define TFD_STAMP 0  // 1: thread 0 of every conv12 block records s_memtime at its phase boundaries
#endif
#define C12_STAMP(k)                                                                       \
  do {                                                                                     \
    if (TFD_STAMP && a.dbg && threadIdx.x == 0) a.dbg[blockIdx.x * 16 + (k)] = (int64_t)__builtin_amdgcn_s_memtime(); \
  } while (0)
// the same from wave 4 (the x / W1 loader), slots 8..15
#define C12_STAMPW(k)                                                                      \
  do {                                                                                     \
    if (TFD_STAMP && a.dbg && threadIdx.x == 256) a.dbg[blockIdx.x * 16 + 8 + (k)] = (int64_t)__builtin_amdgcn_s_memtime(); \
  } while (0)
__global__ __launch_bounds__(512) void conv12_fwd_lds(MnistStepArgs a) {
  C12_STAMP(0);
  C12_STAMPW(0);
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* img = (bf16*)smem_raw;                        // [4][18*24][8]  (conv2 input = pooled conv1)
  bf16* wt = img + 4 * C2F_PLANE * 8;                 // [800][48]
  float* xs = reinterpret_cast<float*>(smem_raw + C12_XOFF);
  float* w1 = reinterpret_cast<float*>(smem_raw + C12_WOFF);
  const int b = blockIdx.x >> 1, nh = blockIdx.x & 1, t = threadIdx.x;
  // 1. wave specialisation of the loads (a wave's vmcnt is in-order, so a load issued behind the
  //    W2 loads could not be consumed before them): waves 0-3 issue the conv2 weight half (12.5 x
  //    16 B per lane, written to LDS only after conv1); waves 4-7 the W1 / bias and the x image
  //    (prefetched row -> x) that conv1 needs first. Both overlap the LDS zeroing.
  const uint16_t* wsrc = a.pbf + OFF_WC2 + nh * 32;
  const int rot = (int)((blockIdx.x * 1031u) % 3200u);  // per-block start: spread L2 channels
  constexpr int NW = (3200 + 255) / 256;
  uint4 vw[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) vw[j] = zero4();  // defined on both roles' paths (else kept in scratch)
  f32x4 xv = f32x4{0.f, 0.f, 0.f, 0.f}, w1v = f32x4{0.f, 0.f, 0.f, 0.f};
  const int u = t - 256;
  // Every load below is unconditional (indices clamped; the LDS stores keep the bounds) and the wave
  // roles branch on a scalar: exec-masked loads merged by a phi made the compiler wait for a load of
  // the other role's path (waves 0-3 for their first W2 chunk, waves 4-7 for W1 before issuing the x
  // image) before the first barrier.
  const bool w2_role = __builtin_amdgcn_readfirstlane(t >> 6) < 4;
  if (w2_role) {
    const int tw = t & 255;  // this role's threads are 0..255 (lets the compiler fold j < NW - 1)
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const int e = tw + 256 * j, i = (min(e, 3199) + rot) % 3200;  // the last chunk of lanes >= 128: a
      vw[j] = *reinterpret_cast<const uint4*>(wsrc + (i >> 2) * 64 + (i & 3) * 8);  // duplicate, never stored
    }
  } else {
    const int uw = min(u, (KTAPS * C1 + C1) / 4 - 1), ux = min(u, 195);
    w1v = reinterpret_cast<const f32x4*>(a.p32 + OFF_WC1)[uw];
    // the prefetched image, loaded speculatively beside its tag and the step
    bool hit = false;
    if (a.perm && a.xpre) {
      xv = reinterpret_cast<const f32x4*>(a.xpre + (size_t)b * 784)[ux];
      hit = a.rows[a.B] == (int)*a.step;
    }
    if (!hit) {
      const float* x = a.data + (size_t)data_row(a, b) * 784;
      xv = reinterpret_cast<const f32x4*>(x)[ux];
    }
  }
  C12_STAMP(1);
  C12_STAMPW(1);
#if TFD_STAMP
  if (t == 256) {  // when wave 4's loads have landed (stamp only; the data wait happens anyway below)
    __builtin_amdgcn_s_waitcnt(0);
    C12_STAMPW(2);
  }
#endif
  // 2. zero the x image border and the p1 image (its border is conv2's SAME padding), then x, W1
  for (int i = t; i < C12_XR * C12_XS / 4; i += 512) reinterpret_cast<f32x4*>(xs)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = t; i < 4 * C2F_PLANE; i += 512) reinterpret_cast<uint4*>(img)[i] = zero4();
  C12_STAMPW(3);
  __syncthreads();
  C12_STAMPW(4);
  if (t >= 256) {
    if (u < (KTAPS * C1 + C1) / 4) reinterpret_cast<f32x4*>(w1)[u] = w1v;
    if (u < 196) {
      const int r = (4 * u) / 28, c = (4 * u) % 28;
      float* d = xs + (r + 2) * C12_XS + c + 2;
      d[0] = xv[0]; d[1] = xv[1]; d[2] = xv[2]; d[3] = xv[3];
    }
  }
  C12_STAMPW(5);
  __syncthreads();
  // the "5-wide row" image: X8[r][c] = bf16(x[r][c .. c+4]) and three zeros (zero-bordered 32 x 32
  // coordinates, c <= 27), so the 8 taps (kh, kw = 0..7) of one kernel row are one 16-B LDS read
  {
    bf16* x8 = reinterpret_cast<bf16*>(smem_raw + C12_X8OFF);
    for (int i = t; i < 32 * 28; i += 512) {
      const int r = i / 28, c = i - r * 28;
      const float* src = xs + r * C12_XS + c;
      bf16x8 e;
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = (bf16)(j < 5 ? src[j] : 0.f);
      *reinterpret_cast<bf16x8*>(x8 + (r * C12_X8P + c) * 8) = e;
    }
    __syncthreads();
  }
  C12_STAMP(2);
  C12_STAMPW(6);
  // 3. conv1 on the matrix core: implicit GEMM M = 784 pixels (pool-window-major, m = pp*4 + win),
  //    N = 32 channels, K = 25 taps padded to 32 -> one v_mfma_f32_16x16x32_bf16 per (M-tile, N-tile);
  //    each lane's 4 accumulator rows are one 2x2 window, so bias + relu + max + argmax happen in
  //    registers. Operands: the x image and W1 rounded to bf16 (the bf16 engine's operand precision;
  //    --dtype fp32 keeps conv1 exact). Wave w owns M-tiles w, w + 8, ... (<= 7): all of its A
  //    fragments are gathered first, then the MFMAs, then the epilogues (no per-tile
  //    LDS -> MFMA -> epilogue latency chain). Pooled values go to the conv2 LDS image, argmax bytes
  //    to an LDS array; both are copied out to global with 16-B stores afterwards (half 0 only).
  {
    const int lane = t & 63, w = t >> 6, g = lane >> 4, col = lane & 15;
    uint8_t* idx_l = reinterpret_cast<uint8_t*>(smem_raw + C12_IOFF);  // [196][32]
    const float bias0 = w1[KTAPS * C1 + col], bias1 = w1[KTAPS * C1 + 16 + col];
    constexpr int MT = 7;  // ceil(49 / 8)
    // K = kernel row kh * 8 + kw (kw < 5 real): MFMA 1 covers kh = 0..3 (lane group g reads kernel
    // row g: one 16-B read of X8), MFMA 2 kh = 4 (every group reads row 4; only group 0's weights
    // are non-zero). 2 MFMAs + 2 ds_read_b128 per M-tile instead of 8 scalar reads + 8 converts.
    bf16x8 bw1[2], bw2[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {  // row 4 read by every lane group, zeroed by a select (an
        // exec-masked read per element was 10 serial LDS round trips, each with lgkmcnt(0))
        const float r4 = jj < 5 ? w1[(20 + jj) * C1 + nt * 16 + col] : 0.f;
        bw1[nt][jj] = (bf16)(jj < 5 ? w1[(g * 5 + jj) * C1 + nt * 16 + col] : 0.f);
        bw2[nt][jj] = (bf16)(g == 0 ? r4 : 0.f);
      }
    const bf16* x8 = reinterpret_cast<const bf16*>(smem_raw + C12_X8OFF);
    bf16x8 af[MT], af2[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int mt = w + 8 * i;
      const int m = min(mt, 48) * 16 + col, pp = m >> 2, win = m & 3;
      const int orow = 2 * (pp / 14) + (win >> 1), ocol = 2 * (pp % 14) + (win & 1);
      af[i] = *reinterpret_cast<const bf16x8*>(x8 + ((orow + g) * C12_X8P + ocol) * 8);
      af2[i] = *reinterpret_cast<const bf16x8*>(x8 + ((orow + 4) * C12_X8P + ocol) * 8);
    }
    f32x4 z[MT][2];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        z[i][nt] = mfma16x16x32(af2[i], bw2[nt], mfma16x16x32(af[i], bw1[nt], f32x4{0.f, 0.f, 0.f, 0.f}));
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int mt = w + 8 * i;
      if (mt >= 49) break;
      const int pq = mt * 4 + g, ph = pq / 14, pw = pq - ph * 14;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int n = nt * 16 + col;
        const float bias = nt ? bias1 : bias0;
        float mx = z[i][nt][0] + bias;
        int am = 0;
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          const float zz = z[i][nt][r] + bias;
          if (zz > mx) { mx = zz; am = r; }
        }
        reinterpret_cast<uint16_t*>(img)[((n >> 3) * C2F_PLANE + (ph + 2) * C2F_W + pw + 2) * 8 + (n & 7)] =
            f2bf_bits(fmaxf(mx, 0.f));
        idx_l[pq * 32 + n] = (uint8_t)am;
      }
    }
  }
  C12_STAMP(3);
  // 4. the W2 half (landed during conv1) into LDS
  if (w2_role) {
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const int i = (t + 256 * j + rot) % 3200;
      if (t + 256 * j < 3200) *reinterpret_cast<uint4*>(wt + c2f_wrow(i >> 2) + (i & 3) * 8) = vw[j];
    }
  }
  __syncthreads();
  if (nh == 0) {  // p1 / idx1 for the backward: 16-B stores from the LDS image and argmax array
    const uint8_t* idx_l = reinterpret_cast<const uint8_t*>(smem_raw + C12_IOFF);
    for (int i = t; i < 196 * 4; i += 512) {
      const int pq = i >> 2, cg = i & 3, ph = pq / 14, pw = pq - ph * 14;
      *reinterpret_cast<uint4*>(a.p1 + ((size_t)b * 196 + pq) * 32 + cg * 8) =
          *reinterpret_cast<const uint4*>(img + (cg * C2F_PLANE + (ph + 2) * C2F_W + pw + 2) * 8);
    }
    for (int i = t; i < 196 * 2; i += 512)
      reinterpret_cast<uint4*>(a.idx1 + (size_t)b * 196 * 32)[i] = reinterpret_cast<const uint4*>(idx_l)[i];
  }
  C12_STAMP(4);
  // 5. conv2 implicit GEMM + bias + relu + pool + argmax (conv2_fwd_lds's main loop and epilogue)
  const int lane = t & 63, w = t >> 6, g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  const int nmt = (w + 8 < 13) ? 2 : 1;
  int base[2];
  f32x4 acc[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    acc[j][0] = acc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int m = (w + 8 * j) * 16 + (lane & 15);
    int px = 0;
    if (m < 196) {
      const int pp = m >> 2, win = m & 3;
      px = (2 * (pp / 7) + (win >> 1)) * C2F_W + 2 * (pp % 7) + (win & 1);
    }
    base[j] = (g * C2F_PLANE + px) * 8;
  }
  const bf16* wcol = wt + c2f_wrow(8 * g + q) + 4 * p4;  // rows tap*32 + 8g + q (+4)
  // the conv2 bias loads before the K loop (in the epilogue they were one more memory round trip
  // after the last MFMA)
  float bbv[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) bbv[nt] = a.p32[OFF_BC2 + nh * 32 + nt * 16 + (lane & 15)];
  conv2_taps(img, wcol, base, acc);
  C12_STAMP(5);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n = nh * 32 + nt * 16 + (lane & 15);
    const float bb = bbv[nt];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m4 = (w + 8 * j) * 16 + 4 * g;
      if (j >= nmt || m4 >= 196) continue;
      float mx = acc[j][nt][0] + bb;
      int am = 0;
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        const float z = acc[j][nt][r] + bb;
        if (z > mx) { mx = z; am = r; }
      }
      const size_t o = (size_t)b * FEAT + (m4 >> 2) * 64 + n;
      a.p2[o] = f2bf_bits(fmaxf(mx, 0.f));
      a.idx2[o] = (uint8_t)am;
    }
  }
  C12_STAMP(6);
}

// ---------------- K3: fc1 forward, split-K slabs ----------------
struct SlabEpi {
  float* __restrict__ out;
  int ld, M, N;
  __device__ __forceinline__ void operator()(int m4, int n, f32x4 v) const {
    if (n >= N) return;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (m4 + r < M) out[(size_t)(m4 + r) * ld + n] = v[r];
  }
};
constexpr int FC1_BM = 64, FC1_BN = 64, FC1_BK = FC1_BK_;
constexpr int FC1_SPLITS = 7;  // 3136 = 7 * 448; each split's whole K range in one round trip (14: +0.5 us)
constexpr int FC1_NKT = FEAT / FC1_SPLITS / FC1_BK;  // K-tiles per split
static_assert(FC1_NKT * FC1_BK * FC1_SPLITS == FEAT, "fc1 split-K must tile K exactly");
__global__ __launch_bounds__(256) void fc1_fwd(MnistStepArgs a, int kper) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  static_assert(FEAT % 8 == 0 && HID % 8 == 0, "whole chunks (DenseLoaderX)");
  DenseLoaderX<true> la{a.p2, FEAT, a.B, FEAT};
  DenseLoaderX<false> lb{a.pbf + OFF_WD1, HID, HID, FEAT};
  const int z = blockIdx.z;
  SlabEpi epi{a.fc1_slab + (size_t)z * a.B * HID, HID, a.B, HID};
  const int kb = z * kper;
  gemm_block_oneshot<FC1_BM, FC1_BN, FC1_BK, FC1_NKT, 2, 2>(la, lb, epi, blockIdx.y * FC1_BM, blockIdx.x * FC1_BN, kb, (bf16*)smem_raw);
}

// ---------------- K4-K9 head: reduce slabs, bias, relu, dropout, FC10, softmax-xent, bwd ----------
// One 256-thread block per batch row; thread t owns hidden units 4t..4t+3.
#define HEAD_STAMP(k)                                                                                    \
  do {                                                                                                   \
    if (TFD_STAMP && a.dbg && threadIdx.x == 0) a.dbg[4 * a.B * 8 + blockIdx.x * 8 + (k)] = (int64_t)__builtin_amdgcn_s_memtime(); \
  } while (0)
__global__ __launch_bounds__(256) void head_kernel(MnistStepArgs a, int train) {
  HEAD_STAMP(0);
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n0 = 4 * t;
  // Every operand that does not depend on the label is requested first, in one memory round trip:
  // the split-K slabs, the fc1 bias, this thread's 4 x 10 output-layer weights (160 contiguous bytes)
  // and the output bias. Then the label chain (step -> tag / prefetched label, or step -> perm ->
  // label): uniform addresses with no store before them in the kernel, so they are scalar loads that
  // run beside the vector loads (issued first, the chain's branches held the slab loads back by three
  // round trips, and the t_out store in front of it made every later load a vector load).
  f32x4 p[FC1_SPLITS];
#pragma unroll
  for (int s = 0; s < FC1_SPLITS; ++s) p[s] = *reinterpret_cast<const f32x4*>(a.fc1_slab + ((size_t)s * a.B + row) * HID + n0);
  f32x4 wo[NCLS];
#pragma unroll
  for (int q = 0; q < NCLS; ++q) wo[q] = reinterpret_cast<const f32x4*>(a.p32 + OFF_OUT + (size_t)n0 * NCLS)[q];
#define HEAD_W(j, c) wo[((j) * NCLS + (c)) >> 2][((j) * NCLS + (c)) & 3]
  float bout[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) bout[c] = a.p32[OFF_BOUT + c];
  f32x4 h = *reinterpret_cast<const f32x4*>(a.p32 + OFF_BD1 + n0);
  const int64_t st = *a.step;
  const int lbl = batch_label(a, row);
  if (a.t_out && row == 0 && t == 0) *a.t_out = st + 1;
#pragma unroll
  for (int s = 0; s < FC1_SPLITS; ++s) h += p[s];
  HEAD_STAMP(1);
  float hd[4], scale[4];
  const float kp = train ? a.keep_prob : 1.0f;
  if (kp < 1.0f) {
    Philox4 r = philox4x32_10((uint32_t)(row * 256 + t), (uint32_t)st, (uint32_t)(st >> 32), a.rank, a.seed,
                              0x5EED1234u);
#pragma unroll
    for (int j = 0; j < 4; ++j) scale[j] = (u01(r.v[j]) < kp) ? (1.0f / kp) : 0.f;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) scale[j] = 1.f;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) hd[j] = fmaxf(h[j], 0.f) * scale[j];
  // logits partials
  float lp[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) lp[c] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int c = 0; c < NCLS; ++c) lp[c] = fmaf(hd[j], HEAD_W(j, c), lp[c]);
  }
  HEAD_STAMP(2);
  __shared__ float red[4][NCLS];
  // DPP wave sums (quad swaps, row shifts, row broadcasts: no LDS round trips) of the 10 partials,
  // interleaved; the wave total lands in lane 63
  wave_sums_to_lane63(lp);
  if (lane == 63) {
#pragma unroll
    for (int c = 0; c < NCLS; ++c) red[wv][c] = lp[c];
  }
  __syncthreads();
  float logit[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) logit[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c] + bout[c];
  float mx = logit[0];
  int am = 0;
#pragma unroll
  for (int c = 1; c < NCLS; ++c)
    if (logit[c] > mx) { mx = logit[c]; am = c; }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < NCLS; ++c) se += __expf(logit[c] - mx);
  const float lse = mx + __logf(se);
  HEAD_STAMP(3);
  if (t == 0) {
    a.loss_row[row] = lse - logit[lbl];
    a.correct_row[row] = (am == lbl) ? 1.f : 0.f;
  }
  if (!train) return;
  const float invB = 1.0f / (float)a.B;
  float dl[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) dl[c] = (__expf(logit[c] - lse) - (c == lbl ? 1.f : 0.f)) * invB;
#pragma unroll
  for (int c = 0; c < NCLS; ++c)
    if (t == c) a.dlogits[row * NCLS + c] = dl[c];
  uint32_t hdw[2], dhw[2];
  float dhv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < NCLS; ++c) d = fmaf(dl[c], HEAD_W(j, c), d);
    dhv[j] = (h[j] > 0.f) ? d * scale[j] : 0.f;
  }
#undef HEAD_W
  hdw[0] = pack_bf2(hd[0], hd[1]); hdw[1] = pack_bf2(hd[2], hd[3]);
  dhw[0] = pack_bf2(dhv[0], dhv[1]); dhw[1] = pack_bf2(dhv[2], dhv[3]);
  *reinterpret_cast<uint2*>(a.hd + (size_t)row * HID + n0) = make_uint2(hdw[0], hdw[1]);
  *reinterpret_cast<uint2*>(a.dh + (size_t)row * HID + n0) = make_uint2(dhw[0], dhw[1]);
  HEAD_STAMP(4);
}

// ---------------- K8 output layer dW/db: [1025][10] = [Hd;1]^T dlogits ----------------
// One 256-thread block owns 64 rows m (thread = row m0 + (t & 63), batch quarter t >> 6); dlogits
// [B][10] staged in LDS; the 4 batch quarters are summed through LDS (deterministic).
constexpr int OUTG_ROWS = 64;
constexpr int OUTG_BLOCKS = (HID + 1 + OUTG_ROWS - 1) / OUTG_ROWS;  // 17 (last block: bias row)
constexpr int OUTG_LB = 16; // hd loads batched per thread (a one-at-a-time loop was a 32-deep latency chain)
__device__ __forceinline__ void out_grad_block(const MnistStepArgs& a, int blk, float* smem) {
  float* dl = smem;                      // [B][10]
  float* part = smem + a.B * NCLS;       // [4][64][10]
  const int t = threadIdx.x, r = t & 63, q = t >> 6;
  for (int i = t; i < a.B * NCLS; i += 256) dl[i] = a.dlogits[i];
  __syncthreads();
  const int m = blk * OUTG_ROWS + r;
  float acc[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) acc[c] = 0.f;
  const int bq = (a.B + 3) >> 2, b0 = q * bq, b1 = min(a.B, b0 + bq);
  if (m < HID) {
    int b = b0;
    for (; b + OUTG_LB <= b1; b += OUTG_LB) {  // OUTG_LB independent loads in flight, then the FMAs
      float hv[OUTG_LB];
#pragma unroll
      for (int u = 0; u < OUTG_LB; ++u) hv[u] = bf2f(a.hd[(size_t)(b + u) * HID + m]);
#pragma unroll
      for (int u = 0; u < OUTG_LB; ++u)
#pragma unroll
        for (int c = 0; c < NCLS; ++c) acc[c] = fmaf(hv[u], dl[(b + u) * NCLS + c], acc[c]);
    }
    for (; b < b1; ++b) {
      const float h = bf2f(a.hd[(size_t)b * HID + m]);
#pragma unroll
      for (int c = 0; c < NCLS; ++c) acc[c] = fmaf(h, dl[b * NCLS + c], acc[c]);
    }
  } else if (m == HID) {
    for (int b = b0; b < b1; ++b)
#pragma unroll
      for (int c = 0; c < NCLS; ++c) acc[c] += dl[b * NCLS + c];
  }
#pragma unroll
  for (int c = 0; c < NCLS; ++c) part[(q * 64 + r) * NCLS + c] = acc[c];
  __syncthreads();
  for (int i = t; i < OUTG_ROWS * NCLS; i += 256) {
    const int rr = i / NCLS, mm = blk * OUTG_ROWS + rr;
    if (mm <= HID) {
      const size_t o = OFF_OUT + (size_t)mm * NCLS + (i - rr * NCLS);
      const float g =
          part[i] + part[OUTG_ROWS * NCLS + i] + part[2 * OUTG_ROWS * NCLS + i] + part[3 * OUTG_ROWS * NCLS + i];
      if (a.gbf_a) {
        a.gbf_a[o] = f2bf_bits(g);
      } else {
        a.grad[o] = g;
      }
    }
  }
}

// ---------------- K10 fc1 dW (+bias row): [3137][1024] = [P2;1]^T dH ----------------
// fp32 into the flat gradient buffer, or (bf16 wire format) bf16 straight into the all-reduce /
// optimizer operand -- the rounding a separate cast pass would do.
// [P2_all; 1]^T as the KC = false A operand: (mn, k) = P2_all[k][mn] for mn < 3136, the bias
// "ones row" at mn == 3136 (a chunk {1, 0, ..., 0}), zeros past K.
struct OnesRowBuf {
  static constexpr bool KC = false;
  const uint16_t* __restrict__ x;
  int k_lim;
  uint32_t nbytes;
  __device__ __forceinline__ uint4 operator()(int mn, int k) const {
    const uint4 v = buf_ld(x, nbytes, (uint32_t)k * FEAT + mn, k < k_lim && mn < FEAT);
    return (mn == FEAT && k < k_lim) ? make_uint4(0x3F80u, 0u, 0u, 0u) : v;
  }
};
static_assert(FEAT % 8 == 0, "the ones row starts a fresh 8-element chunk");

constexpr int FDW_BM = 64, FDW_BN = 64, FDW_BK = FDW_BK_;
// fc1 dW tile epilogue through LDS: the fp32 accumulators go to a [64][68] float image, then every
// thread stores whole 16-B pieces of rows (8 bf16, or 4 fp32 twice) -- a wave writes 1 KiB of row
// bytes per instruction. The round-3 fragment-order epilogue wrote 2-B (4-B) scalars in 32-B row
// pieces per instruction: 6.4 MB of bf16 gradient as 200 K partial-line writes per step.
constexpr int FDW_PITCH = FDW_BN + 4;
__device__ __forceinline__ void fc1_dw_store(f32x4 (&acc)[2][2], float* cs, float* out, uint16_t* outbf, int m0,
                                             int n0, int M) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cs[(wm * 32 + 16 * i + 4 * (lane >> 4) + r) * FDW_PITCH + wn * 32 + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
#pragma unroll
  for (int q = tid; q < FDW_BM * FDW_BN / 8; q += 256) {
    const int row = q >> 3, ch = q & 7, m = m0 + row;
    if (m >= M) continue;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(cs + row * FDW_PITCH + ch * 8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(cs + row * FDW_PITCH + ch * 8 + 4);
    const size_t o = (size_t)m * HID + n0 + ch * 8;
    if (outbf) {
      *reinterpret_cast<uint4*>(outbf + o) =
          make_uint4(pack_bf2(lo[0], lo[1]), pack_bf2(lo[2], lo[3]), pack_bf2(hi[0], hi[1]), pack_bf2(hi[2], hi[3]));
    } else {
      *reinterpret_cast<f32x4*>(out + o) = lo;
      *reinterpret_cast<f32x4*>(out + o + 4) = hi;
    }
  }
}
template <class LA, class LB>
__device__ __forceinline__ void fc1_dw_tile(const MnistStepArgs& a, const LA& la, const LB& lb, int m0, int n0, int K,
                                            bf16* smem) {
  f32x4 acc[2][2];
  gemm_mainloop<FDW_BM, FDW_BN, FDW_BK, 2, 2, LA, LB, GEMM_RS>(la, lb, m0, n0, 0, K, smem, acc);  // ends with a barrier
  fc1_dw_store(acc, reinterpret_cast<float*>(smem), a.grad + OFF_WD1, a.gbf_a ? a.gbf_a + OFF_WD1 : nullptr, m0, n0,
               FEAT + 1);
}
__device__ __forceinline__ void fc1_dw_block(const MnistStepArgs& a, int bx, int by, bf16* smem) {
  OnesRowBuf la{a.p2, a.B, (uint32_t)((int64_t)a.B * FEAT * 2)};
  DenseLoaderX<false> lb{a.dh, HID, HID, a.B};
  fc1_dw_tile(a, la, lb, by * FDW_BM, bx * FDW_BN, a.B, smem);
}

// ---------------- K10 fc1 dX + K11 MaxPoolGrad + ReluGrad -> dz2 (dense, conv2 pre-act grad) --------
// dX tile = BM batch rows x BN features of ONE pooled pixel pp (a 64-wide tile is all 64 channels,
// a 32-wide one half of them). Epilogue through LDS: the fp32 tile goes to a [BM][BN + 4] float
// image; thread (row b, 8-channel chunk cc) loads p2 (relu output, 16 B) and idx2 (argmax, 8 B)
// chunks once, forms g = p2 > 0 ? dX : 0 in bf16, and writes the 2x2 unpool window as four whole
// 16-B chunks of dz2 rows (the argmax position gets g, the other three zeros). The fragment-order
// epilogue it replaces made 16 scattered 2-B stores and 1-2 B loads per lane and value group.
constexpr int FDX_BM = 32, FDX_BN = 64, FDX_BK = FDX_BK_, FDX_BN2 = 32;
template <int BN>
__device__ __forceinline__ void fc1_dx_unpool_store(const MnistStepArgs& a, f32x4 (&acc)[FDX_BM / 32][BN / 32],
                                                    float* cs, int m0, int n0) {
  constexpr int PITCH = BN + 4, CPR = BN / 8;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  constexpr int WTM = FDX_BM / 2, WTN = BN / 2;
  const int b = tid / CPR, cc = tid % CPR, m = m0 + b;
  const bool live = b < FDX_BM && m < a.B;
  // the relu / argmax chunks are issued before the accumulator is staged
  const size_t xo = (size_t)(live ? m : 0) * FEAT + n0 + cc * 8;
  const uint4 pv = *reinterpret_cast<const uint4*>(a.p2 + xo);
  const uint2 iv = *reinterpret_cast<const uint2*>(a.idx2 + xo);
#pragma unroll
  for (int i = 0; i < WTM / 16; ++i)
#pragma unroll
    for (int j = 0; j < WTN / 16; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cs[(wm * WTM + 16 * i + 4 * (lane >> 4) + r) * PITCH + wn * WTN + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  if (!live) return;
  const f32x4 lo = *reinterpret_cast<const f32x4*>(cs + b * PITCH + cc * 8);
  const f32x4 hi = *reinterpret_cast<const f32x4*>(cs + b * PITCH + cc * 8 + 4);
  const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
  uint32_t g[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t p = (pw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
    g[j] = p != 0 ? (uint32_t)f2bf_bits(v[j]) : 0u;  // relu output > 0 (it is >= 0)
  }
  const int pp = n0 >> 6, c0 = (n0 & 63) + cc * 8, ph = pp / 7, pwx = pp - ph * 7;
  const uint32_t iw[2] = {iv.x, iv.y};
#pragma unroll
  for (int wi = 0; wi < 4; ++wi) {
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t i0 = (iw[q >> 1] >> (16 * (q & 1))) & 0xFFu, i1 = (iw[q >> 1] >> (16 * (q & 1) + 8)) & 0xFFu;
      o[q] = (i0 == (uint32_t)wi ? g[2 * q] : 0u) | (i1 == (uint32_t)wi ? g[2 * q + 1] << 16 : 0u);
    }
    const int oh = 2 * ph + (wi >> 1), ow = 2 * pwx + (wi & 1);
    *reinterpret_cast<uint4*>(a.dz2 + ((size_t)(m * 14 + oh) * 14 + ow) * 64 + c0) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}
// fc1 dX tile width: 64 (196 blocks at B = 128) inside the fused fc backward, where the dX tiles
// share the launch with ~800 dW tiles (fc1_dx_block_dma); 32 (392 blocks) when dX runs alone (DP
// step, part 2: the register pipeline below), where 196 blocks left a quarter of the CUs idle (A/B:
// one GPU 64 better by 1.3 us, DP 32 better by 1.5). Register stages of the dX-alone blocks: 2
// (-0.3 us, profiles/ab_fc1_dx_tiles_r2.log)
constexpr int FDX_RS = 1, FDX_RS_ALONE = 2;
// fc1 dX inside the fused fc backward: K = 1024 as 16 steps of 64 on a 4-stage LDS ring filled by
// the buffer-load-to-LDS DMA (3 stages in flight behind the MFMAs, no VGPR staging). With the register
// pipeline (gemm_mainloop, BK 128, RS 1) every one of 8 K steps waited a full memory round trip:
// fc1 dX alone measured 10.3 us for 0.82 GFLOP over a 6.4 MB W1 (profiles/diag_fc1bwd_conv2bwd_r3.txt).
// LDS images: KC [rows][64 bf16], slot s of row r holds chunk s ^ ((r >> 1) & 7) (kc_slot: the 16 rows
// of a 16x16x32 fragment read hit 16 distinct 16-B bank groups). Waves: 2 x 2 of 16 x 32 outputs.
constexpr int FDXD_BK = 64, FDXD_S = 4;
constexpr int FDXD_A = FDX_BM * FDXD_BK * 2, FDXD_B = FDX_BN * FDXD_BK * 2, FDXD_STAGE = FDXD_A + FDXD_B;
constexpr int FDXD_SMEM = FDXD_S * FDXD_STAGE;  // 48 KiB
constexpr int FDXD_NK = HID / FDXD_BK;
static_assert(FDX_BM == 32 && FDX_BN == 64 && FDXD_NK >= FDXD_S, "fc1 dX DMA ring geometry");
__device__ __forceinline__ void fdxd_stage(const DenseKC& sa, const DenseKC& sb, char* img, int m0, int n0, int k0,
                                           int w, int l) {
#if defined(__HIP_DEVICE_COMPILE__)
  {  // A: 32 rows = 4 wave instructions (one per wave)
    const int row = w * 8 + (l >> 3);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(sa.rsrc(), (__attribute__((address_space(3))) void*)(img + w * 1024), 16,
                                             sa.off(m0 + row, k0 + kc_slot(row, l & 7) * 8), 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // B: 64 rows = 8 wave instructions (two per wave)
    const int ins = 2 * w + i, row = ins * 8 + (l >> 3);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(sb.rsrc(), (__attribute__((address_space(3))) void*)(img + FDXD_A + ins * 1024),
                                             16, sb.off(n0 + row, k0 + kc_slot(row, l & 7) * 8), 0, 0, 0);
  }
#else
  (void)sa; (void)sb; (void)img; (void)m0; (void)n0; (void)k0; (void)w; (void)l;
#endif
}
__device__ __forceinline__ void fc1_dx_block_dma(const MnistStepArgs& a, int bx, int by, char* smem) {
  const DenseKC sa{a.dh, HID, a.B, HID};
  const DenseKC sb{a.pbf + OFF_WD1, HID, FEAT, HID};
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = by * FDX_BM, n0 = bx * FDX_BN;
  f32x4 acc[1][2] = {{f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}}};
#pragma unroll
  for (int s = 0; s < FDXD_S - 1; ++s) fdxd_stage(sa, sb, smem + s * FDXD_STAGE, m0, n0, s * FDXD_BK, w, l);
  for (int t = 0; t < FDXD_NK; ++t) {
    // stage t has landed once at most the stages issued after it (3 wave instructions each) are pending
    const int after = min(FDXD_S - 2, FDXD_NK - 1 - t);
    if (after == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage t visible to every wave; every wave is done with stage t - 1's slot
    if (t + FDXD_S - 1 < FDXD_NK)
      fdxd_stage(sa, sb, smem + ((t + FDXD_S - 1) % FDXD_S) * FDXD_STAGE, m0, n0, (t + FDXD_S - 1) * FDXD_BK, w, l);
    const char* As = smem + (t % FDXD_S) * FDXD_STAGE;
    const char* Bs = As + FDXD_A;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = 4 * ks + (l >> 4);
      const int ra = 16 * wm + (l & 15);
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + ra * 128 + (kc_slot(ra, ch) << 4));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int rb = 32 * wn + 16 * j + (l & 15);
        const bf16x8 bf = *reinterpret_cast<const bf16x8*>(Bs + rb * 128 + (kc_slot(rb, ch) << 4));
        acc[0][j] = mfma16x16x32(af, bf, acc[0][j]);
      }
    }
  }
  __syncthreads();  // the ring is dead: the epilogue reuses it
  fc1_dx_unpool_store<FDX_BN>(a, acc, reinterpret_cast<float*>(smem), m0, n0);
}

template <int BN = FDX_BN, int RS = FDX_RS>
__device__ __forceinline__ void fc1_dx_block(const MnistStepArgs& a, int bx, int by, bf16* smem) {
  DenseLoaderX<true> la{a.dh, HID, a.B, HID};
  DenseLoaderX<true> lb{a.pbf + OFF_WD1, HID, FEAT, HID};
  f32x4 acc[FDX_BM / 32][BN / 32];
  gemm_mainloop<FDX_BM, BN, FDX_BK, 2, 2, decltype(la), decltype(lb), RS>(la, lb, by * FDX_BM, bx * BN, 0, HID, smem,
                                                                          acc);  // ends with a barrier
  fc1_dx_unpool_store<BN>(a, acc, reinterpret_cast<float*>(smem), by * FDX_BM, bx * BN);
}

// K8 + K10: every fc-layer gradient in ONE launch (horizontal fusion of three independent
// products that all consume dH / dlogits): [fc1 dW tiles | fc1 dX tiles | out dW/db blocks].
constexpr int FDW_GX = HID / FDW_BN, FDW_GY = (FEAT + 1 + FDW_BM - 1) / FDW_BM;  // 16 x 50
constexpr int FDX_GX = FEAT / FDX_BN;                                             // 49 at BN 64
constexpr int FDX_GX2 = FEAT / FDX_BN2;
static_assert(FEAT % FDX_BN == 0 && FEAT % FDX_BN2 == 0, "fc1 dX tiles cover the 3136 features exactly");
// part 0: all three products; part 1: dW + out-layer grads (bucket A complete); part 2: dX only.
// dX block j of gx * gy tiles -> (bx, by). Workgroups are dealt to the 8 XCDs round-robin by id, so
// blocks j, j + 8, j + 16, ... share an XCD and its L2. Without the remap the gy row tiles reading
// one W1 column tile (bx) sit on gy different XCDs (gx odd), and W1 (6.4 MB) is pulled into L2 gy
// times; with it, tile T = (j % 8) * per + j / 8 (bx = T / gy) keeps each column tile on one XCD.
__device__ __forceinline__ void fdx_tile(int j, int gx, int gy, int& bx, int& by) {
  const int full = (gx * gy) / (8 * gy) * (8 * gy);
  const int T = j < full ? (j & 7) * (full >> 3) + (j >> 3) : j;
  bx = T / gy;
  by = T - bx * gy;
}
__global__ __launch_bounds__(256) void fc1_bwd(MnistStepArgs a, int n_dx, int part) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  int id = blockIdx.x;
  const int gy = (a.B + FDX_BM - 1) / FDX_BM;
  if (part == 2) {
    int bx, by;
    fdx_tile(id, FDX_GX2, gy, bx, by);
    fc1_dx_block<FDX_BN2, FDX_RS_ALONE>(a, bx, by, (bf16*)smem_raw);
    return;
  }
  // the 17 output-layer blocks each walk the whole batch: dispatched first, their latency hides
  // under the GEMM tiles instead of forming the kernel's tail.
  if (id < OUTG_BLOCKS) { out_grad_block(a, id, (float*)smem_raw); return; }
  id -= OUTG_BLOCKS;
  // part 0: the dX blocks (K = 1024: 16 k-steps each) get the lowest block ids so they are
  // dispatched first and the short dW blocks (K = B) fill in around them, instead of the long
  // blocks starting last and forming the kernel's tail.
  if (part == 0) {
    if (id < n_dx) {
      int bx, by;
      fdx_tile(id, FDX_GX, gy, bx, by);
      fc1_dx_block_dma(a, bx, by, smem_raw);
      return;
    }
    id -= n_dx;
  }
  if (id < FDW_GX * FDW_GY) fc1_dw_block(a, id % FDW_GX, id / FDW_GX, (bf16*)smem_raw);
}

// ---------------- DP: fc gradients from all-gathered sufficient factors ----------------
// The reference's PS sums the workers' gradients (/root/reference/mnist_python_m.py:216-222). For
// the two fc layers the per-rank gradients are outer-product sums over the rank's batch, so the
// SUM over ranks is the same GEMM with K = W*B over the ranks' factors concatenated along the
// batch: gathering the factors (p2 [B][3136] + dh/hd [B][1024] bf16 + dlogits [B][10] fp32 =
// 1.33 MB per rank at B = 128) replaces the all-reduce of the 6.4 MB bf16 fc gradient. On xGMI a
// ring all-reduce moves 2(W-1)/W x 6.4 MB per rank, the gather (W-1) x 1.33 MB spread over W-1
// peer links, so below W ~ 9 the gather moves fewer bytes per link (W = 2: 1.33 vs 6.4 MB over the
// one link). Every rank then runs the identical GEMM on identical data: bit-identical gradients on
// all ranks, fp32-accumulated over all W*B rows (no bf16 rounding of per-rank partial sums).
// Branch-free (buffer-load) operands of the K = W*B GEMM, so its RS = 2 register pipeline keeps two
// K-tiles of loads in flight (with branching loads the compiler waits for all of them each step).
// KC = false over per-rank slots: (mn, k) = X[row k % B of rank k / B][mn]; mn_lim % 8 == 0.
struct RankRowsMC {
  static constexpr bool KC = false;
  const uint16_t* __restrict__ x;
  int ld, mn_lim, k_lim, B;
  int64_t rs;       // rank slot stride (elements)
  uint32_t nbytes;  // whole gathered array
  __device__ __forceinline__ uint4 operator()(int mn, int k) const {
    const int r = k / B;
    return buf_ld(x, nbytes, (uint32_t)(r * rs + (int64_t)(k - r * B) * ld + mn), k < k_lim && mn < mn_lim);
  }
};

// Output layer [1025][10] = [Hd;1]^T dlogits over the W*B gathered rows: a block owns 16 rows m
// (lane r = t & 15) x 16 row groups (q = t >> 4) of the K range, so even W = 8 leaves 64 rows per
// thread; partials summed in fixed group order through LDS (deterministic, rank-independent).
constexpr int OUTS_ROWS = 16, OUTS_GROUPS = 16, OUTS_LB = 8;
constexpr int OUTS_BLOCKS = (HID + 1 + OUTS_ROWS - 1) / OUTS_ROWS;  // 65 (the last holds the bias row)
__device__ __forceinline__ void out_grad_sfb_block(const MnistStepArgs& a, int blk, float* part) {
  const int t = threadIdx.x, r = t & (OUTS_ROWS - 1), q = t / OUTS_ROWS;
  const int m = blk * OUTS_ROWS + r;
  const int B = a.B, WB = a.sfb_world * B;
  const int per = (WB + OUTS_GROUPS - 1) / OUTS_GROUPS, k0 = min(WB, q * per), k1 = min(WB, k0 + per);
  const int64_t hoff = (int64_t)B * HID, doff = 2 * (int64_t)B * HID;  // hd / dlogits inside a slot
  float acc[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) acc[c] = 0.f;
  if (m <= HID) {
    for (int kb = k0; kb < k1; kb += OUTS_LB) {
      float hv[OUTS_LB];
      const float* dl[OUTS_LB];
#pragma unroll
      for (int u = 0; u < OUTS_LB; ++u) {  // every load of the batch in flight before the FMAs
        const int k = min(kb + u, k1 - 1), rk = k / B, row = k - rk * B;
        const uint16_t* slot = a.sfb_dr + rk * a.sfb_rs;
        hv[u] = (kb + u < k1) ? (m < HID ? bf2f(slot[hoff + (int64_t)row * HID + m]) : 1.f) : 0.f;
        dl[u] = reinterpret_cast<const float*>(slot + doff) + row * NCLS;
      }
#pragma unroll
      for (int u = 0; u < OUTS_LB; ++u)
#pragma unroll
        for (int c = 0; c < NCLS; ++c) acc[c] = fmaf(hv[u], dl[u][c], acc[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < NCLS; ++c) part[(q * OUTS_ROWS + r) * NCLS + c] = acc[c];
  __syncthreads();
  if (t < OUTS_ROWS * NCLS) {
    const int rr = t / NCLS, c = t - rr * NCLS, mm = blk * OUTS_ROWS + rr;
    float g = 0.f;
#pragma unroll
    for (int qq = 0; qq < OUTS_GROUPS; ++qq) g += part[(qq * OUTS_ROWS + rr) * NCLS + c];
    if (mm <= HID) {
      const size_t o = OFF_OUT + (size_t)mm * NCLS + c;
      if (a.gbf_a) a.gbf_a[o] = f2bf_bits(g);
      else a.grad[o] = g;
    }
  }
}

// XCD-grouped tile order: workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8 share
// one L2; MI355X_MICROARCH.md, workgroup dispatch), so a row-major tile order spreads the 16 tiles
// that read the same A panel (64 dW rows x all K of p2) over all 8 L2s, each fetching it from MALL
// / HBM. Mapping the tiles with b % 8 == x to the contiguous range [x * n/8, (x + 1) * n/8) keeps a
// panel's readers on one XCD: A crosses into each L2 about once instead of 8 times. (The long-K
// GEMM is bound by that traffic: 32 FLOP per byte of A + B for 64 x 64 tiles.)
__device__ __forceinline__ int xcd_grouped_tile(int b, int first, int n) {
  const int x = b & 7;
  const int first_x = first + ((x - first) & 7);  // first block of [first, first + n) with b % 8 == x
  return x * (n >> 3) + ((b - first_x) >> 3);
}


// ---------------- K13 (LDS-staged): conv2 dgrad + conv1 relu/pool-mask epilogue ----------------
// Block = (image b, half h: input rows ih in [7h, 7h + 7)), 512 threads, 68 KiB LDS. dz2 rows oh
// in [7h - 2, 7h + 9) are staged once into a zero-bordered channel-chunk-major LDS image
// [8 chunks][11 rows][20 cols] x 16 B (planes padded to 224 px = 256-B multiple), W2 as
// [tap*32 + ci][co] rows streams through a two-stage ring; no im2col traffic. dX[p][ci] =
// sum_{tap,co} dz2[p - tap][co] W2[tap][ci][co]. M-tile = one input row (16 lanes = iw 0..15, 14
// valid) so the 16 A-fragment lanes read 16 consecutive 16-B slots (conflict-free); N = 32 (2
// tiles); K = 1600. Wave w owns M-tiles {w & 3, (w & 3) + 4}, both N-tiles, every tap and the co
// half w >> 2: 2 A + 2 B fragment reads per 4 MFMAs; the two K halves are summed through LDS.
constexpr int C2D_ROWS = 11, C2D_COLS = 20, C2D_PLANE = 224;
// threads of a conv2_bwd_lds block (either role): 4 waves, and with both roles' LDS under 80 KB two
// blocks share a CU, so the launch's 512 blocks are all resident at once
constexpr int C2B_NT = 256;
// weight rows (tap, ci) x 64 co, staged by LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no
// ds_write pass; one wave instruction fills 1 KiB = 8 rows) into an unpadded image whose 16-B chunk
// c of row r holds global chunk c ^ (r & 7) -- the swizzle is applied to the per-lane SOURCE
// address, and the 16 rows of a B-fragment ds_read_b128 group then hit 16 distinct bank quads
// (time-neutral against register staging into pitch-80 rows, 25 KB less LDS).
__device__ __forceinline__ const bf16* c2d_w(const bf16* wt, int rr, int ch) {
  return wt + rr * 64 + ((ch ^ (rr & 7)) << 3);
}
// 16-B buffer load at voff + soff bytes (both in range; soff a wave-uniform scalar offset)
__device__ __forceinline__ uint4 buf_ld_so(const uint16_t* base, uint32_t nbytes, uint32_t voff, uint32_t soff) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nbytes, 0x00020000);
  const i32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
  return make_uint4((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]);
}
// W2 streams through a two-stage LDS ring of C2D_TPS taps (20 KB a stage) instead of staying whole
// (100 KB): at 69.6 KB two blocks (dgrad or wgrad) share a CU, so the launch's 512 blocks are all
// resident at once and one block's staging waits overlap the other's MFMA phases
#ifndef C2D_TPS
#define C2D_TPS 5
#endif
constexpr int C2D_NST = 25 / C2D_TPS, C2D_WSTAGE = C2D_TPS * 32 * 64;  // stages, elements per stage
static_assert(C2D_NST * C2D_TPS == 25 && C2D_WSTAGE % 512 == 0, "whole W2 stages of 1-KB DMA rows");
constexpr int C2D_SMEM = (8 * C2D_PLANE * 8 + 2 * C2D_WSTAGE) * 2;  // 69,632 B
static_assert(2 * C2D_SMEM <= 160 * 1024, "two conv2_bwd_lds blocks share a CU (the launch's point)");
static_assert(C2D_PLANE * 16 % 256 == 0 && C2D_PLANE >= C2D_ROWS * C2D_COLS, "dz2 plane");
constexpr int C2D_X_OFF = 8 * C2D_PLANE * 8 * 2;          // 28672: the fused tail's buffers (dead weight region)
// The conv1 weight gradient of the tail on the matrix core. dW1[tap][c] =
// sum_px X[tap][px] dz1[px][c] over the half image's 14 x 28 conv1 output pixels (rows padded to
// 32, K = 448 = 14 k-steps) with dz1 the unpooled pre-activation gradient (the bf16-rounded pooled
// gradient at its window's argmax position, zero elsewhere) and X the im2col of the zero-bordered x
// image, read from 5 column-shifted bf16 copies of its 18 rows so every A fragment is one 16-B read;
// row 25 of A is ones (the bias). 8 waves = 2 tap tiles x 2 channel tiles x 2 K halves. Replaces the
// per-thread loop of 25 scalar LDS reads + FMAs per pooled pixel (phase clocks: 7.0 k of the dgrad
// block's 18.4 k cycles, profiles/stamps_dgrad_r3.log).
constexpr int C2D_Z_OFF = C2D_X_OFF;                        // dz1 [448][32] bf16, chunk-swizzled
constexpr int C2D_XS_OFF = C2D_Z_OFF + 448 * 32 * 2;        // x copies [5][18][40] bf16
constexpr int C2D_T_END = C2D_XS_OFF + 5 * 18 * 40 * 2;
static_assert(C2D_T_END <= C2D_SMEM && C2D_XS_OFF % 16 == 0 && (C2D_T_END - C2D_Z_OFF) % 16 == 0, "MFMA tail LDS");
__device__ __forceinline__ int c1w_dz(int px, int c) {  // element offset of dz1[px][c]
  return px * 32 + (((c >> 3) ^ (2 * ((px >> 3) & 1))) << 3) + (c & 7);
}
// timing-stamp builds (TFD_STAMP): thread 0 of dgrad block bid records s_memtime at 8 phase
// boundaries into dbg[5 * B * 8 + bid * 8 + k] (tools/debug/stamps.py dgrad)
#define C2D_STAMP(k)                                                                                     \
  do {                                                                                                   \
    if (TFD_STAMP && a.dbg && threadIdx.x == 0) a.dbg[5 * a.B * 8 + bid * 8 + (k)] = (int64_t)__builtin_amdgcn_s_memtime(); \
  } while (0)
__device__ __forceinline__ void conv2_dgrad_body(const MnistStepArgs& a, const int bid) {
  C2D_STAMP(0);
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* img = (bf16*)smem_raw;                           // [8][224][8]
  bf16* wt = img + 8 * C2D_PLANE * 8;                    // ring: stage s in [s & 1] of [2][C2D_TPS * 32][64]
  const int b = bid >> 1, h = bid & 1, t = threadIdx.x;
  const uint16_t* src = a.dz2 + (size_t)b * 196 * 64;
  const uint16_t* wsrc = a.pbf + OFF_WC2;
  // the tail's x image row: its loads go out before the staging, whose wait then covers them (as a
  // chain issued after the staging, two dependent round trips held the waves at the next barrier)
  const RowPre xr = data_row_pre(a, b);
  // W2 stage st (taps [st * C2D_TPS, +C2D_TPS): rows tap * 32 + ci) -> ring slot st & 1 by LDS-DMA
  // (global_load_lds_dwordx4: no VGPR round trip, no ds_write pass; one wave instruction = 8 rows)
  auto wdma = [&](int st) {
    constexpr int NI = C2D_WSTAGE / 512;  // wave instructions per stage
    static_assert(NI % (C2B_NT / 64) == 0, "whole DMA instructions per wave");
    const int wv = t >> 6, ln = t & 63;
    const uint16_t* s0 = wsrc + st * C2D_WSTAGE;
    bf16* d0 = wt + (st & 1) * C2D_WSTAGE;
#pragma unroll
    for (int k = 0; k < NI / (C2B_NT / 64); ++k) {
      const int ii = wv + (C2B_NT / 64) * k, p = ii * 64 + ln, rr = p >> 3, sl = p & 7;
      __builtin_amdgcn_global_load_lds((const void*)(s0 + rr * 64 + ((sl ^ (rr & 7)) << 3)),
                                       (__attribute__((address_space(3))) void*)(d0 + ii * 64 * 8), 16, 0, 0);
    }
  };
  {
    constexpr int CI = 8 * C2D_PLANE, NI = CI / C2B_NT;  // 1792 chunks -> 7 per thread
    static_assert(CI % C2B_NT == 0, "whole image chunks per thread");
    wdma(0);  // the first two stages of the ring: in flight with the image staging
    wdma(1);
    uint4 vi[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int i = t + C2B_NT * j, ch = i / C2D_PLANE, px = i - ch * C2D_PLANE;
      const int r = px / C2D_COLS + 7 * h - 2, c = px % C2D_COLS - 2;
      vi[j] = buf_ld(src, 196 * 64 * 2, (uint32_t)((r * 14 + c) * 64 + ch * 8),
                     px < C2D_ROWS * C2D_COLS && (unsigned)r < 14u && (unsigned)c < 14u);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) *reinterpret_cast<uint4*>(img + (t + C2B_NT * j) * 8) = vi[j];
  }
  C2D_STAMP(1);
  const int lane = t & 63, w = t >> 6, g = lane >> 4, mt0 = w;
  const int two = (mt0 + 4 < 7);
  // the conv1-wgrad tail's global operands, issued now and consumed after the K loop (which reads
  // only LDS), so their latency hides behind it: the x image, and the conv1 relu outputs and argmax
  // bytes that mask and place this wave's dX rows
  float xpre[4];
  uint32_t p1pre[2][2][4];  // conv1 relu outputs (bf16 bits) and argmax window positions of the dX
  uint32_t ipb[2][2][4];    // values, 32-bit so the asm uses below can pin them in VGPRs
  {
    // (as exec-masked loads each value's bf16 conversion lands in its branch, with vmcnt(0): a
    // branch-free buffer-load form measured +0.3 us, profiles/mnist_kernels_r6_final.txt)
    const float* xrow = a.data + (size_t)data_row_use(a, xr, b) * 784;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = 4 * t + q, r = i >> 5, c = i & 31;
      xpre[q] = (r >= 2 && r < 30 && c >= 2 && c < 30) ? xrow[(r - 2) * 28 + c - 2] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int x = min(4 * g + r, 13), n = nt * 16 + (lane & 15), ih = 7 * h + min(mt0 + 4 * j, 6);
        p1pre[j][nt][r] = a.p1[((size_t)b * 196 + ih * 14 + x) * 32 + n];
        ipb[j][nt][r] = a.idx1[((size_t)b * 196 + ih * 14 + x) * 32 + n];
      }
  __syncthreads();
  C2D_STAMP(2);
  const int iw = lane & 15, nl = lane & 15;
  f32x4 acc[2][2];  // this wave's dX tiles (rows mt0, mt0 + 4) x both N-tiles, summed over all of K
#pragma unroll
  for (int j = 0; j < 2; ++j) acc[j][0] = acc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Fully unrolled, software-pipelined K loop: step st = (tap st >> 1, co half st & 1), both M-tiles
  // (wave 3's second reads rows past the image, never stored) and both N-tiles; step st + 1's fragments
  // are read while step st's MFMAs run. A stage boundary's barrier publishes the next W2 stage (DMA'd a
  // stage earlier) and frees the slot the one after streams into. Bases sit at the most negative tap
  // shift (kh = kw = 4) and ring slot 0: every address is base + a non-negative constant (ds offset).
  {
    const bf16* a0 = img + ((mt0 + 4) * C2D_COLS + iw + 4) * 8 + g * C2D_PLANE * 8 - (4 * C2D_COLS + 4) * 8;
    const bf16* a1 = a0 + 4 * C2D_COLS * 8;
    const bf16* bw[2][2] = {{c2d_w(wt, nl, g), c2d_w(wt, 16 + nl, g)}, {c2d_w(wt, nl, g + 4), c2d_w(wt, 16 + nl, g + 4)}};
    bf16x8 fb[2][2], fa[2][2];
    auto ld = [&](int st, int slot) {
      const int tap = st >> 1, sk = st & 1;
      const int woff = ((tap / C2D_TPS) & 1) * C2D_WSTAGE + (tap % C2D_TPS) * 32 * 64;
      const int kh = tap / 5, kw = tap - kh * 5, aoff = ((4 - kh) * C2D_COLS + 4 - kw) * 8 + sk * 4 * C2D_PLANE * 8;
      fb[slot][0] = *reinterpret_cast<const bf16x8*>(bw[sk][0] + woff);
      fb[slot][1] = *reinterpret_cast<const bf16x8*>(bw[sk][1] + woff);
      fa[slot][0] = *reinterpret_cast<const bf16x8*>(a0 + aoff);
      fa[slot][1] = *reinterpret_cast<const bf16x8*>(a1 + aoff);
    };
    constexpr int NS = 50, SPS = 2 * C2D_TPS;  // steps, steps per W2 stage
    ld(0, 0);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int cur = st & 1;
      if (st + 1 < NS) {
        if ((st + 1) % SPS == 0) {
          __syncthreads();
          if ((st + 1) / SPS + 1 < C2D_NST) wdma((st + 1) / SPS + 1);
        }
        ld(st + 1, cur ^ 1);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[j][0] = mfma16x16x32(fa[cur][j], fb[cur][0], acc[j][0]);
        acc[j][1] = mfma16x16x32(fa[cur][j], fb[cur][1], acc[j][1]);
      }
    }
  }
  // pinned here: wave 3 uses its second M-tile only under a branch (two), and the compiler sank that
  // tile's 100 MFMAs into it, keeping every step's fragments alive across the loop (400+ spills)
#pragma unroll
  for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[j][0]), "+v"(acc[j][1]));
  C2D_STAMP(3);
  __syncthreads();  // every wave is out of the K loop: the ring region becomes the tail's buffers
  for (int i = t; i < (C2D_T_END - C2D_Z_OFF) / 16; i += C2B_NT)  // dz1 and the x copies start zero
    reinterpret_cast<uint4*>(smem_raw + C2D_Z_OFF)[i] = zero4();
  __syncthreads();
  C2D_STAMP(4);
  {
    bf16* dz1 = reinterpret_cast<bf16*>(smem_raw + C2D_Z_OFF);
    bf16* xsh = reinterpret_cast<bf16*>(smem_raw + C2D_XS_OFF);
    // dX through conv1's relu mask, scattered to the argmax pixel. The relu / argmax bytes are first
    // touched here: without these empty asm uses the compiler turned the relu values into compare
    // masks right after their loads, i.e. the waves waited for 32 scattered loads before the K loop.
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(p1pre[j][nt][r]), "+v"(ipb[j][nt][r]));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j == 1 && !two) break;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int n = nt * 16 + (lane & 15), lr = mt0 + 4 * j;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int x = 4 * g + r;
          if (x >= 14) break;
          const int wi = ipb[j][nt][r], px = (2 * lr + (wi >> 1)) * 32 + 2 * x + (wi & 1);
          reinterpret_cast<uint16_t*>(dz1)[c1w_dz(px, n)] = p1pre[j][nt][r] != 0 ? f2bf_bits(acc[j][nt][r]) : (uint16_t)0;
        }
      }
    }
    // x rows 14h .. 14h + 17 of the zero-bordered image, 5 column shifts, bf16
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = 4 * t + q, r = i >> 5, c = i & 31, rr = r - 14 * h;
      if ((unsigned)rr < 18u) {
        const uint16_t xv = f2bf_bits(xpre[q]);
#pragma unroll
        for (int kw = 0; kw < 5; ++kw)
          if (c >= kw) reinterpret_cast<uint16_t*>(xsh)[(kw * 18 + rr) * 40 + c - kw] = xv;
      }
    }
    __syncthreads();
    C2D_STAMP(5);
    const int mi = w & 1, ni = w >> 1;  // tap tile (taps 0..15 / 16..31; 25 = bias), channel tile
    const int tap = 16 * mi + (lane & 15), tc = min(tap, 24), tkh = tc / 5, tkw = tc - 5 * tkh;
    const int q = (lane & 15) >> 2, p4 = lane & 3;
    bf16x8 ones, zer;
#pragma unroll
    for (int e = 0; e < 8; ++e) { ones[e] = (bf16)1.0f; zer[e] = (bf16)0.0f; }
    f32x4 c2 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 14; ++ks) {
      const int px0 = ks * 32 + 8 * g, rl = px0 >> 5, col0 = px0 & 31;
      bf16x8 af = *reinterpret_cast<const bf16x8*>(xsh + (tkw * 18 + rl + tkh) * 40 + col0);
      if (tap >= 25) af = (tap == 25) ? ones : zer;
      const int row0 = ks * 32 + 8 * g + q, col = 16 * ni + 4 * p4;
      const bf16x8 bfr = frag_tr16(dz1 + c1w_dz(row0, col), dz1 + c1w_dz(row0 + 4, col));
      c2 = mfma16x16x32(af, bfr, c2);
    }
    C2D_STAMP(6);
    const int c = 16 * ni + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int to = 16 * mi + 4 * g + r;  // taps 0..24, 25 = bias
      if (to < 26) a.wg1_slab[(size_t)bid * 832 + to * 32 + c] = c2[r];
    }
    C2D_STAMP(7);
  }
}

// ---------------- K14 (LDS-staged): conv2 wgrad (+ K12 bias row) ----------------
// Block = (tap group tg, image group ip), 256 threads; 6 x 32 = 192 blocks at B = 128.
// Per image: p1 (14x14x32) goes into a zero-bordered LDS image [18][18] x 40 ch and dz2 (196 x 64)
// into LDS rows [224][72] (pixel rows 196..223 zero); then dW[tap*32 + ci][co] += sum_px
// p1[px + tap][ci] * dz2[px][co] on MFMA with BOTH fragments read by ds_read_b64_tr_b16 (rows =
// pixels), so the im2col shift of a tap is just a per-lane row address. Wave w owns ci-tile
// w >> 1, co-tiles 2 (w & 1) and 2 (w & 1) + 1 and every tap of its group. One fp32 slab per image group (rows of its tap
// group; tap group 0 also the bias row 800), reduced by the optimizer tail / reduce_conv_grads.
// Replaces the im2col GEMM that re-read p1 25x through L2 (83 MB -> 19 MB of staging).
// Images per block x tap groups (profiles/mnist_conv2_wgrad_grouping_r6.log): 4 x 6 (192 blocks, 32 slabs:
// the optimizer tail reads 6.6 MB of slabs, not 13.1) 59.0-59.4 us/step; 2 x 4 60.2-60.6; 4 x 8 59.7-60.0.
constexpr int C2WL_IMG = 4;  // images per block (= slab count B / C2WL_IMG)
constexpr int C2WL_NTG = 6;  // tap groups (6: five of 4 taps, the last 5)
constexpr int C2WL_TPG = 25 / C2WL_NTG;     // taps per group (the last takes the remainder)
constexpr int C2WL_MAXT = 25 - C2WL_TPG * (C2WL_NTG - 1);
constexpr int C2WL_CS = 48, C2WL_PW = 18;   // padded image: 18 x 18 positions x 48-ch stride
                                            // (A tr-reads: 2296 LDS cycles per image vs 2968 at 40)
constexpr int C2WL_DS = 72, C2WL_KP = 224;  // dz2 rows: pixels padded to 7 k-steps of 32
constexpr int C2WL_IMG_ELEMS = C2WL_PW * C2WL_PW * C2WL_CS;
constexpr int C2WL_BRED_OFF = (C2WL_IMG_ELEMS + C2WL_KP * C2WL_DS) * 2;
constexpr int C2WL_SMEM = C2WL_BRED_OFF + 4 * 64 * 4;  // 64,384 B
static_assert(C2WL_BRED_OFF % 16 == 0 && (C2WL_IMG_ELEMS * 2) % 16 == 0, "LDS carve alignment");
#define C2W_STAMP(k)                                                                                     \
  do {                                                                                                   \
    if (TFD_STAMP && a.dbg && threadIdx.x == 0) a.dbg[7 * a.B * 8 + bid * 8 + (k)] = (int64_t)__builtin_amdgcn_s_memtime(); \
  } while (0)
__device__ __forceinline__ void conv2_wgrad_body(const MnistStepArgs& a, const int bid) {
  C2W_STAMP(0);
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16* img = (bf16*)smem_raw;
  bf16* dz = img + C2WL_IMG_ELEMS;
  float* bred = reinterpret_cast<float*>(smem_raw + C2WL_BRED_OFF);  // [4][64]
  const int tg = bid % C2WL_NTG, ip = bid / C2WL_NTG, t = threadIdx.x;
  const int tap0 = tg * C2WL_TPG, ntaps = (tg == C2WL_NTG - 1) ? 25 - tap0 : C2WL_TPG;
  const int lane = t & 63, w = t >> 6, h = w >> 1, n0 = 2 * (w & 1), g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;
  constexpr int N1 = (784 + C2B_NT - 1) / C2B_NT, N2 = (1568 + C2B_NT - 1) / C2B_NT;  // 16-B chunks per thread
  uint4 v1[N1], v2[N2];
  // branch-free buffer loads; chunk j of a thread is 16 t + 4096 j bytes, so the whole chunks share
  // one offset VGPR with j in the scalar offset (per-j offset VGPRs lived across the MFMA loop and
  // spilled, and every reload waited for the prefetch in flight), the partial last one range-checked
  auto gload = [&](int b) {
    const uint16_t* s1 = a.p1 + (size_t)b * 196 * 32;
    const uint16_t* s2 = a.dz2 + (size_t)b * 196 * 64;
#pragma unroll
    for (int j = 0; j < N1; ++j) {
      const int i = t + C2B_NT * j;
      v1[j] = (C2B_NT * (j + 1) <= 784) ? buf_ld_so(s1, 196 * 32 * 2, 16u * t, 16u * C2B_NT * j)
                                        : buf_ld(s1, 196 * 32 * 2, 8u * i, i < 784);
    }
#pragma unroll
    for (int j = 0; j < N2; ++j) {
      const int i = t + C2B_NT * j;
      v2[j] = (C2B_NT * (j + 1) <= 1568) ? buf_ld_so(s2, 196 * 64 * 2, 16u * t, 16u * C2B_NT * j)
                                         : buf_ld(s2, 196 * 64 * 2, 8u * i, i < 1568);
    }
  };
  if (ip * C2WL_IMG < a.B) gload(ip * C2WL_IMG);  // first image's loads before the LDS zeroing
  // the image border and the dz2 pad rows stay zero for every image of the block
  for (int i = t; i < C2WL_PW * C2WL_PW; i += C2B_NT) {
    const int r = i / C2WL_PW, c = i - r * C2WL_PW;
    if (r < 2 || r >= 16 || c < 2 || c >= 16) {
      uint4* d = reinterpret_cast<uint4*>(img + i * C2WL_CS);
      d[0] = zero4(); d[1] = zero4(); d[2] = zero4(); d[3] = zero4();
    }
  }
  for (int i = t; i < (C2WL_KP - 196) * (C2WL_DS / 8); i += C2B_NT) reinterpret_cast<uint4*>(dz + 196 * C2WL_DS)[i] = zero4();
  // padded-image positions of this lane's two tr-read rows (k-slots 32s + 8g + q and +4) per k-step
  int pos[7][2];
#pragma unroll
  for (int s = 0; s < 7; ++s)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = 32 * s + 8 * g + q + 4 * u;
      pos[s][u] = k < 196 ? (k / 14) * C2WL_PW + (k % 14) : 0;  // pad pixels: dz2 rows are zero
    }
  f32x4 acc[C2WL_MAXT][2];
#pragma unroll
  for (int j = 0; j < C2WL_MAXT; ++j) acc[j][0] = acc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  // image ii + 1's global loads are issued before image ii's MFMAs, so its staging latency hides
  // under them (one image at a time left the CU idle through each ~37 KB load)
  for (int ii = 0; ii < C2WL_IMG; ++ii) {
    const int b = ip * C2WL_IMG + ii;
    if (b >= a.B) break;
    __syncthreads();  // the previous image's fragments are consumed
    {
      int tt = t;  // opaque: the store addresses are recomputed per image, not held across the MFMAs
      asm volatile("" : "+v"(tt));
#pragma unroll
      for (int j = 0; j < N1; ++j) {
        const int i = tt + C2B_NT * j;
        if (i < 784) {
          const int px = i >> 2, ch = i & 3, r = px / 14, c = px - r * 14;
          *reinterpret_cast<uint4*>(img + ((r + 2) * C2WL_PW + c + 2) * C2WL_CS + ch * 8) = v1[j];
        }
      }
#pragma unroll
      for (int j = 0; j < N2; ++j) {
        const int i = tt + C2B_NT * j;
        if (i < 1568) *reinterpret_cast<uint4*>(dz + (i >> 3) * C2WL_DS + (i & 7) * 8) = v2[j];
      }
    }
    __syncthreads();
    C2W_STAMP(1 + 2 * ii);
    if (ii + 1 < C2WL_IMG && b + 1 < a.B) gload(b + 1);
    if (tg == 0) {  // bias row: column sums of dz2 (pixel slice t >> 6 of 4)
      static_assert(196 % (C2B_NT / 64) == 0, "whole pixel slices");
      const bf16* dzc = dz + (t >> 6) * C2WL_DS + (t & 63);
#pragma unroll 7
      for (int k = 0; k < 196 / (C2B_NT / 64); ++k) bsum += bf2f(dzc[k * (C2B_NT / 64) * C2WL_DS]);
    }
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      bf16x8 bfr[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const bf16* bp0 = dz + (32 * s + 8 * g + q) * C2WL_DS + 16 * (n0 + u) + 4 * p4;
        bfr[u] = frag_tr16(bp0, bp0 + 4 * C2WL_DS);
      }
#pragma unroll
      for (int j = 0; j < C2WL_MAXT; ++j) {
        if (j < ntaps) {
          const int tap = tap0 + j, toff = (tap / 5) * C2WL_PW + (tap % 5);
          const bf16* a0 = img + (pos[s][0] + toff) * C2WL_CS + 16 * h + 4 * p4;
          const bf16* a1 = img + (pos[s][1] + toff) * C2WL_CS + 16 * h + 4 * p4;
          const bf16x8 af = frag_tr16(a0, a1);
          acc[j][0] = mfma16x16x32(af, bfr[0], acc[j][0]);
          acc[j][1] = mfma16x16x32(af, bfr[1], acc[j][1]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one k-step's fragments live at a time
    }
    C2W_STAMP(2 + 2 * ii);
  }
#pragma unroll
  for (int j = 0; j < C2WL_MAXT; ++j) asm volatile("" : "+v"(acc[j][0]), "+v"(acc[j][1]));  // (as the dgrad's)
  float* slab = a.wg2_slab + (size_t)ip * 801 * 64;
#pragma unroll
  for (int j = 0; j < C2WL_MAXT; ++j) {
    if (j < ntaps) {
      const int tap = tap0 + j;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          slab[(size_t)(tap * 32 + 16 * h + 4 * g + r) * 64 + 16 * (n0 + u) + (lane & 15)] = acc[j][u][r];
    }
  }
  if (tg == 0) {
    bred[(t >> 6) * 64 + (t & 63)] = bsum;
    __syncthreads();
    if (t < 64) {
      float sm = 0.f;
#pragma unroll
      for (int sl = 0; sl < C2B_NT / 64; ++sl) sm += bred[sl * 64 + t];
      slab[800 * 64 + t] = sm;
    }
  }
  C2W_STAMP(7);
}

// conv2 wgrad and dgrad (+ the conv1 wgrad tail) in ONE launch: both consume only dz2. Blocks [0, nw)
// wgrad, then dgrad; 4-wave blocks at <= 68 KB of LDS, two per CU, all resident at once, so one block's
// operand waits overlap the other's MFMA / LDS phases (8-wave 131-KB blocks ran in two serial waves).
__global__ __launch_bounds__(C2B_NT, 2) void conv2_bwd_lds(MnistStepArgs a, int nw) {
  if ((int)blockIdx.x < nw) {
    conv2_wgrad_body(a, blockIdx.x);
  } else {
    conv2_dgrad_body(a, blockIdx.x - nw);
  }
}

// Deterministic slab reductions of both conv weight-gradient slab sets in ONE launch:
// thread (x = output column of a 64-wide chunk, y = slab phase 0..3); fixed summation order.
template <int XW>  // XW outputs per block row, 256/XW slab phases
__device__ __forceinline__ void reduce_chunk(const float* __restrict__ slab, int nslab, int64_t stride, int n, int i0,
                                             float* __restrict__ out, uint16_t* __restrict__ outbf, float* red) {
  constexpr int NY = 256 / XW;
  const int x = threadIdx.x % XW, y = threadIdx.x / XW, i = i0 + x;
  float s = 0.f;
  if (i < n) {
    int k = y;
    for (; k + 3 * NY < nslab; k += 4 * NY) {  // 4 independent loads in flight per thread
      const float v0 = slab[(size_t)k * stride + i], v1 = slab[(size_t)(k + NY) * stride + i];
      const float v2 = slab[(size_t)(k + 2 * NY) * stride + i], v3 = slab[(size_t)(k + 3 * NY) * stride + i];
      s += (v0 + v1) + (v2 + v3);
    }
    for (; k < nslab; k += NY) s += slab[(size_t)k * stride + i];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (y == 0 && i < n) {
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < NY; ++q) r += red[q * XW + x];
    if (outbf) outbf[i] = f2bf_bits(r);  // DP bf16 wire format: no separate cast pass
    else out[i] = r;
  }
}
constexpr int RED2_BLOCKS = (801 * 64 + 63) / 64;  // 801 blocks x 64 outputs (4 phases over the B/2 slabs)
constexpr int RED1_BLOCKS = (832 + 15) / 16;       // 52 blocks x 16 outputs (16 phases over 2B slabs)
__global__ __launch_bounds__(256) void gather_next_kernel(MnistStepArgs a) { gather_next(a, *a.step + 1, blockIdx.x); }
// gb > 0: the first gb blocks gather the next step's batch (step number from MnistStepArgs::t_out,
// written by this step's head kernel, so nothing here reads the step that block gb bumps) -- one
// launch instead of gather_next_kernel + reduce_conv_grads on the DP path
__device__ __forceinline__ void conv_reduce_block(const MnistStepArgs& a, int blk, int gb, float* red) {
  if (blk < gb) {
    gather_next(a, *a.t_out, blk);
    return;
  }
  const int id = blk - gb;
  if (id < RED2_BLOCKS)
    reduce_chunk<64>(a.wg2_slab, a.wg2_splits, 801 * 64, 801 * 64, id * 64, a.grad + OFF_WC2,
                     a.gbf_b ? a.gbf_b + OFF_WC2 : nullptr, red);
  else
    reduce_chunk<16>(a.wg1_slab, 2 * a.B, 832, 832, (id - RED2_BLOCKS) * 16, a.grad + OFF_WC1,
                     a.gbf_b ? a.gbf_b + OFF_WC1 : nullptr, red);
  if (id == 0 && threadIdx.x == 0 && a.step_bump) *a.step_bump += 1;  // see MnistStepArgs::step_bump
}
__global__ __launch_bounds__(256) void reduce_conv_grads(MnistStepArgs a, int gb) {
  __shared__ float red[256];
  conv_reduce_block(a, blockIdx.x, gb, red);
}

// [output-layer blocks | fc1 dW (+ bias row) tiles over K = W*B | nlead: next-batch gather + conv
// slab-reduce blocks (conv_reduce_block)]. nlead > 0 is the merged DP tail: the slab reduce (a
// latency-bound 5 us launch of its own) runs beside the SFB GEMM's blocks instead of before them.
__global__ __launch_bounds__(256) void fc_grad_sfb(MnistStepArgs a, int gb, int nlead) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  // the GEMM's blocks are dealt first, the short reduce / gather blocks fill in behind them (5 of 6
  // interleaved pairs 0.1-1 us/step faster than reduce-first, profiles/mnist_dp_kernels_r5.txt)
  const int b = blockIdx.x, nsfb = (int)gridDim.x - nlead;
  if (b >= nsfb) {
    conv_reduce_block(a, b - nsfb, gb, (float*)smem_raw);
    return;
  }
  int id = b;
  if (id < OUTS_BLOCKS) { out_grad_sfb_block(a, id, (float*)smem_raw); return; }
  // tile rows: all FDW_GY, or (ZeRO shard) [by_lo, by_hi] plus the bias row's tile
  const bool part = a.sfb_by_hi >= a.sfb_by_lo;
  const int nby = part ? (a.sfb_by_hi - a.sfb_by_lo + 1) + (a.sfb_by_hi < FDW_GY - 1 ? 1 : 0) : FDW_GY;
  static_assert(FDW_GX % 8 == 0, "XCD grouping deals whole residue classes");
  id = xcd_grouped_tile(b, OUTS_BLOCKS, FDW_GX * nby);
  if (part) {
    int by = id / FDW_GX + a.sfb_by_lo;
    if (by > a.sfb_by_hi) by = FDW_GY - 1;  // the bias row (3136) is updated by every rank
    id = by * FDW_GX + id % FDW_GX;
  }
  const int WB = a.sfb_world * a.B;
  OnesRowBuf la{a.sfb_p2, WB, (uint32_t)((int64_t)WB * FEAT * 2)};
  RankRowsMC lb{a.sfb_dr, HID, HID, WB, a.B, a.sfb_rs, (uint32_t)((int64_t)a.sfb_world * a.sfb_rs * 2)};
  fc1_dw_tile(a, la, lb, (id / FDW_GX) * FDW_BM, (id % FDW_GX) * FDW_BN, WB, (bf16*)smem_raw);
}

// ---------------- one-GPU optimizer tail: K16 ApplyAdam with the K12/K14/K15 slab reduce fused ----------------
// Grid = [13 conv1 blocks | 201 conv2 blocks | MAD_FC_BLOCKS grid-stride blocks]:
//   conv1: block owns 16 float4 of the 832 conv1 weight/bias gradients; thread (q = t >> 4, x = t & 15)
//          sums slabs q, q + 16, ... of float4 x (16-lane groups read 256 contiguous bytes per slab,
//          every load issued before the first add), then the 16 partials are summed in LDS in q order;
//   conv2: block owns 64 float4; thread (q = t >> 6, x = t & 63) sums slabs q, q + 4, ... (each wave
//          reads 1 KiB contiguous per slab), then 4 partials in LDS in q order;
//   fc:    plain grid-stride Adam over the flat gradient buffer.
// Every gradient reduction is deterministic (fixed order). t comes from the head kernel
// (MnistStepArgs::t_out), so nothing here reads the global_step that the last block bumps.
// (The previous layout -- one 16-lane group per float4, each lane a different slab -- made every
//  wave instruction touch 64 scattered 16-B pieces: 7.6 us for the conv region alone.)
constexpr int MAD_NT = 256;
constexpr int MAD_C1F4 = (int)(OFF_WC2 / 4);   // 208
constexpr int MAD_C2END = (int)(OFF_WD1 / 4);  // 13024
constexpr int MAD_C1BLK = MAD_C1F4 / 16;       // 13
constexpr int MAD_C2BLK = (MAD_C2END - MAD_C1F4 + 63) / 64;  // 201
constexpr int MAD_FC_BLOCKS = 1024;  // grid-stride blocks of the fc-region Adam (512 / 2048: within noise)
constexpr int MAD_CONV = MAD_C1BLK + MAD_C2BLK;
static_assert(MAD_C1F4 % 16 == 0, "conv1 region: whole blocks");
constexpr int MAD_SL = 16;  // slab loads in flight per thread
__device__ __forceinline__ void adam4_pre(const MnistAdamArgs& o, int64_t i, f32x4 p, f32x4 m, f32x4 v, f32x4 g,
                                          float lr_t, float c1, float c2) {
  m = m + (g - m) * c1;
  v = v + (g * g - v) * c2;
#pragma unroll
  for (int j = 0; j < 4; ++j) p[j] -= lr_t * m[j] / (sqrtf(v[j]) + o.eps);
  reinterpret_cast<f32x4*>(o.p)[i] = p;
  reinterpret_cast<f32x4*>(o.m)[i] = m;
  reinterpret_cast<f32x4*>(o.v)[i] = v;
  if (o.pbf) reinterpret_cast<uint2*>(o.pbf)[i] = make_uint2(pack_bf2(p[0], p[1]), pack_bf2(p[2], p[3]));
}
__device__ __forceinline__ void adam4(const MnistAdamArgs& o, int64_t i, f32x4 g, float lr_t, float c1, float c2) {
  f32x4 p = reinterpret_cast<f32x4*>(o.p)[i];
  f32x4 m = reinterpret_cast<f32x4*>(o.m)[i];
  f32x4 v = reinterpret_cast<f32x4*>(o.v)[i];
  m = m + (g - m) * c1;
  v = v + (g * g - v) * c2;
#pragma unroll
  for (int j = 0; j < 4; ++j) p[j] -= lr_t * m[j] / (sqrtf(v[j]) + o.eps);
  reinterpret_cast<f32x4*>(o.p)[i] = p;
  reinterpret_cast<f32x4*>(o.m)[i] = m;
  reinterpret_cast<f32x4*>(o.v)[i] = v;
  if (o.pbf) reinterpret_cast<uint2*>(o.pbf)[i] = make_uint2(pack_bf2(p[0], p[1]), pack_bf2(p[2], p[3]));
}
// sum over slabs q, q + QS, ... (< ns) of float4 column x of a [ns][stride4] slab array; MAD_SL loads
// issued per batch before any add
template <int QS>
__device__ __forceinline__ f32x4 slab_sum(const f32x4* __restrict__ s4, int64_t stride4, int ns, int q, int x) {
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = q; k0 < ns; k0 += QS * MAD_SL) {
    f32x4 v[MAD_SL];
#pragma unroll
    for (int u = 0; u < MAD_SL; ++u) {
      const int k = k0 + u * QS;
      v[u] = k < ns ? s4[(size_t)k * stride4 + x] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < MAD_SL; ++u) acc += v[u];
  }
  return acc;
}
__global__ __launch_bounds__(MAD_NT) void mnist_adam_kernel(MnistStepArgs a, MnistAdamArgs o, int fcb4) {
  const int gb = gather_blocks(a);
  if ((int)blockIdx.x < gb) {  // the next step's batch; t = the step started next
    gather_next(a, *o.t, blockIdx.x);
    return;
  }
  const int grid = (int)gridDim.x - gb;
  // grid == MAD_CONV: the conv region only; the last conv2 block bumps the step
  if (grid == MAD_CONV && (int)blockIdx.x - gb == grid - 1 && threadIdx.x == 0) *o.step += 1;
  // t (a dependent load of the head's step counter) is awaited only where the update needs it,
  // after this thread's first operand loads are out (the optimizer's first memory round trip)
  auto lr_of = [&]() {
    const int64_t t = *o.t;
    const float b1p = powf(o.beta1, (float)t), b2p = powf(o.beta2, (float)t);
    return o.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  };
  const float c1 = 1.f - o.beta1, c2 = 1.f - o.beta2;
  const int bid = (int)blockIdx.x - gb, tid = threadIdx.x;
  if (bid < MAD_CONV) {
    __shared__ f32x4 red[MAD_NT];
    const bool one = bid < MAD_C1BLK;
    const int q = one ? tid >> 4 : tid >> 6, x = one ? tid & 15 : tid & 63;
    const int64_t i = one ? (int64_t)bid * 16 + x : MAD_C1F4 + (int64_t)(bid - MAD_C1BLK) * 64 + x;
    f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f};
    if (one) {
      g = slab_sum<16>(reinterpret_cast<const f32x4*>(a.wg1_slab) + i, 832 / 4, 2 * a.B, q, 0);
    } else if (i < MAD_C2END) {
      g = slab_sum<4>(reinterpret_cast<const f32x4*>(a.wg2_slab) + (i - MAD_C1F4), 801 * 64 / 4, a.wg2_splits, q, 0);
    }
    red[tid] = g;
    __syncthreads();
    if (q == 0 && i < MAD_C2END) {
      const int nq = one ? 16 : 4, qs = one ? 16 : 64;
      f32x4 s = red[x];
      for (int k = 1; k < nq; ++k) s += red[k * qs + x];
      adam4(o, i, s, lr_of(), c1, c2);
    }
  } else {
    const int64_t i0 = fcb4 + (int64_t)(bid - MAD_CONV) * MAD_NT + tid;  // fcb4: MAD_C2END, or the out layer
    const int64_t STRIDE = (int64_t)(grid - MAD_CONV) * MAD_NT;
    // ADAM_U strides' loads issued before any math/store, so U x 56 B per lane are in flight
    // (the one-at-a-time loop leaves the compiler no room: p/m/v stores may alias the next loads;
    // streaming non-temporal loads/stores were +0.9 us: the next step re-reads p/m/v from MALL)
    if (o.gbf) {
      constexpr int U = ADAM_U;
      const float lr_t = lr_of();
      for (int64_t base = i0; base < TOTAL / 4; base += STRIDE * U) {
        uint2 h[U];
        f32x4 p[U], m[U], v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = base + (int64_t)u * STRIDE;
          if (i < TOTAL / 4) {
            p[u] = reinterpret_cast<const f32x4*>(o.p)[i];
            h[u] = reinterpret_cast<const uint2*>(o.gbf)[i];
            m[u] = reinterpret_cast<const f32x4*>(o.m)[i];
            v[u] = reinterpret_cast<const f32x4*>(o.v)[i];
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = base + (int64_t)u * STRIDE;
          if (i < TOTAL / 4) {
            const f32x4 g = f32x4{__uint_as_float(h[u].x << 16), __uint_as_float(h[u].x & 0xFFFF0000u),
                                  __uint_as_float(h[u].y << 16), __uint_as_float(h[u].y & 0xFFFF0000u)};
            m[u] = m[u] + (g - m[u]) * c1;
            v[u] = v[u] + (g * g - v[u]) * c2;
#pragma unroll
            for (int j = 0; j < 4; ++j) p[u][j] -= lr_t * m[u][j] / (sqrtf(v[u][j]) + o.eps);
            reinterpret_cast<f32x4*>(o.p)[i] = p[u];
            reinterpret_cast<f32x4*>(o.m)[i] = m[u];
            reinterpret_cast<f32x4*>(o.v)[i] = v[u];
            reinterpret_cast<uint2*>(o.pbf)[i] = make_uint2(pack_bf2(p[u][0], p[u][1]), pack_bf2(p[u][2], p[u][3]));
          }
        }
      }
    } else {
      // the first item's p / m / v / g are loaded before t is awaited
      f32x4 p0 = {}, m0 = {}, v0 = {}, g0 = {};
      if (i0 < TOTAL / 4) {
        p0 = reinterpret_cast<const f32x4*>(o.p)[i0];
        m0 = reinterpret_cast<const f32x4*>(o.m)[i0];
        v0 = reinterpret_cast<const f32x4*>(o.v)[i0];
        g0 = reinterpret_cast<const f32x4*>(a.grad)[i0];
      }
      const float lr_t = lr_of();
      if (i0 < TOTAL / 4) adam4_pre(o, i0, p0, m0, v0, g0, lr_t, c1, c2);
      for (int64_t i = i0 + STRIDE; i < TOTAL / 4; i += STRIDE)
        adam4(o, i, reinterpret_cast<const f32x4*>(a.grad)[i], lr_t, c1, c2);
    }
    if (bid == grid - 1 && tid == 0) *o.step += 1;  // see MnistAdamArgs
  }
}

template <auto K>
inline void set_smem(int bytes) {  // raise the kernel's dynamic-LDS limit to the largest size asked so far
  static int limit = 64 * 1024;
  if (bytes > limit) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(K), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    limit = bytes;
  }
}

}  // namespace

int mnist_fc1_splits(int B) { (void)B; return FC1_SPLITS; }
int mnist_wg2_splits(int B) { return (B + C2WL_IMG - 1) / C2WL_IMG; }  // one slab per image group

void mnist_forward(const MnistStepArgs& a, bool train, hipStream_t s) {
  mnist_forward_conv(a, s);
  mnist_forward_fc(a, train, s);
}

void mnist_forward_conv(const MnistStepArgs& a, hipStream_t s) {
  set_smem<conv12_fwd_lds>(C12_SMEM);
  conv12_fwd_lds<<<2 * a.B, 512, C12_SMEM, s>>>(a);
}

void mnist_forward_fc(const MnistStepArgs& a, bool train, hipStream_t s) {
  const int B = a.B;
  {
    constexpr int sm = GemmSmemOneshot<FC1_BM, FC1_BN, FC1_BK, FC1_NKT, DenseLoaderX<true>, DenseLoaderX<false>>::BYTES;
    static_assert(sm <= 160 * 1024, "fc1 one-shot LDS");
    set_smem<fc1_fwd>(sm);
    const int kper = (FEAT + a.fc1_splits - 1) / a.fc1_splits;
    dim3 g(HID / FC1_BN, (B + FC1_BM - 1) / FC1_BM, a.fc1_splits);
    fc1_fwd<<<g, 256, sm, s>>>(a, kper);
  }
  head_kernel<<<B, 256, 0, s>>>(a, train ? 1 : 0);
}

void mnist_backward_a(const MnistStepArgs& a, hipStream_t s, int part) {
  const int B = a.B;
  constexpr int sm_dw = GemmSmem<FDW_BM, FDW_BN, FDW_BK, OnesRowBuf, DenseLoaderX<false>>::BYTES;
  static_assert(sm_dw >= FDW_BM * FDW_PITCH * 4, "fc1 dW staging image fits the GEMM's LDS");
  constexpr int sm_dx = GemmSmem<FDX_BM, FDX_BN, FDX_BK, DenseLoaderX<true>, DenseLoaderX<true>>::BYTES;
  static_assert(sm_dx >= FDX_BM * (FDX_BN + 4) * 4, "fc1 dX staging image fits the GEMM's LDS");
  const int sm_og = (B * NCLS + 4 * OUTG_ROWS * NCLS) * 4;
  const int sm = std::max(std::max(sm_dw, part == 2 ? sm_dx : FDXD_SMEM), sm_og);
  set_smem<fc1_bwd>(sm);
  const int n_dx = FDX_GX * ((B + FDX_BM - 1) / FDX_BM);
  const int nb = part == 2 ? FDX_GX2 * ((B + FDX_BM - 1) / FDX_BM) : FDW_GX * FDW_GY + (part == 0 ? n_dx : 0) + OUTG_BLOCKS;
  fc1_bwd<<<nb, 256, sm, s>>>(a, n_dx, part);
}

void mnist_backward_b(const MnistStepArgs& a, hipStream_t s) {
  // conv2 wgrad (one slab per image group), then dgrad + conv1 wgrad, in one launch (a forked wgrad
  // stream only contended with dgrad for the CUs: 110 vs 100 us/step, profiles/ab_conv_fork.log)
  static_assert(C2WL_SMEM <= C2D_SMEM, "conv2_bwd_lds: the dgrad LDS size covers the wgrad blocks");
  set_smem<conv2_bwd_lds>(C2D_SMEM);
  const int nw = C2WL_NTG * a.wg2_splits;
  conv2_bwd_lds<<<nw + 2 * a.B, C2B_NT, C2D_SMEM, s>>>(a, nw);
}

void mnist_conv_grad_reduce(const MnistStepArgs& a, hipStream_t s) {
  const bool gather = a.step_bump && a.perm && a.xpre;
  if (gather && a.t_out) {  // one launch: gather blocks read the next step from t_out
    reduce_conv_grads<<<a.B + RED2_BLOCKS + RED1_BLOCKS, 256, 0, s>>>(a, a.B);
    return;
  }
  // the next step's batch first (this kernel bumps the step; the gather reads it unbumped)
  if (gather) gather_next_kernel<<<a.B, 256, 0, s>>>(a);
  reduce_conv_grads<<<RED2_BLOCKS + RED1_BLOCKS, 256, 0, s>>>(a, 0);
}

void mnist_adam_fused(const MnistStepArgs& a, const MnistAdamArgs& o, hipStream_t s, bool fc_region) {
  const int gb = (a.perm && a.xpre) ? a.B : 0;
  mnist_adam_kernel<<<gb + MAD_CONV + (fc_region ? MAD_FC_BLOCKS : 0), MAD_NT, 0, s>>>(a, o, (int)(OFF_WD1 / 4));
}

int64_t mnist_sfb_slot_elems(int B) { return ((int64_t)B * (2 * HID + 2 * NCLS) + 63) / 64 * 64; }

void mnist_fc_grad_sfb(const MnistStepArgs& a, hipStream_t s, bool with_reduce) {
  if (a.sfb_world < 1 || !a.sfb_p2 || !a.sfb_dr) throw std::runtime_error("mnist_fc_grad_sfb: no gathered factors");
  constexpr int sm_og = OUTS_ROWS * OUTS_GROUPS * NCLS * 4;
  constexpr int sm_dw = GemmSmem<FDW_BM, FDW_BN, FDW_BK, OnesRowBuf, RankRowsMC>::BYTES;
  constexpr int sm = sm_dw > sm_og ? sm_dw : sm_og;
  static_assert(sm >= 256 * 4, "the merged slab-reduce blocks use the launch's LDS as their 256-float stage");
  set_smem<fc_grad_sfb>(sm);
  const bool part = a.sfb_by_hi >= a.sfb_by_lo;
  if (part && (a.sfb_by_lo < 0 || a.sfb_by_hi >= FDW_GY)) throw std::runtime_error("mnist_fc_grad_sfb: tile rows");
  const int nby = part ? (a.sfb_by_hi - a.sfb_by_lo + 1) + (a.sfb_by_hi < FDW_GY - 1 ? 1 : 0) : FDW_GY;
  int gb = 0, nlead = 0;
  if (with_reduce) {  // the slab reduce's contract (mnist_conv_grad_reduce): gather blocks read t_out
    if (a.step_bump && a.perm && a.xpre && !a.t_out)
      throw std::runtime_error("mnist_fc_grad_sfb: the merged gather reads the next step from t_out");
    gb = (a.step_bump && a.perm && a.xpre) ? a.B : 0;
    nlead = gb + RED2_BLOCKS + RED1_BLOCKS;
  }
  fc_grad_sfb<<<nlead + OUTS_BLOCKS + FDW_GX * nby, 256, sm, s>>>(a, gb, nlead);
}

void mnist_sfb_tile_rows(int row0, int row1, int* by_lo, int* by_hi) {
  *by_lo = row0 / FDW_BM;
  *by_hi = (row1 - 1) / FDW_BM;
}

}  // namespace tfd
