// Reference-precision (fp32) kernels of the MNIST CNN training step: the reference trains in fp32
// (tf.float32 placeholders, tf.random_normal params; /root/reference/mnist_python_m.py:185-200).
// Same fusion structure as the bf16 step (csrc/kernels/mnist.hip) -- bias+relu+2x2 pool+argmax in
// the conv epilogues, Philox dropout + FC10 + softmax-xent fused per batch row, MaxPoolGrad +
// ReluGrad in the dX / dgrad epilogues, deterministic split-K slabs for the long-K weight
// gradients -- but every activation is stored fp32 and every GEMM runs on the fp32 matrix core
// (v_mfma_f32_16x16x4_f32, csrc/gemm_f32.h). No bf16 rounding anywhere: gradients match an fp32
// PyTorch oracle to ~1e-5.
//
// Kernel map: f32_conv12_fwd_lds K1+K3+K2+K3; f32_fc1_fwd K4;
// f32_head K4-finish+K5+K6+K7+K8(dX)+K9; f32_fc1_bwd K8 dW + K10 dW/dX (+K11 unpool epilogue);
// f32_conv2_bwd_lds K13 (+conv1 ReluGrad mask, + the K15/K12 conv1 wgrad tail) + K14 (+K12 bias
// row) slabs. The slab reduce + optimizer are shared with the bf16 step.
#include "../common.h"

#include "../gemm.h"  // buf_ld
#include "../gemm_f32.h"
#include "../mnist_layout.h"
#include "../tfd_kernels.h"

#include <algorithm>

namespace tfd {
using namespace mnist;

namespace {

__device__ __forceinline__ int data_row_f(const int* perm, const int64_t* step, int n_data, int B, int b) {
  if (!perm) return b;
  const int64_t s = *step;
  return perm[(int)((s * (int64_t)B + b) % (int64_t)n_data)];
}

// ---------------- K1+K3+K2+K3: conv1 -> pool -> conv2 (whole-image implicit GEMM from LDS) -> pool ----------------
// The bf16 step's conv2 structure (csrc/kernels/mnist.hip conv12_fwd_lds) on the fp32 matrix core.
// Block = (image b, output-channel half nh), 512 threads (8 waves), 2B blocks. The image's 14x14x32
// fp32 activations are staged ONCE into a zero-bordered, channel-chunk-major LDS image [8 chunks of 4
// channels][18 rows][24 cols] x 16 B, and the block's half of W2 as [32 n][800 k + 4] (k contiguous):
// every A and B fragment of the 25-tap K loop is then one ds_read_b128 (read_frag4_f's K permutation:
// lane group g holds channels 16q + 4g .. + 3 of a tap), with no global re-reads of the 25x-expanded
// im2col matrix and no barrier inside the K loop (the generic-core version: 392 blocks each re-staging
// 64-row A and B tiles through LDS 25 times, a barrier per 32-deep K-tile). M = 196 rows in
// pool-window-major order (13 tiles of 16), N = 32 (2 tiles): 26 fragment tiles, wave w owns tiles
// f = w + 8j (m = f >> 1, n-tile = f & 1), so the SIMDs (waves w, w + 4) carry 7, 7, 6, 6 tiles.
// Row stride 24 px = 8 (mod 16) 16-B slots keeps a 16-lane read group of four pool windows on 16
// distinct slots; W2 rows 804 floats apart (= 36 mod 64 banks) keep the B reads conflict-free.
constexpr int F2F_W = 24, F2F_PLANE = 18 * F2F_W /*432 slots*/, F2F_WROW = 800 + 4;
constexpr int F2F_SMEM = (8 * F2F_PLANE * 4 + 32 * F2F_WROW) * 4;  // 55,296 + 102,912 = 158,208 B
static_assert(F2F_SMEM <= 160 * 1024, "conv2 LDS carve");

template <int NF>
__device__ __forceinline__ void f32_conv2_taps(const float* img, const float* wt, const int (&abase)[4], int bbase,
                                               f32x4 (&acc)[4]) {
  f32x4 a[2][NF], b[2];
  auto load = [&](int step, int slot) {  // step = tap * 2 + q
    const int tap = step >> 1, q = step & 1, kh = tap / 5, kw = tap - 5 * kh;
    const int aoff = ((4 * q) * F2F_PLANE + kh * F2F_W + kw) * 4;
#pragma unroll
    for (int j = 0; j < NF; ++j) a[slot][j] = *reinterpret_cast<const f32x4*>(img + abase[j] + aoff);
    b[slot] = *reinterpret_cast<const f32x4*>(wt + bbase + tap * 32 + 16 * q);
  };
  load(0, 0);
  // step st + 1's reads go out behind step st's first MFMAs (hard scheduling fences: left alone, the
  // scheduler sinks them below the step's last MFMA and every step starts with an LDS round trip)
#pragma unroll
  for (int st = 0; st < 50; ++st) {
    const int cur = st & 1;
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[j] = mfma16x16x4f32(a[cur][j][0], b[cur][0], acc[j]);
    __builtin_amdgcn_sched_barrier(0);
    if (st + 1 < 50) load(st + 1, cur ^ 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 1; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[j] = mfma16x16x4f32(a[cur][j][s], b[cur][s], acc[j]);
  }
}

// K1+K3 fused in front (f32_conv12_fwd_lds): conv1 + bias + relu + 2x2 pool + argmax on the fp32
// matrix core, straight into the LDS image conv2 reads (half 0 also writes p1 / idx1 for the
// backward). Implicit GEMM M = 784 pixels (pool-window-major, m = pp*4 + win), N = 32, K = 25 taps
// padded to 28: lane group g of MFMA step s takes tap 4s + g, one scalar LDS read of the x image per
// (m-tile, step), W1 in registers. Each half of an image recomputes conv1 (~686 MFMAs per block,
// the price of keeping conv2's p1 on chip); the conv2 weight half's loads are issued before it and
// land behind its arithmetic. The x image and W1 are staged in the W2 region, which is written only
// after conv1.
constexpr int F12_XS = 36;  // x image row pitch (floats): zero-bordered 32 x 32 coordinates
__global__ __launch_bounds__(512) void f32_conv12_fwd_lds(MnistF32Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  float* img = reinterpret_cast<float*>(smem_raw);  // [8][18*24] x float4
  float* wt = img + 8 * F2F_PLANE * 4;               // [32][804]
  float* xs = wt;                                    // conv1 staging: [32][36] x image,
  float* w1 = wt + 32 * F12_XS;                      //   [25][32] W1 + [32] bias
  const int b = blockIdx.x >> 1, nh = blockIdx.x & 1, t = threadIdx.x;
  // 1. loads: x / W1 first (needed first; a wave's vmcnt is in order), then the W2 half, which stays
  //    in registers until conv1 is done
  f32x4 xv = zero_f4(), w1v = zero_f4();
  if (t < 196) xv = reinterpret_cast<const f32x4*>(a.data + (size_t)data_row_f(a.perm, a.step, a.n_data, a.B, b) * 784)[t];
  else if (t >= 256 && t < 256 + (KTAPS * C1 + C1) / 4) w1v = reinterpret_cast<const f32x4*>(a.p32 + OFF_WC1)[t - 256];
  constexpr int NW = (800 * 8 + 511) / 512;  // 13 (800 k rows x 8 chunks of 4 n)
  f32x4 w2v[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const int i = t + 512 * j, k = i >> 3, n4 = (i & 7) * 4;
    w2v[j] = buf_ld_f4(a.p32 + OFF_WC2, 800u * 64u * 4u, (uint32_t)(k * 64 + nh * 32 + n4), i < 800 * 8);
  }
  // 2. zero the p1 image (its border is conv2's SAME padding) and the x image, then stage x / W1
  for (int i = t; i < 8 * F2F_PLANE; i += 512) reinterpret_cast<f32x4*>(img)[i] = zero_f4();
  for (int i = t; i < 32 * F12_XS / 4; i += 512) reinterpret_cast<f32x4*>(xs)[i] = zero_f4();
  __syncthreads();
  if (t < 196) {
    const int r = (4 * t) / 28, c = (4 * t) % 28;
    float* d = xs + (r + 2) * F12_XS + c + 2;
    d[0] = xv[0]; d[1] = xv[1]; d[2] = xv[2]; d[3] = xv[3];
  } else if (t >= 256 && t < 256 + (KTAPS * C1 + C1) / 4) {
    reinterpret_cast<f32x4*>(w1)[t - 256] = w1v;
  }
  __syncthreads();
  // 3. conv1 on the matrix core; wave w owns M-tiles w, w + 8, ... (<= 7 of 49)
  {
    const int lane = t & 63, wv = t >> 6, g = lane >> 4, col = lane & 15;
    float bw[7][2];
#pragma unroll
    for (int st = 0; st < 7; ++st) {
      const int k = 4 * st + g;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {  // clamped read + select: no exec-masked LDS read with its own wait
        const float wv1 = w1[min(k, KTAPS - 1) * C1 + nt * 16 + col];
        bw[st][nt] = k < KTAPS ? wv1 : 0.f;
      }
    }
    const float bias0 = w1[KTAPS * C1 + col], bias1 = w1[KTAPS * C1 + 16 + col];
    int toff[7];
#pragma unroll
    for (int st = 0; st < 7; ++st) {
      const int k = min(4 * st + g, KTAPS - 1), kh = k / 5, kw = k - 5 * kh;
      toff[st] = kh * F12_XS + kw;
    }
#pragma unroll
    for (int ii = 0; ii < 7; ++ii) {
      const int mt = wv + 8 * ii;
      if (mt >= 49) break;
      const int m = mt * 16 + col, pp = m >> 2, win = m & 3;
      const int pbase = (2 * (pp / 14) + (win >> 1)) * F12_XS + 2 * (pp % 14) + (win & 1);
      float av[7];
#pragma unroll
      for (int st = 0; st < 7; ++st) av[st] = xs[pbase + toff[st]];
      f32x4 z0 = zero_f4(), z1 = zero_f4();
#pragma unroll
      for (int st = 0; st < 7; ++st) {
        z0 = mfma16x16x4f32(av[st], bw[st][0], z0);
        z1 = mfma16x16x4f32(av[st], bw[st][1], z1);
      }
      const int pq = mt * 4 + g, ph = pq / 14, pw = pq - ph * 14;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const f32x4 z = nt ? z1 : z0;
        const float bias = nt ? bias1 : bias0;
        const int n = nt * 16 + col;
        float mx = z[0] + bias;
        int am = 0;
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          const float zz = z[r] + bias;
          if (zz > mx) { mx = zz; am = r; }
        }
        const float v = fmaxf(mx, 0.f);
        img[((n >> 2) * F2F_PLANE + (ph + 2) * F2F_W + pw + 2) * 4 + (n & 3)] = v;
        if (nh == 0) {
          const size_t o = ((size_t)b * 196 + pq) * 32 + n;
          a.p1[o] = v;
          a.idx1[o] = (uint8_t)am;
        }
      }
    }
  }
  __syncthreads();
  // 4. the W2 half (landed during conv1) into LDS, k rows per output channel
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const int i = t + 512 * j, k = i >> 3, n4 = (i & 7) * 4;
    if (i < 800 * 8) {
#pragma unroll
      for (int e = 0; e < 4; ++e) wt[(n4 + e) * F2F_WROW + k] = w2v[j][e];
    }
  }
  __syncthreads();
  // 2. the 25-tap K loop from LDS
  const int lane = t & 63, w = t >> 6, g = lane >> 4, i = lane & 15, nt = w & 1;
  int abase[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = w + 8 * j, m = (f >> 1) * 16 + i;
    int px = 0;
    if (f < 26 && m < 196) {
      const int pp = m >> 2, win = m & 3;
      px = (2 * (pp / 7) + (win >> 1)) * F2F_W + 2 * (pp % 7) + (win & 1);
    }
    abase[j] = (g * F2F_PLANE + px) * 4;
  }
  const int bbase = (nt * 16 + i) * F2F_WROW + 4 * g;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = zero_f4();
  const int n = nh * 32 + nt * 16 + i;
  const float bb = a.p32[OFF_BC2 + n];  // before the K loop: its latency hides behind the MFMAs
  if (w < 2) f32_conv2_taps<4>(img, wt, abase, bbase, acc);
  else f32_conv2_taps<3>(img, wt, abase, bbase, acc);
  // 3. bias + relu + 2x2 max pool + argmax in registers: lane's 4 rows are one pool window
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = w + 8 * j, m4 = (f >> 1) * 16 + 4 * g;
    if (f >= 26 || m4 >= 196) continue;
    float mx = acc[j][0] + bb;
    int am = 0;
#pragma unroll
    for (int r = 1; r < 4; ++r) {
      const float z = acc[j][r] + bb;
      if (z > mx) { mx = z; am = r; }
    }
    const size_t o = (size_t)b * FEAT + (m4 >> 2) * 64 + n;
    a.p2[o] = fmaxf(mx, 0.f);
    a.idx2[o] = (uint8_t)am;
  }
}

constexpr int F_BK = 32;  // K-tile of the fp32 GEMM blocks (64: 188 vs 172 us/step, fewer blocks per CU; profiles/mnist_fp32_kernels_r5.txt)

// ---------------- K4: fc1 forward, split-K slabs (reduced by the head) ----------------
// Row-major fp32 C (ld, M x N valid, N and ld multiples of 4) stored from the LDS-staged tile: thread
// i of the block stores 16-B chunks of rows (gemm_block_f32's STAGED epilogue form).
struct RowsEpiF {
  static constexpr bool STAGED = true;
  float* __restrict__ out;
  int ld, M, N;
  template <int BM, int BN, int NT>
  __device__ __forceinline__ void tile(const float* img, int P, int m0, int n0) const {
    constexpr int CPR = BN / 4;
#pragma unroll
    for (int i = threadIdx.x; i < BM * CPR; i += NT) {
      const int r = i / CPR, c = (i - r * CPR) * 4, m = m0 + r, n = n0 + c;
      if (m < M && n < N)
        *reinterpret_cast<f32x4*>(out + (size_t)m * ld + n) = *reinterpret_cast<const f32x4*>(img + r * P + c);
    }
  }
};
using SlabEpiF = RowsEpiF;
constexpr int F_FC1_SPLITS = 7;  // 3136 = 7 x 448
__global__ __launch_bounds__(256) void f32_fc1_fwd(MnistF32Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  DenseLoaderF<true> la{a.p2, FEAT, a.B, FEAT};
  DenseLoaderF<false> lb{a.p32 + OFF_WD1, HID, HID, FEAT};
  const int z = blockIdx.z, kper = FEAT / F_FC1_SPLITS;
  SlabEpiF epi{a.fc1_slab + (size_t)z * a.B * HID, HID, a.B, HID};
  gemm_block_f32<64, 64, F_BK, 2, 2>(la, lb, epi, blockIdx.y * 64, blockIdx.x * 64, z * kper, (z + 1) * kper,
                                     (float*)smem_raw);
}

// ---------------- K4..K9 head: slabs + bias + relu + dropout + FC10 + softmax-xent + dlogits/dh -------
// One block per batch row; thread t owns hidden units 4t..4t+3 (same Philox stream as the bf16 step).
__global__ __launch_bounds__(256) void f32_head(MnistF32Args a, int train) {
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n0 = 4 * t;
  // the label-independent operands first (slabs, fc1 bias, output-layer weights and bias: one memory
  // round trip), then the label chain as scalar loads beside them, the t_out store after it (the bf16
  // head kernel's order, mnist.hip)
  f32x4 p[F_FC1_SPLITS];
#pragma unroll
  for (int s = 0; s < F_FC1_SPLITS; ++s) p[s] = *reinterpret_cast<const f32x4*>(a.fc1_slab + ((size_t)s * a.B + row) * HID + n0);
  f32x4 wo[NCLS];
#pragma unroll
  for (int q = 0; q < NCLS; ++q) wo[q] = reinterpret_cast<const f32x4*>(a.p32 + OFF_OUT + (size_t)n0 * NCLS)[q];
  f32x4 h = *reinterpret_cast<const f32x4*>(a.p32 + OFF_BD1 + n0);
  float bout[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) bout[c] = a.p32[OFF_BOUT + c];
  const int64_t st = *a.step;
  const int lbl = a.labels[data_row_f(a.perm, a.step, a.n_data, a.B, row)];
  if (a.t_out && row == 0 && t == 0) *a.t_out = st + 1;
#pragma unroll
  for (int s = 0; s < F_FC1_SPLITS; ++s) h += p[s];
  float hd[4], scale[4];
  const float kp = train ? a.keep_prob : 1.0f;
  if (kp < 1.0f) {
    Philox4 r = philox4x32_10((uint32_t)(row * 256 + t), (uint32_t)st, (uint32_t)(st >> 32), a.rank, a.seed, 0x5EED1234u);
#pragma unroll
    for (int j = 0; j < 4; ++j) scale[j] = (u01(r.v[j]) < kp) ? (1.0f / kp) : 0.f;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) scale[j] = 1.f;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) hd[j] = fmaxf(h[j], 0.f) * scale[j];
#define F32_HEAD_W(j, c) wo[((j) * NCLS + (c)) >> 2][((j) * NCLS + (c)) & 3]
  float lp[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) lp[c] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int c = 0; c < NCLS; ++c) lp[c] = fmaf(hd[j], F32_HEAD_W(j, c), lp[c]);
  }
  __shared__ float red[4][NCLS];
  wave_sums_to_lane63(lp);  // DPP, interleaved over the 10 classes (was 10 shuffle-based wave sums)
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
  for (int c = 0; c < NCLS; ++c) se += expf(logit[c] - mx);
  const float lse = mx + logf(se);
  if (t == 0) {
    a.loss_row[row] = lse - logit[lbl];
    a.correct_row[row] = (am == lbl) ? 1.f : 0.f;
  }
  if (!train) return;
  const float invB = 1.0f / (float)a.B;
  float dl[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) dl[c] = (expf(logit[c] - lse) - (c == lbl ? 1.f : 0.f)) * invB;
#pragma unroll
  for (int c = 0; c < NCLS; ++c)
    if (t == c) a.dlogits[row * NCLS + c] = dl[c];
  float dhv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < NCLS; ++c) d = fmaf(dl[c], F32_HEAD_W(j, c), d);
    dhv[j] = (h[j] > 0.f) ? d * scale[j] : 0.f;
  }
#undef F32_HEAD_W
  *reinterpret_cast<f32x4*>(a.hd + (size_t)row * HID + n0) = f32x4{hd[0], hd[1], hd[2], hd[3]};
  *reinterpret_cast<f32x4*>(a.dh + (size_t)row * HID + n0) = f32x4{dhv[0], dhv[1], dhv[2], dhv[3]};
}

// ---------------- K8: output layer dW/db [1025][10] = [Hd;1]^T dlogits ----------------
constexpr int F_OUTG_ROWS = 64;
constexpr int F_OUTG_BLOCKS = (HID + 1 + F_OUTG_ROWS - 1) / F_OUTG_ROWS;  // 17
__device__ __forceinline__ void f32_out_grad_block(const MnistF32Args& a, int blk, float* smem) {
  float* dl = smem;                 // [B][10]
  float* part = smem + a.B * NCLS;  // [4][64][10]
  const int t = threadIdx.x, r = t & 63, q = t >> 6;
  for (int i = t; i < a.B * NCLS; i += 256) dl[i] = a.dlogits[i];
  __syncthreads();
  const int m = blk * F_OUTG_ROWS + r;
  float acc[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) acc[c] = 0.f;
  const int bq = (a.B + 3) >> 2, b0 = q * bq, b1 = min(a.B, b0 + bq);
  if (m < HID) {
    for (int b = b0; b < b1; ++b) {
      const float h = a.hd[(size_t)b * HID + m];
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
  for (int i = t; i < F_OUTG_ROWS * NCLS; i += 256) {
    const int rr = i / NCLS, mm = blk * F_OUTG_ROWS + rr;
    if (mm <= HID)
      a.grad[OFF_OUT + (size_t)mm * NCLS + (i - rr * NCLS)] =
          part[i] + part[F_OUTG_ROWS * NCLS + i] + part[2 * F_OUTG_ROWS * NCLS + i] + part[3 * F_OUTG_ROWS * NCLS + i];
  }
}

// ---------------- K10: fc1 dW [3137][1024] = [P2;1]^T dH, dX [B][3136] (+ unpool epilogue) ----------------
struct OnesRowMCF {  // (mn, k) = X[k][mn] for mn < mn_real, 1 for mn == mn_real (k < k_lim); 4 along mn
  static constexpr bool KC = false;
  const float* __restrict__ x;
  int ld, mn_real, k_lim;  // mn_real % 4 == 0: a chunk is all data, the ones chunk, or past the end
  __device__ __forceinline__ f32x4 operator()(int mn, int k) const {
    const f32x4 v = buf_ld_f4(x, (uint32_t)k_lim * (uint32_t)ld * 4u, (uint32_t)k * (uint32_t)ld + (uint32_t)mn,
                              mn < mn_real && k < k_lim);
    return mn == mn_real && k < k_lim ? f32x4{1.f, 0.f, 0.f, 0.f} : v;
  }
};
using GradEpiF = RowsEpiF;
// dX tile (BM batch rows x the 64 channels of ONE pooled pixel) -> dz2 through conv2's relu and the
// 2x2 pool's argmax, from the LDS-staged tile: thread (row b, 4-channel chunk) loads the relu output
// (16 B) and argmax (4 B) chunks once and writes the window as four whole 16-B chunks of dz2 (the
// fragment-order form made 16 scattered 4-B stores and 2 x 4 scalar loads per lane and value group).
struct UnpoolEpiF {
  static constexpr bool STAGED = true;
  const float* __restrict__ p2;
  const uint8_t* __restrict__ idx2;
  float* __restrict__ dz2;
  int B;
  template <int BM, int BN, int NT>
  __device__ __forceinline__ void tile(const float* img, int P, int m0, int n0) const {
    static_assert(BN == 64, "a dX tile is the 64 channels of one pooled pixel");
    const int pp = n0 >> 6, ph = pp / 7, pw = pp - ph * 7;
#pragma unroll
    for (int i = threadIdx.x; i < BM * 16; i += NT) {
      const int r = i >> 4, c = (i & 15) * 4, b = m0 + r;
      if (b >= B || pp >= 49) continue;
      const size_t o = (size_t)b * FEAT + n0 + c;
      const f32x4 v = *reinterpret_cast<const f32x4*>(img + r * P + c);
      const f32x4 pv = *reinterpret_cast<const f32x4*>(p2 + o);
      const uint32_t w4 = *reinterpret_cast<const uint32_t*>(idx2 + o);
      f32x4 g;
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] = pv[k] > 0.f ? v[k] : 0.f;  // relu output > 0
#pragma unroll
      for (int wi = 0; wi < 4; ++wi) {
        f32x4 ov;
#pragma unroll
        for (int k = 0; k < 4; ++k) ov[k] = (int)((w4 >> (8 * k)) & 0xffu) == wi ? g[k] : 0.f;
        const int oh = 2 * ph + (wi >> 1), ow = 2 * pw + (wi & 1);
        *reinterpret_cast<f32x4*>(dz2 + ((size_t)(b * 14 + oh) * 14 + ow) * 64 + c) = ov;
      }
    }
  }
};
constexpr int F_DW_GX = HID / 64, F_DW_GY = (FEAT + 1 + 63) / 64;  // 16 x 50
constexpr int F_DX_GX = FEAT / 64;                                  // 49 (x ceil(B/32))
// the dX tiles' K-tile: 64 (K = 1024 in 16 steps; ~1 block per CU, so a K-tile's MFMAs are the only
// cover for the next loads): -0.7 us/step against 32 (profiles/mnist_fp32_fc1_bk_ab_r5.log)
constexpr int F_DX_BK = 64;
// [out-layer grad blocks | dX tiles (long K first) | dW tiles]
__global__ __launch_bounds__(256) void f32_fc1_bwd(MnistF32Args a, int n_dx) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  int id = blockIdx.x;
  if (id < F_OUTG_BLOCKS) { f32_out_grad_block(a, id, (float*)smem_raw); return; }
  id -= F_OUTG_BLOCKS;
  if (id < n_dx) {
    const int bx = id % F_DX_GX, by = id / F_DX_GX;
    DenseLoaderF<true> la{a.dh, HID, a.B, HID};
    DenseLoaderF<true> lb{a.p32 + OFF_WD1, HID, FEAT, HID};
    UnpoolEpiF epi{a.p2, a.idx2, a.dz2, a.B};
    gemm_block_f32<32, 64, F_DX_BK, 2, 2>(la, lb, epi, by * 32, bx * 64, 0, HID, (float*)smem_raw);
    return;
  }
  id -= n_dx;
  const int bx = id % F_DW_GX, by = id / F_DW_GX;
  OnesRowMCF la{a.p2, FEAT, FEAT, a.B};
  DenseLoaderF<false> lb{a.dh, HID, HID, a.B};
  GradEpiF epi{a.grad + OFF_WD1, HID, FEAT + 1, HID};
  gemm_block_f32<64, 64, F_BK, 2, 2>(la, lb, epi, by * 64, bx * 64, 0, a.B, (float*)smem_raw);
}

// ---------------- K13 (LDS-staged): conv2 dgrad + conv1 relu mask, fp32 ----------------
// The bf16 step's dgrad structure (mnist.hip conv2_dgrad_body) on the fp32 matrix core. Block =
// (image b, half h: input rows ih in [7h, 7h + 7)), 512 threads. dz2 rows oh in [7h - 2, 7h + 9) are
// staged ONCE into a zero-bordered channel-chunk-major LDS image [16 chunks of 4 co][11 rows][20
// cols] x 16 B (planes padded to 224 slots); W2 streams through a double-buffered LDS ring of 5-tap
// stages ([tap*32 + ci] rows of 64 co, the 16-B chunk c of row r stored at c ^ (r & 15): the 16 rows
// of a B-fragment read hit 16 distinct bank quads). dX[p][ci] = sum_{tap, co} dz2[p - tap][co]
// W2[tap][ci][co]: M-tile = one input row (16 lanes = iw 0..15, 14 valid) so the 16 lanes of an A
// fragment read 16 consecutive slots; N = 32 (2 tiles); K = 1600 in 100 steps of 16 (read_frag4_f's K
// permutation: lane group g holds co 16q + 4g .. + 3; q = 0..3 per tap).
// 14 fragment tiles (row m, n-tile nt) = 3.5 per SIMD (SIMD s runs waves s and s + 4): waves 0-3 own
// rows {w >> 1, (w >> 1) + 2} of n-tile w & 1, waves 4-7 row 4 + ((w - 4) >> 1) plus HALF of row 6's
// tile w & 1 (co half (w >> 1) & 1: the steps q = 0, 1 or q = 2, 3 of every tap), summed through LDS
// after the loop -- 1400 MFMAs per SIMD instead of 1600 / 1200 with whole tiles.
// Replaces the generic-core dgrad that re-read the 25x-expanded im2col matrix through L2 with a
// barrier per 32-deep K-tile.
constexpr int F2D_COLS = 20, F2D_PLANE = 224, F2D_TPS = 5, F2D_NST = 25 / F2D_TPS;
constexpr int F2D_STAGE = F2D_TPS * 32 * 64;                          // floats per W2 stage (40 KB)
constexpr int F2D_SMEM = 16 * F2D_PLANE * 16 + 2 * F2D_STAGE * 4;      // 57,344 + 81,920 = 139,264 B
constexpr int F2D_BPT = F2D_STAGE / 4 / 512;                           // 16-B pieces per thread per stage
static_assert(F2D_TPS * F2D_NST == 25 && F2D_BPT * 512 * 4 == F2D_STAGE, "stage split");
// the conv1-wgrad tail's own region past the K loop's: the zero-bordered x image [32][32] and the
// half image's conv1 argmax bytes [98][32], both filled before the K loop
constexpr int F2D_XOFF = F2D_SMEM, F2D_IOFF = F2D_XOFF + 32 * 32 * 4, F2D_SMEM_T = F2D_IOFF + 98 * 32;
static_assert(F2D_SMEM_T <= 160 * 1024, "conv2 dgrad LDS carve");

// HALF < 0: both fragment tiles over all K; HALF = 0 / 1: the second tile only over q in {0, 1} / {2, 3}
template <int HALF>
__device__ __forceinline__ void f32_dgrad_stage(const float* img, const float* wb, int tap0, const int (&abase)[2],
                                                int brow, int lane, f32x4 (&acc)[2]) {
  const int g = lane >> 4, i = lane & 15;
  f32x4 a[2][2], b[2];
  auto second = [](int q) { return HALF < 0 || (q >> 1) == HALF; };
  auto load = [&](int st, int slot) {  // st = local tap * 4 + q
    const int lt = st >> 2, q = st & 3, tap = tap0 + lt, kh = tap / 5, kw = tap - 5 * kh;
    const int aoff = ((4 * q) * F2D_PLANE - kh * F2D_COLS - kw) * 4;
    a[slot][0] = *reinterpret_cast<const f32x4*>(img + abase[0] + aoff);
    if (second(q)) a[slot][1] = *reinterpret_cast<const f32x4*>(img + abase[1] + aoff);
    const int row = lt * 32 + brow;
    b[slot] = *reinterpret_cast<const f32x4*>(wb + row * 64 + (((4 * q + g) ^ i) << 2));
  };
  constexpr int NS = F2D_TPS * 4;
  load(0, 0);
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    const int cur = st & 1, q = st & 3;
    acc[0] = mfma16x16x4f32(a[cur][0][0], b[cur][0], acc[0]);
    if (second(q)) acc[1] = mfma16x16x4f32(a[cur][1][0], b[cur][0], acc[1]);
    __builtin_amdgcn_sched_barrier(0);
    if (st + 1 < NS) load(st + 1, cur ^ 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 1; s < 4; ++s) {
      acc[0] = mfma16x16x4f32(a[cur][0][s], b[cur][s], acc[0]);
      if (second(q)) acc[1] = mfma16x16x4f32(a[cur][1][s], b[cur][s], acc[1]);
    }
  }
}

__device__ __forceinline__ float part_at(const char* smem, int q, int k) {
  return reinterpret_cast<const float*>(smem)[q * (26 * 32 + 1) + k];
}
__device__ __forceinline__ void f32_conv2_dgrad_body(const MnistF32Args& a, int bid) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  float* img = reinterpret_cast<float*>(smem_raw);  // [16][224] x float4
  float* wb0 = img + 16 * F2D_PLANE * 4;             // two [160][64] W2 stages
  float* wb1 = wb0 + F2D_STAGE;
  const int b = bid >> 1, h = bid & 1, t = threadIdx.x;
  const float* w2 = a.p32 + OFF_WC2;
  f32x4 wr[F2D_BPT];
  auto gload_w = [&](int stage) {  // piece p = t + 512 j: row p >> 4, LDS chunk p & 15
#pragma unroll
    for (int j = 0; j < F2D_BPT; ++j) {
      const int p = t + 512 * j, row = p >> 4, sl = p & 15;
      wr[j] = *reinterpret_cast<const f32x4*>(w2 + (size_t)(stage * F2D_TPS * 32 + row) * 64 + ((sl ^ (row & 15)) << 2));
    }
  };
  auto sstore_w = [&](float* dst) {
#pragma unroll
    for (int j = 0; j < F2D_BPT; ++j) *reinterpret_cast<f32x4*>(dst + 4 * (t + 512 * j)) = wr[j];
  };
  gload_w(0);
  // the conv1-wgrad tail's global operands, consumed after the K loop (which reads only LDS): the x
  // image (threads < 196) and this half's argmax bytes (threads 256..451)
  f32x4 xv = zero_f4();
  uint4 iv = make_uint4(0u, 0u, 0u, 0u);
  if (t < 196) xv = reinterpret_cast<const f32x4*>(a.data + (size_t)data_row_f(a.perm, a.step, a.n_data, a.B, b) * 784)[t];
  else if (t >= 256 && t < 256 + 196) iv = reinterpret_cast<const uint4*>(a.idx1 + ((size_t)b * 196 + h * 98) * 32)[t - 256];
  float* xs = reinterpret_cast<float*>(smem_raw + F2D_XOFF);
  uint8_t* is = reinterpret_cast<uint8_t*>(smem_raw + F2D_IOFF);
  if (t < 256) reinterpret_cast<f32x4*>(xs)[t] = zero_f4();
  {
    constexpr int NI = 16 * F2D_PLANE / 512;  // 7
    const uint32_t zbytes = (uint32_t)a.B * 196u * 64u * 4u;
    f32x4 v[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int i = t + 512 * j, c = i / F2D_PLANE, q = i - c * F2D_PLANE, rr = q / F2D_COLS, cc = q - rr * F2D_COLS;
      const int r = rr + 7 * h - 2, col = cc - 2;
      const bool ok = q < 11 * F2D_COLS && (unsigned)r < 14u && (unsigned)col < 14u;
      v[j] = buf_ld_f4(a.dz2, zbytes, (uint32_t)(((b * 14 + r) * 14 + col) * 64 + 4 * c), ok);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) *reinterpret_cast<f32x4*>(img + 4 * (t + 512 * j)) = v[j];
  }
  sstore_w(wb0);
  __syncthreads();
  const int lane = t & 63, w = t >> 6, g = lane >> 4, i = lane & 15, nt = w & 1;
  // this wave's two rows: waves 0-3 rows w >> 1 and (w >> 1) + 2, waves 4-7 row 4 + ((w - 4) >> 1)
  // and (half of) row 6
  const int r0 = w < 4 ? (w >> 1) : 4 + ((w - 4) >> 1), r1 = w < 4 ? (w >> 1) + 2 : 6;
  const int abase[2] = {(g * F2D_PLANE + (r0 + 4) * F2D_COLS + i + 4) * 4, (g * F2D_PLANE + (r1 + 4) * F2D_COLS + i + 4) * 4};
  const int brow = nt * 16 + i;
  // conv1's relu outputs that mask this lane's dX values
  float p1pre[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      p1pre[j][e] = a.p1[((size_t)b * 196 + (7 * h + (j ? r1 : r0)) * 14 + min(4 * g + e, 13)) * 32 + nt * 16 + i];
  f32x4 acc[2] = {zero_f4(), zero_f4()};
  const int role = w < 4 ? -1 : ((w >> 1) & 1);
  for (int stg = 0; stg < F2D_NST; ++stg) {
    if (stg + 1 < F2D_NST) gload_w(stg + 1);
    const float* wb = (stg & 1) ? wb1 : wb0;
    if (role < 0) f32_dgrad_stage<-1>(img, wb, stg * F2D_TPS, abase, brow, lane, acc);
    else if (role == 0) f32_dgrad_stage<0>(img, wb, stg * F2D_TPS, abase, brow, lane, acc);
    else f32_dgrad_stage<1>(img, wb, stg * F2D_TPS, abase, brow, lane, acc);
    if (stg + 1 < F2D_NST) sstore_w((stg & 1) ? wb0 : wb1);
    __syncthreads();
  }
  // the tail's x image and argmax bytes into LDS only now (their own regions, untouched by the K
  // loop): stored before it, the x row's dependent chain (step -> perm -> x) and the relu bytes held
  // waves 0-3 at the first K stage; the empty asm uses keep the relu compares from being hoisted to
  // right after their loads for the same reason
  if (t < 196) {  // x into the zero-bordered image (zeroed before the first barrier)
    const int r = (4 * t) / 28, c = (4 * t) % 28;
    float* d = xs + (r + 2) * 32 + c + 2;
    d[0] = xv[0]; d[1] = xv[1]; d[2] = xv[2]; d[3] = xv[3];
  } else if (t >= 256 && t < 256 + 196) {
    reinterpret_cast<uint4*>(is)[t - 256] = iv;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(p1pre[j][e]));
  // row 6: waves 6, 7 (co half 1) park their partial tile, waves 4, 5 (co half 0) add it
  f32x4* park = reinterpret_cast<f32x4*>(smem_raw);  // the dz2 image is dead
  if (w >= 6) park[(w - 6) * 64 + lane] = acc[1];
  __syncthreads();
  if (w == 4 || w == 5) acc[1] += park[(w - 4) * 64 + lane];
  // K15 + K12 tail: conv1 weight + bias gradient of this half image. dX through conv1's relu mask
  // (p1 > 0) is the pooled conv1 gradient; it reaches the conv1 output pixel at its window's argmax
  // only (MaxPoolGrad), so dW1[kh][kw][c] = sum over the 98 pooled pixels of g * x[argmax pixel + tap].
  float* gs = wb0;  // [98][32] masked dX (the W2 ring is dead)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j == 1 && w >= 6) break;
    const int lr = j ? r1 : r0, ci = nt * 16 + i;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int iw = 4 * g + e;
      if (iw >= 14) break;
      gs[(lr * 14 + iw) * 32 + ci] = p1pre[j][e] > 0.f ? acc[j][e] : 0.f;
    }
  }
  __syncthreads();
  {
    const int c = t & 31, sub = t >> 5;  // 16 pixel slices
    float a1[26];
#pragma unroll
    for (int k = 0; k < 26; ++k) a1[k] = 0.f;
    for (int lp = sub; lp < 98; lp += 16) {  // no zero skip: time must not depend on values
      const float gv = gs[lp * 32 + c];
      const int pp = h * 98 + lp, wi = is[lp * 32 + c];
      const int oh = 2 * (pp / 14) + (wi >> 1), ow = 2 * (pp % 14) + (wi & 1);
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) a1[kh * 5 + kw] = fmaf(gv, xs[(oh + kh) * 32 + ow + kw], a1[kh * 5 + kw]);
      a1[25] += gv;
    }
    float* part = reinterpret_cast<float*>(smem_raw);  // [16][26*32 + 1] (the dz2 image / park are dead)
#pragma unroll
    for (int k = 0; k < 26; ++k) part[sub * (26 * 32 + 1) + k * 32 + c] = a1[k];
  }
  __syncthreads();
  for (int k = t; k < 26 * 32; k += 512) {
    float sm = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) sm += part_at(smem_raw, q, k);
    a.wg1_slab[(size_t)bid * 832 + k] = sm;
  }
}

// ---------------- K14 (LDS-staged): conv2 wgrad (+ K12 bias row), fp32 ----------------
// The bf16 step's wgrad structure (mnist.hip conv2_wgrad_body). Block = (tap group tg, image pair ip),
// 512 threads; 4 x 64 = 256 blocks at B = 128. Per image: p1 (14x14x32) into a zero-bordered LDS image
// [18][18] positions x 48-float channel stride and dz2 (196 x 64) into LDS rows of 80 floats; then
// dW[tap*32 + ci][co] += sum_px p1[px + tap][ci] dz2[px][co] on the fp32 matrix core: K = the image's
// 196 pixels (49 MFMA k-steps of 4, lane group g = pixel 4kk + g), so the im2col shift of a tap is a
// per-lane position offset and every operand is one conflict-free scalar LDS read (16 lanes = 16
// consecutive channels; the 4 pixel groups land 16 banks apart: strides 48 and 80 = 48 / 16 mod 64
// per position / pixel). Wave w owns ci-tile w >> 2, co-tile w & 3 and every tap of its group (6, the
// last 7): one B read feeds 6-7 MFMAs. One fp32 slab per image pair (rows of its tap group; tap group 0
// also the bias row 800), reduced by the optimizer tail. Image ii + 1's global loads are issued before
// image ii's MFMAs. Replaces the im2col GEMM that re-read p1 25x through L2.
// 2 images x 4 tap groups: 4 x 4 / 4 x 6 / 4 x 8 / 2 x 6 were +1.6 ... +8.5 us (profiles/mnist_conv2_wgrad_grouping_r6.log)
constexpr int F2W_NTG = 4, F2W_TPG = 25 / F2W_NTG, F2W_MAXT = 25 - F2W_TPG * (F2W_NTG - 1);  // 6 / 7
constexpr int F2W_IMG = 2, F2W_PW = 18, F2W_CS = 48, F2W_DS = 80;
constexpr int F2W_IMG_F = F2W_PW * F2W_PW * F2W_CS;        // 15,552 floats
constexpr int F2W_DZ_F = 196 * F2W_DS;                     // 15,680 floats
constexpr int F2W_SMEM = (F2W_IMG_F + F2W_DZ_F + 8 * 64) * 4;  // 126,976 B
static_assert(F2W_SMEM <= F2D_SMEM, "one LDS size for both block kinds of the launch");
constexpr int F2W_N1 = (196 * 8 + 511) / 512, F2W_N2 = (196 * 16 + 511) / 512;  // 4, 7 float4 per thread

__device__ __forceinline__ void f32_conv2_wgrad_body(const MnistF32Args& a, int bid) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  float* img = reinterpret_cast<float*>(smem_raw);
  float* dz = img + F2W_IMG_F;
  float* bred = dz + F2W_DZ_F;  // [8][64]
  const int tg = bid % F2W_NTG, ip = bid / F2W_NTG, t = threadIdx.x;
  const int tap0 = tg * F2W_TPG, ntaps = (tg == F2W_NTG - 1) ? F2W_MAXT : F2W_TPG;
  const int lane = t & 63, w = t >> 6, cit = w >> 2, ct = w & 3, g = lane >> 4, i = lane & 15;
  f32x4 v1[F2W_N1], v2[F2W_N2];
  auto gload = [&](int b) {
    const f32x4* s1 = reinterpret_cast<const f32x4*>(a.p1 + (size_t)b * 196 * 32);
    const f32x4* s2 = reinterpret_cast<const f32x4*>(a.dz2 + (size_t)b * 196 * 64);
#pragma unroll
    for (int j = 0; j < F2W_N1; ++j) { const int k = t + 512 * j; v1[j] = k < 196 * 8 ? s1[k] : zero_f4(); }
#pragma unroll
    for (int j = 0; j < F2W_N2; ++j) { const int k = t + 512 * j; v2[j] = k < 196 * 16 ? s2[k] : zero_f4(); }
  };
  if (ip * F2W_IMG < a.B) gload(ip * F2W_IMG);
  // the image border stays zero for every image of the block
  for (int k = t; k < F2W_PW * F2W_PW; k += 512) {
    const int r = k / F2W_PW, c = k - r * F2W_PW;
    if (r < 2 || r >= 16 || c < 2 || c >= 16) {
      f32x4* d = reinterpret_cast<f32x4*>(img + k * F2W_CS);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = zero_f4();
    }
  }
  f32x4 acc[F2W_MAXT];
#pragma unroll
  for (int j = 0; j < F2W_MAXT; ++j) acc[j] = zero_f4();
  float bsum = 0.f;
  for (int ii = 0; ii < F2W_IMG; ++ii) {
    const int b = ip * F2W_IMG + ii;
    if (b >= a.B) break;
    __syncthreads();  // the previous image's operands are consumed
#pragma unroll
    for (int j = 0; j < F2W_N1; ++j) {
      const int k = t + 512 * j;
      if (k < 196 * 8) {
        const int px = k >> 3, ch = k & 7, r = px / 14, c = px - r * 14;
        *reinterpret_cast<f32x4*>(img + ((r + 2) * F2W_PW + c + 2) * F2W_CS + ch * 4) = v1[j];
      }
    }
#pragma unroll
    for (int j = 0; j < F2W_N2; ++j) {
      const int k = t + 512 * j;
      if (k < 196 * 16) *reinterpret_cast<f32x4*>(dz + (k >> 4) * F2W_DS + (k & 15) * 4) = v2[j];
    }
    __syncthreads();
    if (ii + 1 < F2W_IMG && b + 1 < a.B) gload(b + 1);
    if (tg == 0) {  // bias row: column sums of dz2 (pixel slice t >> 6 of 8)
      for (int px = t >> 6; px < 196; px += 8) bsum += dz[px * F2W_DS + (t & 63)];
    }
    auto operands = [&](int kk, float& bv, float (&av)[F2W_MAXT]) {
      const int px = 4 * kk + g, oh = px / 14, ow = px - oh * 14;
      bv = dz[px * F2W_DS + ct * 16 + i];
      const float* ap = img + (oh * F2W_PW + ow) * F2W_CS + cit * 16 + i;
#pragma unroll
      for (int j = 0; j < F2W_MAXT; ++j) {
        const int tap = tap0 + (j < ntaps ? j : 0), kh = tap / 5, kw = tap - 5 * kh;
        av[j] = ap[(kh * F2W_PW + kw) * F2W_CS];
      }
    };
    float bv[2], av[2][F2W_MAXT];
    operands(0, bv[0], av[0]);
#pragma unroll
    for (int kk = 0; kk < 49; ++kk) {
      const int cur = kk & 1;
      acc[0] = mfma16x16x4f32(av[cur][0], bv[cur], acc[0]);
      __builtin_amdgcn_sched_barrier(0);
      if (kk + 1 < 49) operands(kk + 1, bv[cur ^ 1], av[cur ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 1; j < F2W_MAXT; ++j)
        if (j < ntaps) acc[j] = mfma16x16x4f32(av[cur][j], bv[cur], acc[j]);
    }
  }
  float* slab = a.wg2_slab + (size_t)ip * 801 * 64;
#pragma unroll
  for (int j = 0; j < F2W_MAXT; ++j) {
    if (j < ntaps) {
      const int tap = tap0 + j;
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(size_t)(tap * 32 + cit * 16 + 4 * g + r) * 64 + ct * 16 + i] = acc[j][r];
    }
  }
  if (tg == 0) {
    bred[(t >> 6) * 64 + (t & 63)] = bsum;
    __syncthreads();
    if (t < 64) {
      float sm = 0.f;
#pragma unroll
      for (int sl = 0; sl < 8; ++sl) sm += bred[sl * 64 + t];
      slab[800 * 64 + t] = sm;
    }
  }
}

// conv2 wgrad (blocks [0, nw)) and dgrad in ONE launch: both consume only dz2, and one LDS size
// (one block per CU) lets each CU run a dgrad block as soon as its wgrad block is done
__global__ __launch_bounds__(512) void f32_conv2_bwd_lds(MnistF32Args a, int nw) {
  if ((int)blockIdx.x < nw) f32_conv2_wgrad_body(a, blockIdx.x);
  else f32_conv2_dgrad_body(a, blockIdx.x - nw);
}

template <auto K>
inline void set_smem_f(int bytes) {
  static bool done = false;
  if (!done && bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(K), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  done = true;
}

}  // namespace

int mnist_f32_fc1_splits() { return F_FC1_SPLITS; }
int mnist_f32_wg2_splits(int B) { return (B + F2W_IMG - 1) / F2W_IMG; }  // one slab per image pair

void mnist_f32_forward(const MnistF32Args& a, bool train, hipStream_t s) {
  const int B = a.B;
  set_smem_f<f32_conv12_fwd_lds>(F2F_SMEM);
  f32_conv12_fwd_lds<<<2 * B, 512, F2F_SMEM, s>>>(a);
  {
    constexpr int sm = GemmSmemF<64, 64, F_BK, DenseLoaderF<true>, DenseLoaderF<false>>::BYTES;
    set_smem_f<f32_fc1_fwd>(sm);
    f32_fc1_fwd<<<dim3(HID / 64, (B + 63) / 64, F_FC1_SPLITS), 256, sm, s>>>(a);
  }
  f32_head<<<B, 256, 0, s>>>(a, train ? 1 : 0);
}

void mnist_f32_backward(const MnistF32Args& a, hipStream_t s) {
  const int B = a.B;
  {
    constexpr int sm_dw = GemmSmemF<64, 64, F_BK, OnesRowMCF, DenseLoaderF<false>>::BYTES;
    constexpr int sm_dx = GemmSmemF<32, 64, F_DX_BK, DenseLoaderF<true>, DenseLoaderF<true>>::BYTES;
    const int sm_og = (B * NCLS + 4 * F_OUTG_ROWS * NCLS) * 4;
    const int sm = std::max(std::max(sm_dw, sm_dx), sm_og);
    set_smem_f<f32_fc1_bwd>(sm);
    const int n_dx = F_DX_GX * ((B + 31) / 32);
    f32_fc1_bwd<<<F_OUTG_BLOCKS + n_dx + F_DW_GX * F_DW_GY, 256, sm, s>>>(a, n_dx);
  }
  set_smem_f<f32_conv2_bwd_lds>(F2D_SMEM_T);
  const int nw = F2W_NTG * a.wg2_splits;
  f32_conv2_bwd_lds<<<nw + 2 * B, 512, F2D_SMEM_T, s>>>(a, nw);
}

}  // namespace tfd
