// Generic NHWC implicit-GEMM convolution (forward / input-gradient / weight-gradient) and dense
// layers on MFMA (bf16 operands, fp32 accumulate) for the ResNet-style model family of
// BASELINE.json configs 4-5 (strided 7x7 / 3x3 / 1x1 convs).
//
// Layouts (TF conventions, like the reference): activations NHWC bf16, filters HWIO
// ([R][S][C][K] == [R*S*C][K]) bf16, weight gradients fp32 (the flat optimizer buffer).
//   fwd  : Y[m=(n,ho,wo)][k]  = sum_{t=(r,s,c)} X[n, ho*st-pad+r, wo*st-pad+s, c] * W[t][k]
//   dgrad: dX[m=(n,h,w)][c]   = sum_{(r,s,k)} dY[n, (h+pad-r)/st, (w+pad-s)/st, k] * W[r][s][c][k]
//          (taps whose (h+pad-r) or (w+pad-s) is not a multiple of st contribute zero)
//   wgrad: dW[t=(r,s,c)][k]  += sum_{m} X[n, ho*st-pad+r, wo*st-pad+s, c] * dY[m][k]   (split-K
//          over pixels; fp32 atomics only when split, plain stores otherwise)
// All index math on the loaders' hot path uses multiply-shift division (FastDiv) by runtime
// constants. C and K must be multiples of 8 (16-B chunks); the 3-channel stem input is padded to 8.
// 1x1 / stride-1 / pad-0 convolutions are plain GEMMs and take the dense loaders.
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "../common.h"
#include "../conv_kernels.h"
#include "../gemm.h"
#include "../gemm256.h"
#include "../bn_affine.h"

namespace tfd {
namespace {

// n / d for 0 <= n < 2^31 with a runtime divisor (libdivide "round-up + add" variant)
struct FastDiv {
  uint32_t d, m, s;
  __host__ __device__ FastDiv() : d(1), m(0), s(0) {}
  __host__ explicit FastDiv(uint32_t div) : d(div) {
    s = 0;
    while ((1ull << s) < div) ++s;
    m = (uint32_t)(((1ull << 32) * ((1ull << s) - div)) / div + 1);
    if (div == 1) { m = 0; s = 0; }
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    const uint64_t hi = ((uint64_t)n * m) >> 32;
    return (uint32_t)((hi + n) >> s);
  }
};

struct Geo {
  int N, H, W, C, K, R, S, st, pad, Ho, Wo;
  int stw, padw;  // width stride / left pad (= st / pad except for the width-paired stem)
  int M;       // rows of the GEMM
  int KD;      // reduction length
  uint32_t xbytes, ybytes, wbytes;  // buffer-descriptor ranges of input, output(-gradient), filter
  FastDiv howo, wo, c, k, s, hw, w;
};

// Every loader below is BRANCH-FREE: one raw buffer load (a descriptor over the whole operand,
// built from kernel arguments, so scalar) per 16-B chunk, and an out-of-range chunk gets an offset
// past the descriptor's range, which the hardware range check returns as zeros. With a plain load
// under `if (in range)` the compiler emits an exec-masked branch per load and cannot count the
// loads in flight across the joins, so a deeper register pipeline (TFD_CONV_RS > 1) degenerated to
// vmcnt(0) waits (measured: ResNet-50 b128 19.6 -> 24.5 ms/step at RS = 2).
// (buf_ld: csrc/gemm.h)

// Row-major X[rows][ld] bf16 with whole 16-B chunks (lims and ld multiples of 8; host-checked):
//  KC=true : (mn, k) = X[mn][k];  KC=false: (mn, k) = X[k][mn]
// Every loader also exposes rsrc() + off(mn, k) (byte offset of the chunk, or past the range): the
// 256-row core (csrc/gemm256.h) DMAs the same chunks straight into LDS.
__device__ __forceinline__ uint4 rsrc_ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const i32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_uint4((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]);
}
__device__ __forceinline__ uint32_t boff(uint32_t elem, bool ok) { return ok ? elem * 2u : kBufOOB; }
#define TFD_LOADER_CALL                                                                        \
  __device__ __forceinline__ uint4 operator()(int mn, int k) const { return rsrc_ld(rsrc(), off(mn, k)); }

template <bool KC_>
struct DenseX {
  static constexpr bool KC = KC_;
  const uint16_t* __restrict__ x;
  int ld, mn_lim, k_lim;
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    return make_rsrc(x, (uint32_t)(KC ? mn_lim : k_lim) * (uint32_t)ld * 2u);
  }
  __device__ __forceinline__ uint32_t off(int mn, int k) const {
    const bool ok = mn < mn_lim && k < k_lim;
    return boff(KC ? (uint32_t)mn * ld + k : (uint32_t)k * ld + mn, ok);
  }
  __device__ __forceinline__ int chan(int mn, int k) const { return KC ? k : mn; }  // [pixel][channel] operands
  TFD_LOADER_CALL
};

// ---- forward: A = im2col(X) (KC), B = W [KD][K] (not KC) ----
struct FwdA {
  static constexpr bool KC = true;
  const uint16_t* __restrict__ x;
  Geo g;
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return make_rsrc(x, g.xbytes); }
  __device__ __forceinline__ uint32_t off(int m, int k) const {
    const int n = g.howo.div(m), r1 = m - n * g.Ho * g.Wo, ho = g.wo.div(r1), wo = r1 - ho * g.Wo;
    const int tap = g.c.div(k), c = k - tap * g.C, r = g.s.div(tap), s = tap - r * g.S;
    const int h = ho * g.st - g.pad + r, w = wo * g.stw - g.padw + s;
    const bool ok = m < g.M && k < g.KD && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
    return boff((uint32_t)((n * g.H + h) * g.W + w) * g.C + c, ok);
  }
  __device__ __forceinline__ int chan(int m, int k) const { return k - g.c.div(k) * g.C; }
  TFD_LOADER_CALL
};

// ---- dgrad: A = "col2im" gather of dY (KC), B = W as [C][(r,s,k)] (KC) ----
struct DgradA {
  static constexpr bool KC = true;
  const uint16_t* __restrict__ dy;
  Geo g;  // M = N*H*W, KD = R*S*K
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return make_rsrc(dy, g.ybytes); }
  TFD_LOADER_CALL
  __device__ __forceinline__ uint32_t off(int m, int kk) const {
    const int n = g.hw.div(m), r1 = m - n * g.H * g.W, h = g.w.div(r1), w = r1 - h * g.W;
    const int tap = g.k.div(kk), k = kk - tap * g.K, r = g.s.div(tap), s = tap - r * g.S;
    const int hn = h + g.pad - r, wn = w + g.pad - s;
    bool ok = m < g.M && kk < g.KD && hn >= 0 && wn >= 0;
    int ho = hn, wo = wn;
    if (g.st != 1) {  // uniform branch, no load inside
      ho = hn / g.st;
      wo = wn / g.st;
      ok = ok && ho * g.st == hn && wo * g.st == wn;
    }
    ok = ok && ho < g.Ho && wo < g.Wo;
    return boff((uint32_t)((n * g.Ho + ho) * g.Wo + wo) * g.K + k, ok);
  }
};
struct DgradB {
  static constexpr bool KC = true;
  const uint16_t* __restrict__ w;
  Geo g;
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return make_rsrc(w, g.wbytes); }
  __device__ __forceinline__ uint32_t off(int c, int kk) const {
    const int tap = g.k.div(kk), k = kk - tap * g.K;
    return boff((uint32_t)(tap * g.C + c) * g.K + k, c < g.C && kk < g.KD);
  }
  TFD_LOADER_CALL
};

// ---- strided dgrad, one output phase (h % st, w % st) at a time ----
// Input pixel (h, w) = (hh*st + ph, ww*st + pw) receives exactly the taps r = r0 + i*st
// (r0 = (ph + pad) % st), s = s0 + j*st, each from dY[ho = hh + dh - i][wo = ww + dw - j] with
// dh = (ph + pad - r0) / st: a dense implicit GEMM over the phase grid with KD = nr*ns*K and no
// zero taps (the plain DgradA gathers st^2 x more MFMA work, 3/4 of it on zeros at st = 2).
struct PhaseGeo {
  int N, Hp, Wp, Ho, Wo, K, C, st, ph, pw, H, W;
  int r0, s0, nr, ns, dh, dw;
  int M, KD;
  uint32_t ybytes, wbytes;
  FastDiv hpwp, wp, k, nsd;
};
struct DgradPhaseA {
  static constexpr bool KC = true;
  const uint16_t* __restrict__ dy;
  PhaseGeo g;
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return make_rsrc(dy, g.ybytes); }
  __device__ __forceinline__ uint32_t off(int m, int kk) const {
    const int n = g.hpwp.div(m), r1 = m - n * g.Hp * g.Wp, hh = g.wp.div(r1), ww = r1 - hh * g.Wp;
    const int t = g.k.div(kk), k = kk - t * g.K, i = g.nsd.div(t), j = t - i * g.ns;
    const int ho = hh + g.dh - i, wo = ww + g.dw - j;
    const bool ok = m < g.M && kk < g.KD && (unsigned)ho < (unsigned)g.Ho && (unsigned)wo < (unsigned)g.Wo;
    return boff((uint32_t)((n * g.Ho + ho) * g.Wo + wo) * g.K + k, ok);
  }
  TFD_LOADER_CALL
};
struct DgradPhaseB {  // (c, kk) -> W[r][s][c][k], S = filter width
  static constexpr bool KC = true;
  const uint16_t* __restrict__ w;
  PhaseGeo g;
  int S;
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return make_rsrc(w, g.wbytes); }
  __device__ __forceinline__ uint32_t off(int c, int kk) const {
    const int t = g.k.div(kk), k = kk - t * g.K, i = g.nsd.div(t), j = t - i * g.ns;
    const int r = g.r0 + i * g.st, s = g.s0 + j * g.st;
    return boff((uint32_t)((r * S + s) * g.C + c) * g.K + k, c < g.C && kk < g.KD);
  }
  TFD_LOADER_CALL
};
struct PhaseRows {  // phase GEMM row -> pixel row of dX
  PhaseGeo g;
  __device__ __forceinline__ uint32_t operator()(int m) const {
    if (m >= g.M) return 0u;
    const int n = g.hpwp.div(m), r1 = m - n * g.Hp * g.Wp, hh = g.wp.div(r1), ww = r1 - hh * g.Wp;
    return (uint32_t)((n * g.H + hh * g.st + g.ph) * g.W + ww * g.st + g.pw);
  }
};

// ---- wgrad: A = im2col(X)^T (not KC: chunk of 8 channels at one pixel), B = dY [pix][K] ----
struct WgradA {
  static constexpr bool KC = false;
  const uint16_t* __restrict__ x;
  Geo g;  // M = R*S*C rows (taps), KD = N*Ho*Wo pixels
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return make_rsrc(x, g.xbytes); }
  __device__ __forceinline__ uint32_t off(int t, int m) const {
    const int tap = g.c.div(t), c = t - tap * g.C, r = g.s.div(tap), s = tap - r * g.S;
    const int n = g.howo.div(m), r1 = m - n * g.Ho * g.Wo, ho = g.wo.div(r1), wo = r1 - ho * g.Wo;
    const int h = ho * g.st - g.pad + r, w = wo * g.stw - g.padw + s;
    const bool ok = t < g.M && m < g.KD && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
    return boff((uint32_t)((n * g.H + h) * g.W + w) * g.C + c, ok);
  }
  __device__ __forceinline__ int chan(int t, int m) const { return t - g.c.div(t) * g.C; }
  TFD_LOADER_CALL
};

// ---- the producing layer's batch norm + relu, applied while staging (the forward BN fold) ----
// A conv whose input is relu(bn(y)) of a single-consumer batch norm reads y itself and stages
// relu(fmaf(y, sc, sh)) rounded to bf16 (bn_affine constants) -- bit for bit the bn_apply_kernel
// output, which is then never written: one full read + write pass per such BN disappears, and the
// weight gradient of the same conv rebuilds its X operand the same way. Chunks the loader zero-fills
// (padding taps, tails) stay zero (tag -1). The per-channel (sc, sh) pairs live in an LDS table the
// block builds once (gemm_mainloop's LoaderXF hook); C <= kBnReluMaxC.
struct BnReluArgs {
  const float *mean, *invstd, *gamma, *beta;
  int C;
};
template <class L>
struct BnRelu : L {
  static constexpr int XF_BYTES = kBnReluMaxC * 8;
  BnReluArgs bn;
  // table: [C/2] x {sc[2i], sc[2i+1], sh[2i], sh[2i+1]} (one float4 per channel pair: bn_relu2 operands)
  __device__ __forceinline__ void stage(char* tab) const {
    float4* t = reinterpret_cast<float4*>(tab);
    for (int i = threadIdx.x; 2 * i < bn.C; i += blockDim.x) {
      float4 e;
      bn_affine(bn.mean[2 * i], bn.invstd[2 * i], bn.gamma[2 * i], bn.beta[2 * i], e.x, e.z);
      bn_affine(bn.mean[2 * i + 1], bn.invstd[2 * i + 1], bn.gamma[2 * i + 1], bn.beta[2 * i + 1], e.y, e.w);
      t[i] = e;
    }
  }
  __device__ __forceinline__ uint4 load(int mn, int k, int& tag) const {
    const uint32_t o = this->off(mn, k);
    tag = o == kBufOOB ? -1 : this->chan(mn, k);
    return rsrc_ld(this->rsrc(), o);
  }
  // all N chunks of a thread share one 8-channel group (gemm_mainloop asserts the layout), so the
  // group's constants are read once per K-tile: 4 ds_read_b128, then 24 VALU per chunk
  template <int N>
  __device__ __forceinline__ void xform(uint4 (&v)[N], const int (&tag)[N], const char* tab) const {
    int ch = tag[0];
#pragma unroll
    for (int c = 1; c < N; ++c) ch = max(ch, tag[c]);
    const float4* t = reinterpret_cast<const float4*>(tab) + (max(ch, 0) >> 1);
    const float4 t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3];
#pragma unroll
    for (int c = 0; c < N; ++c) {
      uint4 o;
      o.x = bn_relu2(v[c].x, (bn_f32x2){t0.x, t0.y}, (bn_f32x2){t0.z, t0.w});
      o.y = bn_relu2(v[c].y, (bn_f32x2){t1.x, t1.y}, (bn_f32x2){t1.z, t1.w});
      o.z = bn_relu2(v[c].z, (bn_f32x2){t2.x, t2.y}, (bn_f32x2){t2.z, t2.w});
      o.w = bn_relu2(v[c].w, (bn_f32x2){t3.x, t3.y}, (bn_f32x2){t3.z, t3.w});
      v[c] = tag[c] < 0 ? make_uint4(0u, 0u, 0u, 0u) : o;
    }
  }
};

// ---- epilogues ----
struct StoreBf16 {  // Y[m][n] bf16, ld = N
  uint16_t* __restrict__ y;
  int M, N;
  __device__ __forceinline__ void operator()(int m4, int n, f32x4 v) const {
    if (n >= N) return;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (m4 + r < M) y[(size_t)(m4 + r) * N + n] = f2bf_bits(v[r]);
  }
};
struct AddStoreBf16 {  // Y[m][n] bf16 = v + A[m][n] (fp32 add, one rounding). A and Y are distinct
  uint16_t* __restrict__ y;  // buffers: no aliasing, so the unrolled epilogue issues every load of A
  const uint16_t* __restrict__ add;  // before its stores instead of one load->store round trip each
  int M, N;
  __device__ __forceinline__ void operator()(int m4, int n, f32x4 v) const {
    if (n >= N) return;
    float a[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] = m4 + r < M ? bf2f(add[(size_t)(m4 + r) * N + n]) : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (m4 + r < M) y[(size_t)(m4 + r) * N + n] = f2bf_bits(v[r] + a[r]);
  }
};
struct BiasStoreF32 {  // out[m][n] fp32 = v + bias[n] (dense layer logits)
  float* __restrict__ y;
  const float* __restrict__ bias;
  int M, N;
  __device__ __forceinline__ void operator()(int m4, int n, f32x4 v) const {
    if (n >= N) return;
    const float b = bias ? bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (m4 + r < M) y[(size_t)(m4 + r) * N + n] = v[r] + b;
  }
};
struct AccF32 {  // dW[m][n] fp32: += (atomic, split-K) or = (single split)
  float* __restrict__ y;
  int M, N, atomic;
  __device__ __forceinline__ void operator()(int m4, int n, f32x4 v) const {
    if (n >= N) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (m4 + r >= M) break;
      float* p = y + (size_t)(m4 + r) * N + n;
      if (atomic) atomicAdd(p, v[r]);
      else *p = v[r];
    }
  }
};

// Forward conv epilogue + batch-norm statistics: bf16 store, and per-column sums of the STORED
// (bf16-rounded) values -- exactly what bn_partial_kernel would read back -- accumulated in the
// calling lane's registers (WANTS_IJ: j is the compile-time column-tile index after unrolling).
template <int TN>
struct StoreBf16Stats {
  static constexpr bool WANTS_IJ = true;
  uint16_t* __restrict__ y;
  int M, N;
  float* s;  // [TN] per-lane column sums
  float* q;  // [TN] per-lane column sums of squares
  __device__ __forceinline__ void operator()(int m4, int n, f32x4 v, int i, int j) const {
    (void)i;
    if (n >= N) return;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (m4 + r < M) {
        const uint16_t b = f2bf_bits(v[r]);
        y[(size_t)(m4 + r) * N + n] = b;
        const float f = bf2f(b);
        s[j] += f;
        q[j] = fmaf(f, f, q[j]);
      }
  }
};

// Residual-join add operand of a bf16-output epilogue: x[m][n] bf16, or -- bits != nullptr -- the
// gradient through a residual batch norm's relu, x = that BN's dout and bits = the forward's relu
// bits ([M][N/8] bytes): the masked dout is exactly the dres bn_bwd would have written (a bf16 value
// or zero), so the BN backward skips that full-tensor write (ResNet identity shortcuts).
// sub_w != 0: x lives on the stride-2 grid [N][Ho][Wo][C] of the output's [N][sub_h][sub_w] pixels --
// a downsample block's 1x1 stride-2 shortcut dgrad, whose other three phases are zero -- and is added
// at the even (h, w) pixels only (abytes: its size), so those zeros are never written nor read.
struct AddSrc {
  const uint16_t* x = nullptr;
  const uint8_t* bits = nullptr;
  uint32_t sub_w = 0, sub_h = 0, sub_wo = 0, sub_ho = 0, abytes = 0;
  __host__ __device__ AddSrc() {}
  __host__ __device__ AddSrc(const uint16_t* p) : x(p) {}  // NOLINT: plain add operand
  __host__ __device__ AddSrc(const uint16_t* p, const uint8_t* b) : x(p), bits(b) {}
};
// row of the add operand for output row `row`; clears ok where a stride-2 operand has no value
__device__ __forceinline__ uint32_t add_row(const AddSrc& a, uint32_t row, bool& ok) {
  if (!a.sub_w) return row;
  const uint32_t w = row % a.sub_w, hw = row / a.sub_w, h = hw % a.sub_h, img = hw / a.sub_h;
  ok = ok && !(w & 1u) && !(h & 1u);
  return (img * a.sub_ho + (h >> 1)) * a.sub_wo + (w >> 1);
}
__device__ __forceinline__ uint4 add_masked(uint4 q, uint32_t bits) {  // bit j keeps element j
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
  uint32_t o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    o[k] = ((bits >> (2 * k)) & 1u ? w[k] & 0xFFFFu : 0u) | ((bits >> (2 * k + 1)) & 1u ? w[k] & 0xFFFF0000u : 0u);
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// ---- LDS-staged epilogue (bf16 outputs) ----
// The fragment-order epilogues above store 2 B per lane in 4 row-strided 32-B pieces per wave
// instruction, and AddStoreBf16 serialises its scalar residual loads on memory latency (the
// residual-join dgrad measured 3.6x slower with it). Here the block's fp32 accumulator tile goes to
// LDS (row-major, pitch BN + 4 floats: the 4 row groups of a fragment store land 16 banks apart),
// then every thread owns whole 8-column chunks: its residual chunks are loaded with 16-B buffer
// loads issued BEFORE the accumulator is staged, and each output chunk leaves as ONE 16-B store, so
// a wave writes whole 128-B lines. The sum v + add is formed in fp32 and rounded once (bit-identical
// to AddStoreBf16). STATS: per-column sums / sums of squares of the stored (bf16-rounded) values,
// fixed summation order (deterministic), written to part[blockIdx.y][2][N].
template <int BM, int BN, int WM, int WN>
struct LdsEpi {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int PITCH = BN + 4;            // floats
  static constexpr int CPR = BN / 8;              // 8-column chunks per row
  static constexpr int CH = BM * CPR / NT;        // chunks per thread
  static constexpr int RG = NT / CPR;             // row groups (threads sharing a chunk column)
  static constexpr int BYTES = BM * PITCH * 4;
  static_assert(BM * CPR % NT == 0 && NT % CPR == 0, "whole chunks per thread");
};
// GEMM row m -> output row (identity; the strided-dgrad phase GEMMs scatter to every st-th pixel; the
// halo-tile convs map tile rows to pixels and mark those past the image edge kNoRow: not stored)
constexpr uint32_t kNoRow = 0xFFFFFFFFu;
struct RowId {
  __device__ __forceinline__ uint32_t operator()(int m) const { return (uint32_t)m; }
};
// BN-backward statistics in a dgrad epilogue (BS::MODE >= 0): the dgrad output is the dout of the
// batch norm whose output was this conv's input, so the epilogue also sums, per column, d and
// d * xhat with d = the STORED bf16 gradient through that BN's relu mask and xhat = (y - mean) *
// invstd -- exactly what bn_partial_kernel<1, MODE> reads back from memory, without the second pass
// over dout and y. MODE 0: no relu; 2: mask recomputed from y with the forward's constants; 3: the
// forward's relu bits ([M][N/8] bytes). Partials go to part[blockIdx.y][2][N] (bn_final's layout).
struct NoBnB {
  static constexpr int MODE = -1;
};
template <int MK>
struct BnB {
  static constexpr int MODE = MK;
  const uint16_t* __restrict__ y;
  const float *mean, *invstd, *gamma, *beta;
  const uint8_t* __restrict__ bits;
};
template <int BM, int BN, int WM, int WN, bool ADD, bool STATS, class RM = RowId, class BS = NoBnB>
__device__ __forceinline__ void lds_epilogue(f32x4 (&acc)[BM / WM / 16][BN / WN / 16], char* smem, uint16_t* __restrict__ y,
                                             AddSrc add, int M, int N, int m0, int n0,
                                             BnPart part, RM rowmap = RM{}, uint32_t ybytes = 0,
                                             BS bs = BS{}) {
  using E = LdsEpi<BM, BN, WM, WN>;
  constexpr bool BSTAT = BS::MODE >= 0;
  static_assert(!(STATS && BSTAT), "one statistics kind per epilogue");
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int cc = tid % E::CPR, g0 = tid / E::CPR;  // this thread's chunk column and first row
  const int n = n0 + cc * 8;
  if (ybytes == 0) ybytes = (uint32_t)M * (uint32_t)N * 2u;
  uint4 q[E::CH];
  [[maybe_unused]] uint32_t qb[E::CH];
  uint32_t orow[E::CH];
#pragma unroll
  for (int c = 0; c < E::CH; ++c) orow[c] = rowmap(m0 + g0 + c * E::RG);
  if constexpr (ADD) {
#pragma unroll
    for (int c = 0; c < E::CH; ++c) {
      const int m = m0 + g0 + c * E::RG;
      const bool ok = m < M && n < N && orow[c] != kNoRow;
      bool aok = ok;
      const uint32_t ar = add_row(add, orow[c], aok);
      q[c] = buf_ld(add.x, add.abytes ? add.abytes : ybytes, ar * (uint32_t)N + (uint32_t)n, aok);
      if (add.bits) qb[c] = buf_ld_u8(add.bits, ybytes / 16u, orow[c] * (uint32_t)(N / 8) + (uint32_t)(n / 8), ok);
    }
  }
  float* cs = reinterpret_cast<float*>(smem);
  __syncthreads();  // (the mainloop's last barrier already retired the operand images; cheap insurance)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r0 = wm * WTM + 16 * i + 4 * (lane >> 4), col = wn * WTN + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[(r0 + r) * E::PITCH + col] = acc[i][j][r];
    }
  // BN-backward operands: y chunks (and relu bytes) issued once the accumulator is staged (its
  // registers are free), in flight across the barrier
  [[maybe_unused]] uint4 yq[E::CH];
  [[maybe_unused]] uint32_t mbits[E::CH];
  [[maybe_unused]] float bmu[8], bis[8], bsc[8], bsh[8];
  if constexpr (BSTAT) {
#pragma unroll
    for (int c = 0; c < E::CH; ++c) {
      const int m = m0 + g0 + c * E::RG;
      const bool ok = m < M && n < N && orow[c] != kNoRow;
      yq[c] = buf_ld(bs.y, ybytes, orow[c] * (uint32_t)N + (uint32_t)n, ok);
      if constexpr (BS::MODE == 3) mbits[c] = buf_ld_u8(bs.bits, ybytes / 16u, orow[c] * (uint32_t)(N / 8) + (uint32_t)(n / 8), ok);
    }
    const int nc = n < N ? n : 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bmu[k] = bs.mean[nc + k];
      bis[k] = bs.invstd[nc + k];
      if constexpr (BS::MODE == 2) {
        bn_affine(bmu[k], bis[k], bs.gamma[nc + k], bs.beta[nc + k], bsc[k], bsh[k]);
      }
    }
  }
  __syncthreads();
  float s[8], sq[8];
  if constexpr (STATS || BSTAT) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { s[k] = 0.f; sq[k] = 0.f; }
  }
#pragma unroll
  for (int c = 0; c < E::CH; ++c) {
    const int row = g0 + c * E::RG, m = m0 + row;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(cs + row * E::PITCH + cc * 8);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(cs + row * E::PITCH + cc * 8 + 4);
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if constexpr (ADD) {
      if (add.bits) q[c] = add_masked(q[c], qb[c]);
      const uint32_t w[4] = {q[c].x, q[c].y, q[c].z, q[c].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] += __uint_as_float(w[k] << 16);
        v[2 * k + 1] += __uint_as_float(w[k] & 0xFFFF0000u);
      }
    }
    const uint4 o = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
    if (m < M && n < N && orow[c] != kNoRow) {
      *reinterpret_cast<uint4*>(y + (size_t)orow[c] * N + n) = o;
      if constexpr (STATS) {
        const uint32_t w[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float f0 = __uint_as_float(w[k] << 16), f1 = __uint_as_float(w[k] & 0xFFFF0000u);
          s[2 * k] += f0;
          sq[2 * k] = fmaf(f0, f0, sq[2 * k]);
          s[2 * k + 1] += f1;
          sq[2 * k + 1] = fmaf(f1, f1, sq[2 * k + 1]);
        }
      }
      if constexpr (BSTAT) {  // bn_partial_kernel<1, MODE>'s per-element math, same operands
        const uint32_t w[4] = {o.x, o.y, o.z, o.w};
        const uint32_t yw[4] = {yq[c].x, yq[c].y, yq[c].z, yq[c].w};
        float d[8], yv[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[2 * k] = __uint_as_float(w[k] << 16);
          d[2 * k + 1] = __uint_as_float(w[k] & 0xFFFF0000u);
          yv[2 * k] = __uint_as_float(yw[k] << 16);
          yv[2 * k + 1] = __uint_as_float(yw[k] & 0xFFFF0000u);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if constexpr (BS::MODE == 2) d[k] = fmaf(yv[k], bsc[k], bsh[k]) > 0.f ? d[k] : 0.f;
          if constexpr (BS::MODE == 3) d[k] = (mbits[c] >> k) & 1u ? d[k] : 0.f;
          s[k] += d[k];
          sq[k] = fmaf(d[k], (yv[k] - bmu[k]) * bis[k], sq[k]);
        }
      }
    }
  }
  if constexpr (STATS || BSTAT) {
    static_assert(2 * E::RG * BN * 4 <= E::BYTES, "stats reduction fits in the staged tile");
    __syncthreads();  // every thread has read its chunks: reuse the tile for [2][RG][BN]
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      cs[g0 * BN + cc * 8 + k] = s[k];
      cs[(E::RG + g0) * BN + cc * 8 + k] = sq[k];
    }
    __syncthreads();
    for (int col = tid; col < BN; col += E::NT) {
      const int nn = n0 + col;
      if (nn >= N) continue;
      float a = 0.f, b = 0.f;
#pragma unroll 8
      for (int g = 0; g < E::RG; ++g) { a += cs[g * BN + col]; b += cs[(E::RG + g) * BN + col]; }
      put_bn_part(part, blockIdx.y, N, nn, a, b);
    }
  }
}

#include "../conv_halo.h"

template <int BM, int BN>
struct Tile {
  static constexpr int WM = 2, WN = 2, BK = 64;
};

// One register stage (global-load prefetch depth) and a 64-deep K-tile for every conv GEMM tile: two
// stages doubled the 128x128 tile's accumulators to 368 VGPR+AGPR (one wave per SIMD, ResNet-50
// 18.9 -> 21.6 ms), BK = 32 halved the LDS but doubled the barriers (20.8 ms) -- docs/DESIGN.md §5,
// profiles/resnet_small_tile_rs_ab_r2.log.
template <int BM, int BN>
constexpr int conv_rs() { return 1; }
constexpr int CBK = 64;
// XR: renumber the blocks so that each XCD runs a run of consecutive (n, m, split) tiles -- dispatch
// deals block ids round-robin over the 8 XCDs, which puts the n-tiles sharing one A chunk (and the
// m-tiles sharing one B chunk) on different XCDs, each L2 fetching the chunk from the fabric.
template <int BM, int BN, class LA, class LB, class EPI, bool XR = false>
__global__ __launch_bounds__(256) void gemm_kernel(LA la, LB lb, EPI epi, int kchunk, int KD) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if constexpr (XR) {
    const int nx = gridDim.x, ny = gridDim.y, total = nx * ny * gridDim.z;
    if ((total & 7) == 0) {
      const int id = bx + nx * (by + ny * bz), l = (id & 7) * (total >> 3) + (id >> 3);
      bx = l % nx;
      by = (l / nx) % ny;
      bz = l / (nx * ny);
    }
  }
  const int kb = bz * kchunk, ke = min(KD, kb + kchunk);
  gemm_block<BM, BN, CBK, 2, 2, LA, LB, EPI, conv_rs<BM, BN>()>(la, lb, epi, by * BM, bx * BN, kb, ke, (bf16*)smem_raw);
}


// bf16-output GEMM with the LDS-staged epilogue: Y = A B (+ add), no split-K.
template <int BM, int BN, class LA, class LB, bool ADD>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(LA la, LB lb, uint16_t* y, AddSrc add,
                                                                      int M, int N, int KD) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  f32x4 acc[BM / 32][BN / 32];
  gemm_mainloop<BM, BN, CBK, 2, 2, LA, LB, conv_rs<BM, BN>()>(la, lb, blockIdx.y * BM, blockIdx.x * BN, 0, KD,
                                                       (bf16*)smem_raw, acc);
  lds_epilogue<BM, BN, 2, 2, ADD, false>(acc, smem_raw, y, add, M, N, blockIdx.y * BM, blockIdx.x * BN, BnPart{});
}

// dgrad (+ add) whose epilogue also emits the BN-backward partials of its output (BnB above)
template <int BM, int BN, class LA, class LB, bool ADD, class BS>
__global__ __launch_bounds__(256) void gemm_bf16_bnb_kernel(LA la, LB lb, uint16_t* y, AddSrc add,
                                                                          int M, int N, int KD, BnPart part, BS bs) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  f32x4 acc[BM / 32][BN / 32];
  gemm_mainloop<BM, BN, CBK, 2, 2, LA, LB, conv_rs<BM, BN>()>(la, lb, blockIdx.y * BM, blockIdx.x * BN, 0, KD,
                                                       (bf16*)smem_raw, acc);
  lds_epilogue<BM, BN, 2, 2, ADD, false, RowId, BS>(acc, smem_raw, y, add, M, N, blockIdx.y * BM, blockIdx.x * BN, part,
                                                    RowId{}, 0u, bs);
}

// Forward conv + BN statistics: the block's column partials (sum, sum of squares over its BM rows)
// go to part[blockIdx.y][2][N] -- the [nblk][2][C] layout bn_final_kernel reduces -- so the
// forward BN needs no separate pass over the conv output. Fixed reduction order (deterministic).
template <int BM, int BN, class LA, class LB>
__global__ __launch_bounds__(256) void gemm_stats_kernel(LA la, LB lb, uint16_t* y, int M, int N, int KD,
                                                         BnPart part) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  constexpr int WM = 2, WN = 2;
  f32x4 acc[BM / 32][BN / 32];
  gemm_mainloop<BM, BN, CBK, WM, WN, LA, LB, conv_rs<BM, BN>()>(la, lb, blockIdx.y * BM, blockIdx.x * BN, 0, KD,
                                                         (bf16*)smem_raw, acc);
  lds_epilogue<BM, BN, WM, WN, false, true>(acc, smem_raw, y, nullptr, M, N, blockIdx.y * BM, blockIdx.x * BN, part);
}

// one phase of a strided dgrad: Y rows scattered to the phase's pixels (+ add)
// BS (BnB<MODE>): the phase's rows of the BN-backward partials go to part[blockIdx.y] (part is
// offset per phase by the caller, so the phases' row blocks stack)
template <int BM, int BN, bool ADD, class BS = NoBnB>
__global__ __launch_bounds__(256) void dgrad_phase_kernel(DgradPhaseA la, DgradPhaseB lb, uint16_t* dx,
                                                                        AddSrc add, BnPart part = BnPart{},
                                                                        BS bs = BS{}) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  f32x4 acc[BM / 32][BN / 32];
  gemm_mainloop<BM, BN, CBK, 2, 2, DgradPhaseA, DgradPhaseB, conv_rs<BM, BN>()>(la, lb, blockIdx.y * BM, blockIdx.x * BN, 0,
                                                                         la.g.KD, (bf16*)smem_raw, acc);
  const uint32_t xbytes = (uint32_t)la.g.N * la.g.H * la.g.W * la.g.C * 2u;
  lds_epilogue<BM, BN, 2, 2, ADD, false, PhaseRows, BS>(acc, smem_raw, dx, add, la.g.M, la.g.C, blockIdx.y * BM,
                                                       blockIdx.x * BN, part, PhaseRows{la.g}, xbytes, bs);
}

// pixels of tap-less phases (a 1x1 stride-2 conv leaves 3 of 4 input pixels without a tap):
// dX = add there, or 0. One thread per 8-channel chunk of a pixel of such a phase.
__global__ __launch_bounds__(256) void dgrad_empty_phase_kernel(uint16_t* __restrict__ dx, const uint16_t* __restrict__ add,
                                                                int N, int H, int W, int C, int st, int pad, int R,
                                                                int S) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, cpp = C / 8;
  if (i >= (int64_t)N * H * W * cpp) return;
  const int64_t pix = i / cpp;
  const int w = (int)(pix % W), h = (int)((pix / W) % H);
  const int r0 = (h % st + pad) % st, s0 = (w % st + pad) % st;
  if (r0 < R && s0 < S) return;  // a phase with taps: written by its GEMM
  reinterpret_cast<uint4*>(dx)[i] = add ? reinterpret_cast<const uint4*>(add)[i] : make_uint4(0u, 0u, 0u, 0u);
}

template <int BM, int BN, class LA, class LB>
constexpr int stats_smem() {
  constexpr int g = GemmSmem<BM, BN, CBK, LA, LB>::BYTES;
  return LdsEpi<BM, BN, 2, 2>::BYTES > g ? LdsEpi<BM, BN, 2, 2>::BYTES : g;
}

template <int BM, int BN, class LA, class LB, bool ADD>
void launch_gemm_bf16(const LA& la, const LB& lb, uint16_t* y, AddSrc add, int M, int N, int KD,
                      hipStream_t st) {
  constexpr int sm = stats_smem<BM, BN, LA, LB>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_bf16_kernel<BM, BN, LA, LB, ADD>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, sm);
    attr = true;
  }
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, 1);
  gemm_bf16_kernel<BM, BN, LA, LB, ADD><<<grid, 256, sm, st>>>(la, lb, y, add, M, N, KD);
}

template <int BM, int BN, class LA, class LB, bool ADD, class BS>
void launch_gemm_bf16_bnb(const LA& la, const LB& lb, uint16_t* y, AddSrc add, int M, int N, int KD, float* part,
                          const BS& bs, hipStream_t st) {
  constexpr int sm = stats_smem<BM, BN, LA, LB>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_bf16_bnb_kernel<BM, BN, LA, LB, ADD, BS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, sm);
    attr = true;
  }
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, 1);
  gemm_bf16_bnb_kernel<BM, BN, LA, LB, ADD, BS><<<grid, 256, sm, st>>>(la, lb, y, add, M, N, KD, BnPart{part, bn_slots()},
                                                                        bs);
}

template <int BM, int BN, class LA, class LB>
void launch_gemm_stats(const LA& la, const LB& lb, uint16_t* y, int M, int N, int KD, float* part, hipStream_t st) {
  constexpr int sm = stats_smem<BM, BN, LA, LB>();
  static_assert(sm >= 2 * 2 * BN * 4, "stats reduction fits in the GEMM's LDS");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_stats_kernel<BM, BN, LA, LB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, sm);
    attr = true;
  }
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, 1);
  gemm_stats_kernel<BM, BN, LA, LB><<<grid, 256, sm, st>>>(la, lb, y, M, N, KD, BnPart{part, bn_slots()});
}

// same tile choice as dispatch(): 128x128 when that fills the chip
bool use_big_tiles(int M, int N) { return (long)((M + 127) / 128) * ((N + 127) / 128) >= 256 && N >= 128; }

// bf16-output tile (fwd, fwd + stats, dgrad): 128x128 when that fills the chip; for a 64-column
// output (the C = 64 stage of a ResNet) 128x64 when that does, else 64x64 (the 128x64 arm:
// profiles/resnet_tall_tiles_ab_r2.log, resnet50_tall_tiles_ab_r4.log).
enum OutTile { OT64, OT128x64, OT128 };
OutTile out_tile(int M, int N) {
  if (use_big_tiles(M, N)) return OT128;
  if (N == 64 && (long)((M + 127) / 128) >= 256) return OT128x64;
  return OT64;
}
int out_tile_rows(int M, int N) { return out_tile(M, N) == OT64 ? (M + 63) / 64 : (M + 127) / 128; }

template <int BM, int BN, bool XR = false, class LA, class LB, class EPI>
void launch_gemm(const LA& la, const LB& lb, const EPI& epi, int M, int N, int KD, int splits, hipStream_t st) {
  constexpr int sm = GemmSmem<BM, BN, CBK, LA, LB>::BYTES;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<BM, BN, LA, LB, EPI, XR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, sm);
    attr = true;
  }
  if (splits < 1) splits = 1;
  int kchunk = ((KD + splits - 1) / splits + CBK - 1) / CBK * CBK;
  splits = (KD + kchunk - 1) / kchunk;
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, splits);
  gemm_kernel<BM, BN, LA, LB, EPI, XR><<<grid, 256, sm, st>>>(la, lb, epi, kchunk, KD);
}

// pick 128x128 tiles when the problem has enough of them to fill the chip, else 64x64
template <class LA, class LB, class EPI>
void dispatch(const LA& la, const LB& lb, const EPI& epi, int M, int N, int KD, int splits, hipStream_t st) {
  const long big = (long)((M + 127) / 128) * ((N + 127) / 128) * splits;
  if (big >= 256 && N >= 128) launch_gemm<128, 128>(la, lb, epi, M, N, KD, splits, st);
  else launch_gemm<64, 64>(la, lb, epi, M, N, KD, splits, st);
}

// bf16-output GEMM (optionally + add), same tile choice as dispatch()
template <class LA, class LB>
void dispatch_bf16(const LA& la, const LB& lb, uint16_t* y, AddSrc add, int M, int N, int KD, hipStream_t st) {
  const OutTile t = out_tile(M, N);
  if (add.x) {
    if (t == OT128) launch_gemm_bf16<128, 128, LA, LB, true>(la, lb, y, add, M, N, KD, st);
    else if (t == OT128x64) launch_gemm_bf16<128, 64, LA, LB, true>(la, lb, y, add, M, N, KD, st);
    else launch_gemm_bf16<64, 64, LA, LB, true>(la, lb, y, add, M, N, KD, st);
  } else {
    if (t == OT128) launch_gemm_bf16<128, 128, LA, LB, false>(la, lb, y, add, M, N, KD, st);
    else if (t == OT128x64) launch_gemm_bf16<128, 64, LA, LB, false>(la, lb, y, add, M, N, KD, st);
    else launch_gemm_bf16<64, 64, LA, LB, false>(la, lb, y, add, M, N, KD, st);
  }
}

template <class LA, class LB, class BS>
void dispatch_bf16_bnb(const LA& la, const LB& lb, uint16_t* y, AddSrc add, int M, int N, int KD, float* part,
                       const BS& bs, hipStream_t st) {
  const OutTile t = out_tile(M, N);
  if (add.x) {
    if (t == OT128) launch_gemm_bf16_bnb<128, 128, LA, LB, true>(la, lb, y, add, M, N, KD, part, bs, st);
    else if (t == OT128x64) launch_gemm_bf16_bnb<128, 64, LA, LB, true>(la, lb, y, add, M, N, KD, part, bs, st);
    else launch_gemm_bf16_bnb<64, 64, LA, LB, true>(la, lb, y, add, M, N, KD, part, bs, st);
  } else {
    if (t == OT128) launch_gemm_bf16_bnb<128, 128, LA, LB, false>(la, lb, y, add, M, N, KD, part, bs, st);
    else if (t == OT128x64) launch_gemm_bf16_bnb<128, 64, LA, LB, false>(la, lb, y, add, M, N, KD, part, bs, st);
    else launch_gemm_bf16_bnb<64, 64, LA, LB, false>(la, lb, y, add, M, N, KD, part, bs, st);
  }
}

Geo make_geo(const ConvShape& c, int M, int KD) {
  Geo g;
  g.N = c.N; g.H = c.H; g.W = c.W; g.C = c.C; g.K = c.K; g.R = c.R; g.S = c.S; g.st = c.stride; g.pad = c.pad;
  g.stw = c.sw(); g.padw = c.pw();
  g.Ho = c.Ho(); g.Wo = c.Wo();
  g.M = M; g.KD = KD;
  g.howo = FastDiv(g.Ho * g.Wo); g.wo = FastDiv(g.Wo); g.c = FastDiv(g.C); g.k = FastDiv(g.K); g.s = FastDiv(g.S);
  g.hw = FastDiv(g.H * g.W); g.w = FastDiv(g.W);
  g.xbytes = (uint32_t)((int64_t)c.N * c.H * c.W * c.C * 2);
  g.ybytes = (uint32_t)((int64_t)c.N * g.Ho * g.Wo * c.K * 2);
  g.wbytes = (uint32_t)((int64_t)c.R * c.S * c.C * c.K * 2);
  return g;
}

bool is_pointwise(const ConvShape& c) { return c.R == 1 && c.S == 1 && c.stride == 1 && c.pad == 0 && !c.w_override(); }

// ---------------- the conv GEMMs on the 256-row core (csrc/gemm256.h) ----------------
// Block tile 256 x BN (BN = 256 / 128 / 64 by the output width), 8 waves, 32x32x16 MFMA, operands
// DMA'd into LDS through the same loaders (their off() / rsrc()). Forward: A = im2col(X) (KC), B = the
// HWIO weight (MNC, transposed fragment reads); dgrad: A = dY gather, B = W as [C][(r,s,k)] (both KC);
// weight gradient: A = im2col(X)^T, B = dY (both MNC). The core choice (conv_gemm_core(), the op
// tfd::conv_gemm_core that the per-layer probe tools/debug/gemm_probe.py and the numerics tests
// switch): 0 = the 128-row core everywhere, 1 (default) = this core where its tiles fill the chip with
// >= 1024-channel bf16 outputs, 2 = wherever it applies (profiles/resnet50_core_ab_r4.log).
int g256_mode_v = 1;  // conv_gemm_core(): 0 / 1 (default) / 2, see above
int g256_mode() { return g256_mode_v; }
int g256_bn(int N) { return N >= 256 ? 256 : (N >= 128 ? 128 : 64); }
long g256_tiles(int M, int N) { return (long)((M + 255) / 256) * ((N + g256_bn(N) - 1) / g256_bn(N)); }
// Mode 1 takes the 256-row core only where the per-layer A/B measured it faster
// (profiles/gemm256_conv_layers_r4.txt): bf16-output GEMMs (forward, dgrad) with >= 1024 output
// channels -- e.g. ResNet-50 l3 1x1 256->1024 forward 30.8 vs 33.8 us, l4 1x1 2048->512 dgrad 22.7 vs
// 26.9. Narrower outputs (fewer, 256-row tiles for the chip; one 8-wave block per CU instead of 3-4
// 4-wave blocks hiding each other's latency on these short-K, often memory-bound layers) and every
// weight gradient measured slower there; ResNet-50 b128 13.65 ms/step with the 128-row core
// everywhere, 14.37 with the 256-row core wherever it had >= 256 tiles, 19.6 with it everywhere.
bool use_g256(int M, int N) {
  const int mode = g256_mode();
  if (mode == 0 || N % 8) return false;
  return mode == 2 || (N >= 1024 && g256_tiles(M, N) >= 32);
}

// ---- 3x3 stride-1 convs on LDS halo tiles (csrc/conv_halo.h) ----
// conv_halo_mode(): 0 = off (the im2col gather everywhere), 1 (default) = forward and stride-1 dgrad of
// the 3x3 stride-1 pad-1 convs where the per-layer probe measured the halo tiles faster -- maps at least
// 32 pixels wide (ResNet-50 stage 1, 56 x 56 x 64: fwd 74.2 -> 64.5 us, dgrad 76.8 -> 62.8 us); on the
// 28- and 14-wide maps an 8 x 16 tile leaves 23 % of its rows past the image edge and the gather wins
// (profiles/halo_probe_r5.log) -- 2 = every eligible shape (tests, probes).
int g_halo_mode = 1;
bool use_halo(const ConvShape& c, int cin, int cout) {
  if (g_halo_mode == 0 || c.R != 3 || c.S != 3 || c.stride != 1 || c.pad != 1 || c.w_override()) return false;
  if (cin % HL_CK || cout % 64) return false;
  return g_halo_mode == 2 || c.W >= 32;
}
HaloGeo halo_geo(const ConvShape& c, bool dgrad) {
  HaloGeo g;
  g.N = c.N; g.H = c.H; g.W = c.W;
  g.Cin = dgrad ? c.K : c.C;
  g.Cout = dgrad ? c.C : c.K;
  g.tx = (c.W + HL_TW - 1) / HL_TW;
  g.ty = (c.H + HL_TH - 1) / HL_TH;
  g.mtiles = c.N * g.tx * g.ty;
  const uint32_t px = (uint32_t)c.N * (uint32_t)c.H * (uint32_t)c.W;
  g.xbytes = px * (uint32_t)g.Cin * 2u;
  g.ybytes = px * (uint32_t)g.Cout * 2u;
  g.wbytes = 9u * (uint32_t)c.C * (uint32_t)c.K * 2u;
  return g;
}
template <int BN, bool DG, bool ADD, bool STATS, class BS>
void halo_launch_bn(const uint16_t* x, const uint16_t* w, uint16_t* y, const HaloGeo& g, const AddSrc& add, float* part,
                    const BS& bs, hipStream_t st) {
  constexpr int sm = HaloSmem<BN>::BYTES;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_halo_kernel<BN, DG, ADD, STATS, BS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, sm);
    attr = true;
  }
  conv3x3_halo_kernel<BN, DG, ADD, STATS, BS><<<dim3(g.Cout / BN, g.mtiles), 256, sm, st>>>(
      x, w, y, g, add, BnPart{part, bn_slots()}, bs);
}
template <bool DG, bool ADD, bool STATS, class BS = NoBnB>
void halo_launch(const uint16_t* x, const uint16_t* w, uint16_t* y, const HaloGeo& g, const AddSrc& add, float* part,
                 hipStream_t st, const BS& bs = BS{}) {
  if (g.Cout % 128 == 0) halo_launch_bn<128, DG, ADD, STATS, BS>(x, w, y, g, add, part, bs, st);
  else halo_launch_bn<64, DG, ADD, STATS, BS>(x, w, y, g, add, part, bs, st);
}

template <int BN> struct G256WM { static constexpr int v = BN == 256 ? 2 : 4; };

// bf16 epilogue of a 256 x BN tile, in two 128-row halves through an fp32 LDS image (pitch BN + 8:
// the two row groups of an accumulator register write land 32 banks apart): each thread then owns
// whole 8-column chunks -- residual chunks loaded as 16-B buffer loads before the half is staged, one
// 16-B store per output chunk, the sum v + add formed in fp32 and rounded once. STATS: per-column sums
// / sums of squares of the stored bf16 values; BnB (BS::MODE >= 0): the BN-backward sums of the stored
// gradient (see lds_epilogue). Both halves accumulate in registers; one partial row per tile at part.
template <int BN>
struct G256Epi {
  static constexpr int PITCH = BN + 8, CPR = BN / 8, RG = 512 / CPR, CH = 128 / RG;
  static constexpr int BYTES = 128 * PITCH * 4;
  static_assert(2 * RG * BN * 4 <= BYTES, "stats reduction fits");
};
template <class C, bool ADD, bool STATS, class RM, class BS>
__device__ __forceinline__ void g256_epilogue(f32x16 (&acc)[C::TM][C::TN], char* smem, uint16_t* __restrict__ y,
                                              AddSrc add, int M, int N, int m0, int n0,
                                              BnPart part, RM rowmap, uint32_t ybytes, BS bs) {
  using E = G256Epi<C::BN>;
  constexpr bool BSTAT = BS::MODE >= 0;
  static_assert(!(STATS && BSTAT), "one statistics kind per epilogue");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w / C::WN, wn = w % C::WN;
  const int cc = tid % E::CPR, g0 = tid / E::CPR, n = n0 + cc * 8;
  const int my_half = (wm * C::WTM) >> 7;
  if (ybytes == 0) ybytes = (uint32_t)M * (uint32_t)N * 2u;
  float s[8], sq[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[k] = 0.f; sq[k] = 0.f; }
  [[maybe_unused]] float bmu[8], bis[8], bsc[8], bsh[8];
  if constexpr (BSTAT) {
    const int nc = n < N ? n : 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bmu[k] = bs.mean[nc + k];
      bis[k] = bs.invstd[nc + k];
      if constexpr (BS::MODE == 2) {
        bn_affine(bmu[k], bis[k], bs.gamma[nc + k], bs.beta[nc + k], bsc[k], bsh[k]);
      }
    }
  }
  float* cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int mb = m0 + 128 * h;
    uint32_t orow[E::CH];
    [[maybe_unused]] uint4 q[E::CH], yq[E::CH];
    [[maybe_unused]] uint32_t mbits[E::CH], qb[E::CH];
#pragma unroll
    for (int c = 0; c < E::CH; ++c) {
      const int m = mb + g0 + c * E::RG;
      orow[c] = rowmap(m);
      const bool ok = m < M && n < N;
      if constexpr (ADD) {
        bool aok = ok;
        const uint32_t ar = add_row(add, orow[c], aok);
        q[c] = buf_ld(add.x, add.abytes ? add.abytes : ybytes, ar * (uint32_t)N + (uint32_t)n, aok);
        if (add.bits) qb[c] = buf_ld_u8(add.bits, ybytes / 16u, orow[c] * (uint32_t)(N / 8) + (uint32_t)(n / 8), ok);
      }
      if constexpr (BSTAT) {
        yq[c] = buf_ld(bs.y, ybytes, orow[c] * (uint32_t)N + (uint32_t)n, ok);
        if constexpr (BS::MODE == 3) mbits[c] = buf_ld_u8(bs.bits, ybytes / 16u, orow[c] * (uint32_t)(N / 8) + (uint32_t)(n / 8), ok);
      }
    }
    __syncthreads();  // the previous half's chunks (or the mainloop's operands) are consumed
    if (my_half == h) {
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            cs[(g256_row<C>(wm, i, r, lane) - 128 * h) * E::PITCH + g256_col<C>(wn, j, lane)] = acc[i][j][r];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < E::CH; ++c) {
      const int row = g0 + c * E::RG, m = mb + row;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(cs + row * E::PITCH + cc * 8);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(cs + row * E::PITCH + cc * 8 + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if constexpr (ADD) {
        if (add.bits) q[c] = add_masked(q[c], qb[c]);
        const uint32_t wq[4] = {q[c].x, q[c].y, q[c].z, q[c].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] += __uint_as_float(wq[k] << 16);
          v[2 * k + 1] += __uint_as_float(wq[k] & 0xFFFF0000u);
        }
      }
      const uint4 o = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
      if (m < M && n < N) {
        *reinterpret_cast<uint4*>(y + (size_t)orow[c] * N + n) = o;
        const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
        float d[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[2 * k] = __uint_as_float(ow[k] << 16);
          d[2 * k + 1] = __uint_as_float(ow[k] & 0xFFFF0000u);
        }
        if constexpr (STATS) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            s[k] += d[k];
            sq[k] = fmaf(d[k], d[k], sq[k]);
          }
        }
        if constexpr (BSTAT) {
          const uint32_t yw[4] = {yq[c].x, yq[c].y, yq[c].z, yq[c].w};
          float yv[8];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            yv[2 * k] = __uint_as_float(yw[k] << 16);
            yv[2 * k + 1] = __uint_as_float(yw[k] & 0xFFFF0000u);
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if constexpr (BS::MODE == 2) d[k] = fmaf(yv[k], bsc[k], bsh[k]) > 0.f ? d[k] : 0.f;
            if constexpr (BS::MODE == 3) d[k] = (mbits[c] >> k) & 1u ? d[k] : 0.f;
            s[k] += d[k];
            sq[k] = fmaf(d[k], (yv[k] - bmu[k]) * bis[k], sq[k]);
          }
        }
      }
    }
  }
  if constexpr (STATS || BSTAT) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      cs[g0 * C::BN + cc * 8 + k] = s[k];
      cs[(E::RG + g0) * C::BN + cc * 8 + k] = sq[k];
    }
    __syncthreads();
    for (int col = tid; col < C::BN; col += 512) {
      const int nn = n0 + col;
      if (nn >= N) continue;
      float a = 0.f, b = 0.f;
#pragma unroll 8
      for (int g = 0; g < E::RG; ++g) { a += cs[g * C::BN + col]; b += cs[(E::RG + g) * C::BN + col]; }
      put_bn_part(part, 0, N, nn, a, b);  // part: already the tile's row (or slot), see g256_conv_kernel
    }
  }
}

template <int BN>
constexpr int g256_smem() {
  using C = G256<BN, G256WM<BN>::v>;
  return C::SMEM > G256Epi<BN>::BYTES ? C::SMEM : G256Epi<BN>::BYTES;
}

// bf16-output conv GEMM: part (STATS / BnB) gets one row per 256-row tile at part + tile_m * 2N (slot
// mode: added into slot tile_m % part.slots)
template <int BN, bool AKC, bool BKC, class SA, class SB, bool ADD, bool STATS, class RM, class BS>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void g256_conv_kernel(
    SA sa, SB sb, uint16_t* y, AddSrc add, int M, int N, int KD, BnPart part, RM rm, uint32_t ybytes, BS bs,
    int tiles_m, int tiles_n) {
  using C = G256<BN, G256WM<BN>::v, AKC, BKC>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  int tm, tn;
  g256_tile(blockIdx.x, gridDim.x, tiles_m, tiles_n, tm, tn);
  f32x16 acc[C::TM][C::TN];
  g256_mainloop<C>(sa, sb, tm * 256, tn * BN, 0, KD, smem_raw, acc);
  g256_epilogue<C, ADD, STATS, RM, BS>(acc, smem_raw, y, add, M, N, tm * 256, tn * BN,
                                       BnPart{part.p ? part.p + (size_t)bn_part_row(part, tm) * 2 * N : nullptr,
                                              part.slots}, rm, ybytes, bs);
}

// (plain template launchers, no generic lambdas: instantiating the kernel template from a host
// lambda made hipcc's host pass reject the device-only DMA builtin inside it)
template <int BN, bool AKC, bool BKC, bool ADD, bool STATS, class SA, class SB, class RM, class BS>
void g256_launch_bf16_bn(const SA& sa, const SB& sb, uint16_t* y, AddSrc add, int M, int N, int KD, float* part,
                         hipStream_t st, RM rm, uint32_t ybytes, BS bs) {
  auto* k = &g256_conv_kernel<BN, AKC, BKC, SA, SB, ADD, STATS, RM, BS>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                              g256_smem<BN>());
    attr = true;
  }
  const int tm = (M + 255) / 256, tn = (N + BN - 1) / BN;
  k<<<tm * tn, 512, g256_smem<BN>(), st>>>(sa, sb, y, add, M, N, KD, BnPart{part, bn_slots()}, rm, ybytes, bs, tm, tn);
}
template <bool AKC, bool BKC, bool ADD, bool STATS, class SA, class SB, class RM = RowId, class BS = NoBnB>
void g256_launch_bf16(const SA& sa, const SB& sb, uint16_t* y, AddSrc add, int M, int N, int KD, float* part,
                      hipStream_t st, RM rm = RM{}, uint32_t ybytes = 0, BS bs = BS{}) {
  const int bn = g256_bn(N);
  if (bn == 256) g256_launch_bf16_bn<256, AKC, BKC, ADD, STATS>(sa, sb, y, add, M, N, KD, part, st, rm, ybytes, bs);
  else if (bn == 128) g256_launch_bf16_bn<128, AKC, BKC, ADD, STATS>(sa, sb, y, add, M, N, KD, part, st, rm, ybytes, bs);
  else g256_launch_bf16_bn<64, AKC, BKC, ADD, STATS>(sa, sb, y, add, M, N, KD, part, st, rm, ybytes, bs);
}

// weight gradient: dW [M = R*S*C][N = K] fp32, split-K over pixels (KD); the accumulator registers go
// straight out (a 32 x 32 register holds two 128-B row segments: full-rate stores and atomics)
template <int BN, class SA, class SB>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void g256_wgrad_kernel(
    SA sa, SB sb, float* dw, int M, int N, int KD, int kchunk, int tiles_m, int tiles_n, int atomic) {
  using C = G256<BN, G256WM<BN>::v, false, false>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tiles = tiles_m * tiles_n, split = blockIdx.x / tiles;
  int tm, tn;
  g256_tile(blockIdx.x - split * tiles, tiles, tiles_m, tiles_n, tm, tn);
  const int kb = split * kchunk, ke = min(KD, kb + kchunk);
  f32x16 acc[C::TM][C::TN];
  g256_mainloop<C>(sa, sb, tm * 256, tn * BN, kb, ke, smem_raw, acc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w / C::WN, wn = w % C::WN;
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int col = tn * BN + g256_col<C>(wn, j, lane);
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tm * 256 + g256_row<C>(wm, i, r, lane);
        if (row >= M) continue;
        float* p = dw + (size_t)row * N + col;
        if (atomic) atomicAdd(p, acc[i][j][r]);
        else *p = acc[i][j][r];
      }
    }
}

template <int BN, class SA>
void g256_launch_wgrad_bn(const SA& sa, const DenseX<false>& sb, float* dw, int M, int N, int KD, int splits,
                          hipStream_t st) {
  using C = G256<BN, G256WM<BN>::v, false, false>;
  auto* k = &g256_wgrad_kernel<BN, SA, DenseX<false>>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, C::SMEM);
    attr = true;
  }
  const int tm = (M + 255) / 256, tn = (N + BN - 1) / BN;
  const int kchunk = ((KD + splits - 1) / splits + 63) / 64 * 64;
  const int sp = (KD + kchunk - 1) / kchunk;
  k<<<tm * tn * sp, 512, C::SMEM, st>>>(sa, sb, dw, M, N, KD, kchunk, tm, tn, sp > 1 ? 1 : 0);
}
template <class SA>
void g256_launch_wgrad(const SA& sa, const DenseX<false>& sb, float* dw, int M, int N, int KD, int splits, hipStream_t st) {
  const int bn = g256_bn(N);
  if (bn == 256) g256_launch_wgrad_bn<256>(sa, sb, dw, M, N, KD, splits, st);
  else if (bn == 128) g256_launch_wgrad_bn<128>(sa, sb, dw, M, N, KD, splits, st);
  else g256_launch_wgrad_bn<64>(sa, sb, dw, M, N, KD, splits, st);
}

}  // namespace

static BnReluArgs bn_relu_args(const ConvShape& c, const BnReluIn* act) {
  if (c.C > kBnReluMaxC) throw std::runtime_error("conv: folded BN input with C > kBnReluMaxC");
  return BnReluArgs{act->mean, act->invstd, act->gamma, act->beta, c.C};
}

void conv_fwd(const ConvShape& c, const uint16_t* x, const uint16_t* w, uint16_t* y, hipStream_t st,
              const BnReluIn* act) {
  const int M = c.N * c.Ho() * c.Wo(), KD = c.R * c.S * c.C;
  DenseX<false> lb{w, c.K, c.K, KD};
  if (act) {  // the 128-row core: its loaders stage through registers, where the transform happens
    const BnReluArgs a = bn_relu_args(c, act);
    if (is_pointwise(c)) dispatch_bf16(BnRelu<DenseX<true>>{{x, c.C, M, c.C}, a}, lb, y, nullptr, M, c.K, KD, st);
    else dispatch_bf16(BnRelu<FwdA>{{x, make_geo(c, M, KD)}, a}, lb, y, nullptr, M, c.K, KD, st);
    return;
  }
  if (use_halo(c, c.C, c.K)) {
    halo_launch<false, false, false>(x, w, y, halo_geo(c, false), AddSrc{}, nullptr, st);
    return;
  }
  if (use_g256(M, c.K)) {  // A = im2col(X) (KC), B = HWIO weight (MNC)
    if (is_pointwise(c)) g256_launch_bf16<true, false, false, false>(DenseX<true>{x, c.C, M, c.C}, lb, y, nullptr, M, c.K, KD, nullptr, st);
    else g256_launch_bf16<true, false, false, false>(FwdA{x, make_geo(c, M, KD)}, lb, y, nullptr, M, c.K, KD, nullptr, st);
    return;
  }
  if (is_pointwise(c)) dispatch_bf16(DenseX<true>{x, c.C, M, c.C}, lb, y, nullptr, M, c.K, KD, st);
  else dispatch_bf16(FwdA{x, make_geo(c, M, KD)}, lb, y, nullptr, M, c.K, KD, st);
}


int conv_fwd_stats_rows(const ConvShape& c, bool folded) {  // row blocks of the partials
  if (bn_slots() > 0) return bn_slots();
  const int M = c.N * c.Ho() * c.Wo();
  if (!folded && use_halo(c, c.C, c.K)) return halo_geo(c, false).mtiles;
  if (!folded && use_g256(M, c.K)) return (M + 255) / 256;
  return out_tile_rows(M, c.K);
}

void conv_fwd_stats(const ConvShape& c, const uint16_t* x, const uint16_t* w, uint16_t* y, float* part,
                    hipStream_t st, const BnReluIn* act) {
  const int M = c.N * c.Ho() * c.Wo(), KD = c.R * c.S * c.C;
  DenseX<false> lb{w, c.K, c.K, KD};
  if (!act && use_halo(c, c.C, c.K)) {
    halo_launch<false, false, true>(x, w, y, halo_geo(c, false), AddSrc{}, part, st);
    return;
  }
  if (!act && use_g256(M, c.K)) {
    if (is_pointwise(c)) g256_launch_bf16<true, false, false, true>(DenseX<true>{x, c.C, M, c.C}, lb, y, nullptr, M, c.K, KD, part, st);
    else g256_launch_bf16<true, false, false, true>(FwdA{x, make_geo(c, M, KD)}, lb, y, nullptr, M, c.K, KD, part, st);
    return;
  }
  const OutTile t = out_tile(M, c.K);
  auto go = [&](const auto& la) {
    using LA = std::decay_t<decltype(la)>;
    if (t == OT128) launch_gemm_stats<128, 128, LA, DenseX<false>>(la, lb, y, M, c.K, KD, part, st);
    else if (t == OT128x64) launch_gemm_stats<128, 64, LA, DenseX<false>>(la, lb, y, M, c.K, KD, part, st);
    else launch_gemm_stats<64, 64, LA, DenseX<false>>(la, lb, y, M, c.K, KD, part, st);
  };
  if (act) {
    const BnReluArgs a = bn_relu_args(c, act);
    if (is_pointwise(c)) go(BnRelu<DenseX<true>>{{x, c.C, M, c.C}, a});
    else go(BnRelu<FwdA>{{x, make_geo(c, M, KD)}, a});
  } else if (is_pointwise(c)) {
    go(DenseX<true>{x, c.C, M, c.C});
  } else {
    go(FwdA{x, make_geo(c, M, KD)});
  }
}

template <class Epi>
static void conv_dgrad_impl(const ConvShape& c, const uint16_t* dy, const uint16_t* w, Epi epi, hipStream_t st) {
  const int M = c.N * c.H * c.W, KD = c.R * c.S * c.K;
  if (is_pointwise(c)) {  // dX = dY W^T: W [C][K] read k-contiguous
    DenseX<true> la{dy, c.K, M, c.K};
    DenseX<true> lb{w, c.K, c.C, c.K};
    dispatch(la, lb, epi, M, c.C, KD, 1, st);
  } else {
    Geo g = make_geo(c, M, KD);
    DgradA la{dy, g};
    DgradB lb{w, g};
    dispatch(la, lb, epi, M, c.C, KD, 1, st);
  }
}

template <int BM, int BN, bool ADD, class BS = NoBnB>
static void launch_phase(const DgradPhaseA& la, const DgradPhaseB& lb, uint16_t* dx, const AddSrc& add,
                         hipStream_t st, float* part = nullptr, const BS& bs = BS{}) {
  constexpr int sm = GemmSmem<BM, BN, CBK, DgradPhaseA, DgradPhaseB>::BYTES > LdsEpi<BM, BN, 2, 2>::BYTES
                         ? GemmSmem<BM, BN, CBK, DgradPhaseA, DgradPhaseB>::BYTES : LdsEpi<BM, BN, 2, 2>::BYTES;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dgrad_phase_kernel<BM, BN, ADD, BS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, sm);
    attr = true;
  }
  dim3 grid((la.g.C + BN - 1) / BN, (la.g.M + BM - 1) / BM, 1);
  dgrad_phase_kernel<BM, BN, ADD, BS><<<grid, 256, sm, st>>>(la, lb, dx, add, BnPart{part, bn_slots()}, bs);
}
// BS != NoBnB: every phase also emits its BN-backward partial rows at part + (rows so far) * 2 * C
// (callers ensure no phase is tap-less: those pixels would carry no partials). Returns the rows.
template <class BS = NoBnB>
static int dgrad_strided(const ConvShape& c, const uint16_t* dy, const uint16_t* w, uint16_t* dx, const AddSrc& add,
                         hipStream_t st, float* part = nullptr, const BS& bs = BS{}) {
  const int s = c.stride;
  bool empty = false;
  int rows = 0;
  for (int ph = 0; ph < s; ++ph)
    for (int pw = 0; pw < s; ++pw) {
      PhaseGeo g;
      g.N = c.N; g.H = c.H; g.W = c.W; g.C = c.C; g.K = c.K; g.st = s; g.ph = ph; g.pw = pw;
      g.Ho = c.Ho(); g.Wo = c.Wo();
      g.Hp = (c.H - ph + s - 1) / s; g.Wp = (c.W - pw + s - 1) / s;
      g.r0 = (ph + c.pad) % s; g.s0 = (pw + c.pad) % s;
      g.nr = g.r0 < c.R ? (c.R - g.r0 + s - 1) / s : 0;
      g.ns = g.s0 < c.S ? (c.S - g.s0 + s - 1) / s : 0;
      if (g.nr == 0 || g.ns == 0 || g.Hp <= 0 || g.Wp <= 0) { empty = empty || (g.Hp > 0 && g.Wp > 0); continue; }
      g.dh = (ph + c.pad - g.r0) / s; g.dw = (pw + c.pad - g.s0) / s;
      g.M = c.N * g.Hp * g.Wp; g.KD = g.nr * g.ns * c.K;
      g.ybytes = (uint32_t)((int64_t)c.N * g.Ho * g.Wo * c.K * 2);
      g.wbytes = (uint32_t)((int64_t)c.R * c.S * c.C * c.K * 2);
      g.hpwp = FastDiv(g.Hp * g.Wp); g.wp = FastDiv(g.Wp); g.k = FastDiv(c.K); g.nsd = FastDiv(g.ns);
      DgradPhaseA la{dy, g};
      DgradPhaseB lb{w, g, c.S};
      // slot mode: every phase adds into the same slots
      float* pp = part ? part + (bn_slots() > 0 ? (size_t)0 : (size_t)rows * 2 * c.C) : nullptr;
      if (use_g256(g.M, c.C)) {
        rows += (g.M + 255) / 256;
        const uint32_t xbytes = (uint32_t)((int64_t)c.N * c.H * c.W * c.C * 2);
        if (add.x) g256_launch_bf16<true, true, true, false>(la, lb, dx, add, g.M, c.C, g.KD, pp, st, PhaseRows{g}, xbytes, bs);
        else g256_launch_bf16<true, true, false, false>(la, lb, dx, add, g.M, c.C, g.KD, pp, st, PhaseRows{g}, xbytes, bs);
        continue;
      }
      const OutTile ot = out_tile(g.M, c.C);
      rows += ot == OT64 ? (g.M + 63) / 64 : (g.M + 127) / 128;
      if (add.x) {
        if (ot == OT128) launch_phase<128, 128, true>(la, lb, dx, add, st, pp, bs);
        else if (ot == OT128x64) launch_phase<128, 64, true>(la, lb, dx, add, st, pp, bs);
        else launch_phase<64, 64, true>(la, lb, dx, add, st, pp, bs);
      } else {
        if (ot == OT128) launch_phase<128, 128, false>(la, lb, dx, add, st, pp, bs);
        else if (ot == OT128x64) launch_phase<128, 64, false>(la, lb, dx, add, st, pp, bs);
        else launch_phase<64, 64, false>(la, lb, dx, add, st, pp, bs);
      }
    }
  if (empty) {
    const int64_t total = (int64_t)c.N * c.H * c.W * (c.C / 8);
    // tap-less phases: the add operand there, or zeros (a stride-2 operand must sit on tap phases)
    if (add.sub_w && (c.pad % s) != 0) throw std::runtime_error("dgrad: stride-2 add operand over a tap-less phase");
    dgrad_empty_phase_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>(dx, add.sub_w ? nullptr : add.x, c.N, c.H, c.W,
                                                                         c.C, s, c.pad, c.R, c.S);
  }
  return rows;
}

static AddSrc make_add(const ConvShape& c, const uint16_t* add, const uint8_t* add_bits, bool add_sub2) {
  AddSrc a{add, add_bits};
  if (add_sub2) {  // the operand is on the stride-2 grid of this dgrad's output (see AddSrc)
    a.sub_w = (uint32_t)c.W;
    a.sub_h = (uint32_t)c.H;
    a.sub_wo = (uint32_t)((c.W + 1) / 2);
    a.sub_ho = (uint32_t)((c.H + 1) / 2);
    a.abytes = (uint32_t)((int64_t)c.N * a.sub_ho * a.sub_wo * c.C * 2);
  }
  return a;
}

void conv_dgrad(const ConvShape& c, const uint16_t* dy, const uint16_t* w, uint16_t* dx, hipStream_t st,
                const uint16_t* add, const uint8_t* add_bits, bool add_sub2) {
  if (c.w_override()) throw std::runtime_error("conv dgrad: width overrides are forward / weight-gradient only");
  const int M = c.N * c.H * c.W;
  if (add_bits && (!add || c.stride != 1))
    throw std::runtime_error("conv_dgrad: a relu-masked add operand needs a stride-1 dgrad");
  if (add_sub2 && !add) throw std::runtime_error("conv_dgrad: stride-2 add operand without add");
  if (add_bits && add_sub2) throw std::runtime_error("conv_dgrad: one add-operand form at a time");
  const AddSrc aa = make_add(c, add, add_bits, add_sub2);
  if (c.stride > 1) {  // one dense GEMM per output phase (profiles/resnet50_dgrad_phases_ab_r2.log)
    dgrad_strided(c, dy, w, dx, aa, st);
    return;
  }
  if (use_halo(c, c.K, c.C)) {
    if (add) halo_launch<true, true, false>(dy, w, dx, halo_geo(c, true), aa, nullptr, st);
    else halo_launch<true, false, false>(dy, w, dx, halo_geo(c, true), aa, nullptr, st);
    return;
  }
  if (use_g256(M, c.C)) {  // A = dY gather, B = W as [C][(r,s,k)]: both KC
    const int KD = c.R * c.S * c.K;
    auto go = [&](const auto& la, const auto& lb) {
      if (add) g256_launch_bf16<true, true, true, false>(la, lb, dx, aa, M, c.C, KD, nullptr, st);
      else g256_launch_bf16<true, true, false, false>(la, lb, dx, aa, M, c.C, KD, nullptr, st);
    };
    if (is_pointwise(c)) {
      go(DenseX<true>{dy, c.K, M, c.K}, DenseX<true>{w, c.K, c.C, c.K});
    } else {
      Geo g = make_geo(c, M, KD);
      go(DgradA{dy, g}, DgradB{w, g});
    }
    return;
  }
  const int KD = c.R * c.S * c.K;
  if (is_pointwise(c)) {
    dispatch_bf16(DenseX<true>{dy, c.K, M, c.K}, DenseX<true>{w, c.K, c.C, c.K}, dx, aa, M, c.C, KD, st);
  } else {
    Geo g = make_geo(c, M, KD);
    dispatch_bf16(DgradA{dy, g}, DgradB{w, g}, dx, aa, M, c.C, KD, st);
  }
}

// stride 1, or a strided dgrad by output phases none of which is tap-less (every input pixel is in
// some phase GEMM, e.g. ResNet v1.5's 3x3 stride-2 convs)
bool conv_dgrad_bn_supported(const ConvShape& c) {
  if (c.C % 8 != 0) return false;
  return c.stride == 1 || (c.R >= c.stride && c.S >= c.stride);
}
static int bf16_out_rows(int M, int N) { return use_g256(M, N) ? (M + 255) / 256 : out_tile_rows(M, N); }
int conv_dgrad_bn_rows(const ConvShape& c) {
  if (bn_slots() > 0) return bn_slots();
  if (c.stride == 1 && use_halo(c, c.K, c.C)) return halo_geo(c, true).mtiles;
  if (c.stride == 1) return bf16_out_rows(c.N * c.H * c.W, c.C);
  int rows = 0;
  for (int ph = 0; ph < c.stride; ++ph)
    for (int pw = 0; pw < c.stride; ++pw) {
      const int Hp = (c.H - ph + c.stride - 1) / c.stride, Wp = (c.W - pw + c.stride - 1) / c.stride;
      if (Hp > 0 && Wp > 0) rows += bf16_out_rows(c.N * Hp * Wp, c.C);
    }
  return rows;
}

void conv_dgrad_bn(const ConvShape& c, const uint16_t* dy, const uint16_t* w, uint16_t* dx, hipStream_t st,
                   const uint16_t* add, const BnBwdStats& b, float* part, const uint8_t* add_bits, bool add_sub2) {
  if (c.w_override()) throw std::runtime_error("conv dgrad: width overrides are forward / weight-gradient only");
  if (!conv_dgrad_bn_supported(c)) throw std::runtime_error("conv_dgrad_bn: unsupported conv (C % 8, tap-less phases)");
  if (add_bits && (!add || c.stride != 1))
    throw std::runtime_error("conv_dgrad_bn: a relu-masked add operand needs a stride-1 dgrad");
  if (add_sub2 && !add) throw std::runtime_error("conv_dgrad_bn: stride-2 add operand without add");
  if (add_bits && add_sub2) throw std::runtime_error("conv_dgrad_bn: one add-operand form at a time");
  const AddSrc aa = make_add(c, add, add_bits, add_sub2);
  const int M = c.N * c.H * c.W, KD = c.R * c.S * c.K;
  auto go = [&](const auto& bs) {
    if (c.stride > 1) {
      dgrad_strided(c, dy, w, dx, aa, st, part, bs);
    } else if (use_halo(c, c.K, c.C)) {
      using BSt = std::decay_t<decltype(bs)>;
      if (add) halo_launch<true, true, false, BSt>(dy, w, dx, halo_geo(c, true), aa, part, st, bs);
      else halo_launch<true, false, false, BSt>(dy, w, dx, halo_geo(c, true), aa, part, st, bs);
    } else if (use_g256(M, c.C)) {
      auto g2 = [&](const auto& la, const auto& lb) {
        if (add) g256_launch_bf16<true, true, true, false>(la, lb, dx, aa, M, c.C, KD, part, st, RowId{}, 0u, bs);
        else g256_launch_bf16<true, true, false, false>(la, lb, dx, aa, M, c.C, KD, part, st, RowId{}, 0u, bs);
      };
      if (is_pointwise(c)) g2(DenseX<true>{dy, c.K, M, c.K}, DenseX<true>{w, c.K, c.C, c.K});
      else {
        Geo g = make_geo(c, M, KD);
        g2(DgradA{dy, g}, DgradB{w, g});
      }
    } else if (is_pointwise(c)) {
      dispatch_bf16_bnb(DenseX<true>{dy, c.K, M, c.K}, DenseX<true>{w, c.K, c.C, c.K}, dx, aa, M, c.C, KD, part, bs, st);
    } else {
      Geo g = make_geo(c, M, KD);
      dispatch_bf16_bnb(DgradA{dy, g}, DgradB{w, g}, dx, aa, M, c.C, KD, part, bs, st);
    }
  };
  if (b.mode == 0) go(BnB<0>{b.y, b.mean, b.invstd, b.gamma, b.beta, b.bits});
  else if (b.mode == 2) go(BnB<2>{b.y, b.mean, b.invstd, b.gamma, b.beta, b.bits});
  else if (b.mode == 3) go(BnB<3>{b.y, b.mean, b.invstd, b.gamma, b.beta, b.bits});
  else throw std::runtime_error("conv_dgrad_bn: mask mode must be 0 (no relu), 2 (from y) or 3 (relu bits)");
}

// Weight-gradient tile: dW is [R*S*C][K] with a very long reduction over pixels (split-K), so the
// block's operand traffic per MFMA decides its speed. 64x64 tiles stream 32 FLOP per staged byte,
// 128x64 43 and 128x128 64; the wide tiles are used whenever dW has the rows/columns for them
// (profiles/resnet50_wgrad_tiles_ab_r2.log: the 3x3 weight gradients 24-31 % faster than 64x64).
enum WgTile { WG64x64, WG128x64, WG128x128 };
WgTile wgrad_tile(const ConvShape& c) {
  const int MT = c.R * c.S * c.C;
  if (MT < 128) return WG64x64;
  if (c.K % 128 == 0) return WG128x128;
  return WG128x64;
}

// split-K of a weight gradient: about kWgradBlocks (tile x split) blocks, each split keeping at least
// kWgradMinPx pixels of K (round 3, 2,048: 13.80 ms, 1,024: 13.79, 512: 13.90,
// profiles/resnet50_wgrad_minpx_ab_r3.log; round 5 with the per-XCD renumbering, 3 interleaved rounds:
// 1,024 vs 2,048 ResNet-50 12.82-12.85 vs 12.86-12.92 ms, ResNet-18 4.74-4.76 vs 4.83; a 256-block
// target +0.6 ms, profiles/resnet50_wgrad_ab_r5.log; the 64x64-tile target:
// profiles/resnet50_wgrad_small_splits_ab_r4.log)
constexpr int kWgradMinPx = 1024, kWgradBlocks = 512, kWgradBlocksSmall = 512;
// weight gradients on the 256-row core: mode 2 only (the A/B switch)
static bool use_g256_wgrad(const ConvShape& c) {
  const int mode = g256_mode(), P = c.N * c.Ho() * c.Wo(), MT = c.R * c.S * c.C;
  if (mode == 0 || c.K % 8 || c.C % 8) return false;
  (void)P; (void)MT;
  return mode == 2;  // measured slower than the 128-row core on every ResNet-50 weight gradient
}
static int g256_wgrad_splits(const ConvShape& c) {
  const int P = c.N * c.Ho() * c.Wo();
  const long tiles = g256_tiles(c.R * c.S * c.C, c.K);
  int s = (int)std::max<long>(1, 256 / std::max<long>(1, tiles));
  return std::min(s, std::max(1, P / 4096));
}
int conv_wgrad_splits(const ConvShape& c, bool folded) {
  if (!folded && use_g256_wgrad(c)) return g256_wgrad_splits(c);
  // enough (tile x split) blocks to fill the chip; each split keeps >= kWgradMinPx pixels of K
  const int P = c.N * c.Ho() * c.Wo(), MT = c.R * c.S * c.C;
  const WgTile t = wgrad_tile(c);
  const int bm = t == WG64x64 ? 64 : 128, bn = t == WG128x128 ? 128 : 64;
  const long tiles = (long)((MT + bm - 1) / bm) * ((c.K + bn - 1) / bn);
  const long target = t == WG64x64 ? kWgradBlocksSmall : kWgradBlocks;
  int s = (int)std::max<long>(1, target / std::max<long>(1, tiles));
  s = std::min(s, std::max(1, P / kWgradMinPx));
  return s;
}

// Weight gradients run with the per-XCD block renumbering (gemm_kernel<XR>): ResNet-50 b128 12.98 ->
// 12.82-12.90 ms/step, l1 1x1 64->256 61 -> 44 us, l2 downsample 78 -> 63 us. Measured and not kept
// (profiles/resnet50_wgrad_ab_r5.log): two register stages, more or fewer splits, an LDS-staged atomic
// epilogue, 8-wave blocks halving each split's K over two 4-wave groups, the 256-row core with
// re-tuned splits.
template <class LA>
static void wgrad_launch(const ConvShape& c, const LA& la, const DenseX<false>& lb, const AccF32& epi, int MT, int P,
                         int splits, hipStream_t st) {
  switch (wgrad_tile(c)) {
    case WG128x128: launch_gemm<128, 128, true>(la, lb, epi, MT, c.K, P, splits, st); break;
    case WG128x64: launch_gemm<128, 64, true>(la, lb, epi, MT, c.K, P, splits, st); break;
    default: launch_gemm<64, 64, true>(la, lb, epi, MT, c.K, P, splits, st);
  }
}

// The split-K accumulator's zero fill as a kernel: a hipMemsetAsync issued into a stream capture here
// did not clear the buffer on graph replays (the width-paired stem's gradient, zeroed=False, grew to
// inf from the second replay on: tools/debug/stem_mode_check.py), so no captured path depends on it.
__global__ __launch_bounds__(256) void zero_f32_kernel(float* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = 0.f;
}
static void zero_f32(float* p, int64_t n, hipStream_t st) {  // dw may be a 4-B aligned view of a flat buffer
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(2048, (n + 255) / 256));
  zero_f32_kernel<<<grid, 256, 0, st>>>(p, n);
}

static int g_wgrad_clear = 0;
int conv_wgrad_clear_mode(int mode) {
  const int old = g_wgrad_clear;
  if (mode >= 0) g_wgrad_clear = mode;
  return old;
}

void conv_wgrad(const ConvShape& c, const uint16_t* x, const uint16_t* dy, float* dw, int splits, hipStream_t st,
                bool zeroed, const BnReluIn* act) {
  const int P = c.N * c.Ho() * c.Wo(), MT = c.R * c.S * c.C;
  if (splits > 1 && !zeroed) {
    if (g_wgrad_clear == 1) (void)hipMemsetAsync(dw, 0, (size_t)MT * c.K * sizeof(float), st);
    else zero_f32(dw, (int64_t)MT * c.K, st);
  }
  AccF32 epi{dw, MT, c.K, splits > 1 ? 1 : 0};
  DenseX<false> lb{dy, c.K, c.K, P};
  if (act) {
    const BnReluArgs a = bn_relu_args(c, act);
    if (is_pointwise(c)) wgrad_launch(c, BnRelu<DenseX<false>>{{x, c.C, c.C, P}, a}, lb, epi, MT, P, splits, st);
    else wgrad_launch(c, BnRelu<WgradA>{{x, make_geo(c, MT, P)}, a}, lb, epi, MT, P, splits, st);
    return;
  }
  if (use_g256_wgrad(c)) {  // A = im2col(X)^T, B = dY: both MNC
    if (is_pointwise(c)) g256_launch_wgrad(DenseX<false>{x, c.C, c.C, P}, lb, dw, MT, c.K, P, splits, st);
    else g256_launch_wgrad(WgradA{x, make_geo(c, MT, P)}, lb, dw, MT, c.K, P, splits, st);
    return;
  }
  if (is_pointwise(c)) {  // dW = X^T dY
    DenseX<false> la{x, c.C, c.C, P};
    wgrad_launch(c, la, lb, epi, MT, P, splits, st);
  } else {
    WgradA la{x, make_geo(c, MT, P)};
    wgrad_launch(c, la, lb, epi, MT, P, splits, st);
  }
}

int conv_halo_mode(int mode) {  // -1: query
  const int old = g_halo_mode;
  if (mode >= 0) g_halo_mode = mode;
  return old;
}
int conv_gemm_core(int mode) {  // -1: query
  const int old = g256_mode();
  if (mode >= 0) g256_mode_v = mode;
  return old;
}

void linear_fwd(const uint16_t* x, const uint16_t* w, const float* bias, float* y, int M, int Kin, int N,
                hipStream_t st) {
  DenseX<true> la{x, Kin, M, Kin};
  DenseX<false> lb{w, N, N, Kin};
  BiasStoreF32 epi{y, bias, M, N};
  dispatch(la, lb, epi, M, N, Kin, 1, st);
}

void linear_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int M, int Kin, int N, hipStream_t st) {
  // dX[M][Kin] = dY[M][N] W^T ; W is [Kin][N] -> B operand (n = kin, k = n) is k-contiguous
  DenseX<true> la{dy, N, M, N};
  DenseX<true> lb{w, N, Kin, N};
  StoreBf16 epi{dx, M, Kin};
  dispatch(la, lb, epi, M, Kin, N, 1, st);
}

void linear_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int M, int Kin, int N, hipStream_t st) {
  // dW[Kin][N] = X^T dY over the M rows
  DenseX<false> la{x, Kin, Kin, M};
  DenseX<false> lb{dy, N, N, M};
  AccF32 epi{dw, Kin, N, 0};
  dispatch(la, lb, epi, Kin, N, M, 1, st);
}

}  // namespace tfd
