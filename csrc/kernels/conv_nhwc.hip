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
#include "../common.h"
#include "../conv_kernels.h"
#include "../gemm.h"

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
  int M;       // rows of the GEMM
  int KD;      // reduction length
  FastDiv howo, wo, c, k, s, hw, w;
};

// ---- forward: A = im2col(X) (KC), B = W [KD][K] (not KC) ----
struct FwdA {
  static constexpr bool KC = true;
  const uint16_t* __restrict__ x;
  Geo g;
  __device__ __forceinline__ uint4 operator()(int m, int k) const {
    if (m >= g.M || k >= g.KD) return zero4();
    const int n = g.howo.div(m), r1 = m - n * g.Ho * g.Wo, ho = g.wo.div(r1), wo = r1 - ho * g.Wo;
    const int tap = g.c.div(k), c = k - tap * g.C, r = g.s.div(tap), s = tap - r * g.S;
    const int h = ho * g.st - g.pad + r, w = wo * g.st - g.pad + s;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return zero4();
    return *reinterpret_cast<const uint4*>(x + ((size_t)(n * g.H + h) * g.W + w) * g.C + c);
  }
};

// ---- dgrad: A = "col2im" gather of dY (KC), B = W as [C][(r,s,k)] (KC) ----
struct DgradA {
  static constexpr bool KC = true;
  const uint16_t* __restrict__ dy;
  Geo g;  // M = N*H*W, KD = R*S*K
  __device__ __forceinline__ uint4 operator()(int m, int kk) const {
    if (m >= g.M || kk >= g.KD) return zero4();
    const int n = g.hw.div(m), r1 = m - n * g.H * g.W, h = g.w.div(r1), w = r1 - h * g.W;
    const int tap = g.k.div(kk), k = kk - tap * g.K, r = g.s.div(tap), s = tap - r * g.S;
    const int hn = h + g.pad - r, wn = w + g.pad - s;
    if (hn < 0 || wn < 0) return zero4();
    int ho = hn, wo = wn;
    if (g.st != 1) {
      ho = hn / g.st;
      wo = wn / g.st;
      if (ho * g.st != hn || wo * g.st != wn) return zero4();
    }
    if (ho >= g.Ho || wo >= g.Wo) return zero4();
    return *reinterpret_cast<const uint4*>(dy + ((size_t)(n * g.Ho + ho) * g.Wo + wo) * g.K + k);
  }
};
struct DgradB {
  static constexpr bool KC = true;
  const uint16_t* __restrict__ w;
  Geo g;
  __device__ __forceinline__ uint4 operator()(int c, int kk) const {
    if (c >= g.C || kk >= g.KD) return zero4();
    const int tap = g.k.div(kk), k = kk - tap * g.K;
    return *reinterpret_cast<const uint4*>(w + ((size_t)tap * g.C + c) * g.K + k);
  }
};

// ---- wgrad: A = im2col(X)^T (not KC: chunk of 8 channels at one pixel), B = dY [pix][K] ----
struct WgradA {
  static constexpr bool KC = false;
  const uint16_t* __restrict__ x;
  Geo g;  // M = R*S*C rows (taps), KD = N*Ho*Wo pixels
  __device__ __forceinline__ uint4 operator()(int t, int m) const {
    if (t >= g.M || m >= g.KD) return zero4();
    const int tap = g.c.div(t), c = t - tap * g.C, r = g.s.div(tap), s = tap - r * g.S;
    const int n = g.howo.div(m), r1 = m - n * g.Ho * g.Wo, ho = g.wo.div(r1), wo = r1 - ho * g.Wo;
    const int h = ho * g.st - g.pad + r, w = wo * g.st - g.pad + s;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return zero4();
    return *reinterpret_cast<const uint4*>(x + ((size_t)(n * g.H + h) * g.W + w) * g.C + c);
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

template <int BM, int BN>
struct Tile {
  static constexpr int WM = 2, WN = 2, BK = 64;
};

template <int BM, int BN, class LA, class LB, class EPI>
__global__ __launch_bounds__(256) void gemm_kernel(LA la, LB lb, EPI epi, int kchunk, int KD) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int kb = blockIdx.z * kchunk, ke = min(KD, kb + kchunk);
  gemm_block<BM, BN, 64, 2, 2, LA, LB, EPI, 1>(la, lb, epi, blockIdx.y * BM, blockIdx.x * BN, kb, ke,
                                               (bf16*)smem_raw);
}

template <int BM, int BN, class LA, class LB, class EPI>
void launch_gemm(const LA& la, const LB& lb, const EPI& epi, int M, int N, int KD, int splits, hipStream_t st) {
  constexpr int sm = GemmSmem<BM, BN, 64, LA, LB>::BYTES;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<BM, BN, LA, LB, EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, sm);
    attr = true;
  }
  if (splits < 1) splits = 1;
  int kchunk = ((KD + splits - 1) / splits + 63) / 64 * 64;
  splits = (KD + kchunk - 1) / kchunk;
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, splits);
  gemm_kernel<BM, BN, LA, LB, EPI><<<grid, 256, sm, st>>>(la, lb, epi, kchunk, KD);
}

// pick 128x128 tiles when the problem has enough of them to fill the chip, else 64x64
template <class LA, class LB, class EPI>
void dispatch(const LA& la, const LB& lb, const EPI& epi, int M, int N, int KD, int splits, hipStream_t st) {
  const long big = (long)((M + 127) / 128) * ((N + 127) / 128) * splits;
  if (big >= 256 && N >= 128) launch_gemm<128, 128>(la, lb, epi, M, N, KD, splits, st);
  else launch_gemm<64, 64>(la, lb, epi, M, N, KD, splits, st);
}

Geo make_geo(const ConvShape& c, int M, int KD) {
  Geo g;
  g.N = c.N; g.H = c.H; g.W = c.W; g.C = c.C; g.K = c.K; g.R = c.R; g.S = c.S; g.st = c.stride; g.pad = c.pad;
  g.Ho = c.Ho(); g.Wo = c.Wo();
  g.M = M; g.KD = KD;
  g.howo = FastDiv(g.Ho * g.Wo); g.wo = FastDiv(g.Wo); g.c = FastDiv(g.C); g.k = FastDiv(g.K); g.s = FastDiv(g.S);
  g.hw = FastDiv(g.H * g.W); g.w = FastDiv(g.W);
  return g;
}

bool is_pointwise(const ConvShape& c) { return c.R == 1 && c.S == 1 && c.stride == 1 && c.pad == 0; }

}  // namespace

void conv_fwd(const ConvShape& c, const uint16_t* x, const uint16_t* w, uint16_t* y, hipStream_t st) {
  const int M = c.N * c.Ho() * c.Wo(), KD = c.R * c.S * c.C;
  StoreBf16 epi{y, M, c.K};
  DenseLoader<false> lb{w, c.K, c.K, KD};
  if (is_pointwise(c)) {
    DenseLoader<true> la{x, c.C, M, c.C};
    dispatch(la, lb, epi, M, c.K, KD, 1, st);
  } else {
    FwdA la{x, make_geo(c, M, KD)};
    dispatch(la, lb, epi, M, c.K, KD, 1, st);
  }
}

template <class Epi>
static void conv_dgrad_impl(const ConvShape& c, const uint16_t* dy, const uint16_t* w, Epi epi, hipStream_t st) {
  const int M = c.N * c.H * c.W, KD = c.R * c.S * c.K;
  if (is_pointwise(c)) {  // dX = dY W^T: W [C][K] read k-contiguous
    DenseLoader<true> la{dy, c.K, M, c.K};
    DenseLoader<true> lb{w, c.K, c.C, c.K};
    dispatch(la, lb, epi, M, c.C, KD, 1, st);
  } else {
    Geo g = make_geo(c, M, KD);
    DgradA la{dy, g};
    DgradB lb{w, g};
    dispatch(la, lb, epi, M, c.C, KD, 1, st);
  }
}

void conv_dgrad(const ConvShape& c, const uint16_t* dy, const uint16_t* w, uint16_t* dx, hipStream_t st,
                const uint16_t* add) {
  const int M = c.N * c.H * c.W;
  if (add) conv_dgrad_impl(c, dy, w, AddStoreBf16{dx, add, M, c.C}, st);
  else conv_dgrad_impl(c, dy, w, StoreBf16{dx, M, c.C}, st);
}

void conv_wgrad(const ConvShape& c, const uint16_t* x, const uint16_t* dy, float* dw, int splits, hipStream_t st,
                bool zeroed) {
  const int P = c.N * c.Ho() * c.Wo(), MT = c.R * c.S * c.C;
  if (splits > 1 && !zeroed) (void)hipMemsetAsync(dw, 0, (size_t)MT * c.K * sizeof(float), st);
  AccF32 epi{dw, MT, c.K, splits > 1 ? 1 : 0};
  DenseLoader<false> lb{dy, c.K, c.K, P};
  if (is_pointwise(c)) {  // dW = X^T dY
    DenseLoader<false> la{x, c.C, c.C, P};
    dispatch(la, lb, epi, MT, c.K, P, splits, st);
  } else {
    WgradA la{x, make_geo(c, MT, P)};
    dispatch(la, lb, epi, MT, c.K, P, splits, st);
  }
}

int conv_wgrad_splits(const ConvShape& c) {
  // enough (tile x split) blocks to fill the chip; each split keeps >= 2048 pixels of K
  const int P = c.N * c.Ho() * c.Wo(), MT = c.R * c.S * c.C;
  const long tiles = (long)((MT + 63) / 64) * ((c.K + 63) / 64);
  int s = (int)std::max<long>(1, 512 / std::max<long>(1, tiles));
  s = std::min(s, std::max(1, P / 2048));
  return s;
}

void linear_fwd(const uint16_t* x, const uint16_t* w, const float* bias, float* y, int M, int Kin, int N,
                hipStream_t st) {
  DenseLoader<true> la{x, Kin, M, Kin};
  DenseLoader<false> lb{w, N, N, Kin};
  BiasStoreF32 epi{y, bias, M, N};
  dispatch(la, lb, epi, M, N, Kin, 1, st);
}

void linear_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int M, int Kin, int N, hipStream_t st) {
  // dX[M][Kin] = dY[M][N] W^T ; W is [Kin][N] -> B operand (n = kin, k = n) is k-contiguous
  DenseLoader<true> la{dy, N, M, N};
  DenseLoader<true> lb{w, N, Kin, N};
  StoreBf16 epi{dx, M, Kin};
  dispatch(la, lb, epi, M, Kin, N, 1, st);
}

void linear_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int M, int Kin, int N, hipStream_t st) {
  // dW[Kin][N] = X^T dY over the M rows
  DenseLoader<false> la{x, Kin, Kin, M};
  DenseLoader<false> lb{dy, N, N, M};
  AccF32 epi{dw, Kin, N, 0};
  dispatch(la, lb, epi, Kin, N, M, 1, st);
}

}  // namespace tfd
