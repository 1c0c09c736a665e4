// Batch normalisation (training + inference), pooling and the softmax-cross-entropy head for the
// NHWC ResNet-style models (see csrc/conv_kernels.h). Activations are bf16 [M = N*H*W][C]; all
// statistics and parameter gradients are fp32. Reductions are two-level and deterministic:
// per-block partials over a row chunk (8 channels per thread, 16-B loads), then a per-channel
// finalize kernel in a fixed order.
#include <stdexcept>

#include "../common.h"
#include "../conv_kernels.h"
#include "../gemm.h"  // buf_ld
#include "../bn_affine.h"

// (Round 2 measured a variant that summed the statistics in the producing launch by last-arriver
// tickets instead of the bn_final launch: ResNet-50 b128 13.98 -> 17.60 ms/step, the hand-off words
// need write-through / sc1 round trips and the last group's reduction is a serial tail after every
// other block -- profiles/resnet50_bn_totals_ab_r2.log. Removed in round 4.)

namespace tfd {
namespace {

constexpr int NT = 256;

struct RowSplit {
  int tpr;   // threads per row (one 8-channel chunk each, C/8 <= 256)
  int rg;    // row groups per block
  int nblk;  // blocks
  int rb;    // rows per block
};
RowSplit row_split(int M, int C) {
  RowSplit r;
  r.tpr = C / 8;
  r.rg = NT / r.tpr;
  r.nblk = std::max(1, std::min(1024, (M + 31) / 32));
  r.rb = (M + r.nblk - 1) / r.nblk;
  r.nblk = (M + r.rb - 1) / r.rb;
  return r;
}

__device__ __forceinline__ void unpack8(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
}

// The backward's relu mask is (out > 0). Without a residual, out = relu(y * sc + sh) with the
// forward's per-channel sc = invstd * gamma, sh = beta - mean * sc (bn_apply_kernel), so the mask
// is recomputed from y -- the same fmaf, bit for bit -- instead of reading `out` (one bf16 array
// less per backward pass). out == nullptr selects that form (bn_backward: residual-free BNs).
__device__ __forceinline__ void relu_mask_from_y(const float (&v)[8], const float (&sc)[8], const float (&sh)[8],
                                                 float (&d)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = fmaf(v[j], sc[j], sh[j]) > 0.f ? d[j] : 0.f;
}

// MASK 3: the forward's relu mask as bits ([M][C/8] bytes, bit j = channel c0 + j of the chunk was
// > 0 after the relu), written by bn_apply_kernel for the residual BNs, where the mask cannot be
// recomputed from y alone: the backward reads 1 bit instead of the 16-bit output per element
// (two full-tensor reads of `out` per residual BN backward). Rows past the chunk read a clamped
// in-range byte (branch-free); their dout is zero-filled, so the bits do not matter.
__device__ __forceinline__ uint32_t mask_byte(const uint8_t* __restrict__ mask, int r, int r1, int cpr, int ch) {
  return mask[(size_t)min(r, r1 - 1) * cpr + ch];
}
__device__ __forceinline__ void apply_mask_bits(uint32_t bits, float (&d)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = (bits >> j) & 1u ? d[j] : 0.f;
}

// Rows are walked in batches of RU rows per thread: every 16-B load of a batch (y, dout, out) is
// issued before the first use, through buffer descriptors whose hardware range check zero-fills the
// rows past the block's chunk (no exec-masked branch around a load, so the loads of a batch are all
// in flight together). With one row per iteration these kernels waited one memory latency per row.
// rows per batch of the BN passes, all their loads issued before the first use (2 and 8 measured no
// better, profiles/resnet50_bn_ru_ab_r4.log)
constexpr int RU = 4;
__device__ __forceinline__ uint4 row_ld(const uint16_t* base, uint32_t nbytes, int r, int r1, int C, int c0) {
  return buf_ld(base, nbytes, (uint32_t)r * (uint32_t)C + (uint32_t)c0, r < r1);
}

// partial sums of (a, b) per channel over a row chunk; MODE 0: a = y, b = y^2 ; MODE 1 (backward):
// a = dz, b = dz * xhat with dz = relu-masked dout. MASK (MODE 1): 0 no relu, 1 mask = out > 0,
// 2 mask recomputed from y (relu_mask_from_y).
template <int MODE, int MASK>
__global__ __launch_bounds__(NT) void bn_partial_kernel(const uint16_t* __restrict__ y,
                                                        const uint16_t* __restrict__ dout,
                                                        const uint16_t* __restrict__ out,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, int M, int C, int tpr,
                                                        int rg, int rb, float* __restrict__ part,
                                                        const uint8_t* __restrict__ mbits) {
  __shared__ float red[2][NT][8];
  const int t = threadIdx.x, ch = t % tpr, g = t / tpr, c0 = ch * 8;
  const uint32_t nbytes = (uint32_t)M * (uint32_t)C * 2u;
  float sa[8], sb[8], mu[8], is[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sa[j] = 0.f; sb[j] = 0.f; }
  if (MODE == 1 && g < rg) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mu[j] = mean[c0 + j];
      is[j] = invstd[c0 + j];
      if (MASK == 2) bn_affine(mu[j], is[j], gamma[c0 + j], beta[c0 + j], sc[j], sh[j]);
    }
  }
  const int r0 = blockIdx.x * rb, r1 = min(M, r0 + rb);
  if (g < rg) {
    for (int rbase = r0 + g; rbase < r1; rbase += RU * rg) {
      uint4 Y[RU], D[RU], O[RU];
      uint32_t MB[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int r = rbase + u * rg;
        Y[u] = row_ld(y, nbytes, r, r1, C, c0);
        if (MODE == 1) D[u] = row_ld(dout, nbytes, r, r1, C, c0);
        if (MODE == 1 && MASK == 1) O[u] = row_ld(out, nbytes, r, r1, C, c0);
        if (MODE == 1 && MASK == 3) MB[u] = mask_byte(mbits, r, r1, tpr, ch);
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {  // rows past r1 loaded as zeros: they add nothing
        float v[8];
        unpack8(Y[u], v);
        if (MODE == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) { sa[j] += v[j]; sb[j] = fmaf(v[j], v[j], sb[j]); }
        } else {
          float d[8];
          unpack8(D[u], d);
          if (MASK == 1) {
            float ov[8];
            unpack8(O[u], ov);
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = ov[j] > 0.f ? d[j] : 0.f;
          } else if (MASK == 2) {
            relu_mask_from_y(v, sc, sh, d);
          } else if (MASK == 3) {
            apply_mask_bits(MB[u], d);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) { sa[j] += d[j]; sb[j] = fmaf(d[j], (v[j] - mu[j]) * is[j], sb[j]); }
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][t][j] = sa[j]; red[1][t][j] = sb[j]; }
  __syncthreads();
  if ((rg & (rg - 1)) == 0) {  // power-of-two row groups: log2(rg) tree levels instead of rg - 1 serial adds
    for (int h = rg >> 1; h > 0; h >>= 1) {
      if (g < h) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sa[j] += red[0][t + h * tpr][j];
          sb[j] += red[1][t + h * tpr][j];
          red[0][t][j] = sa[j];
          red[1][t][j] = sb[j];
        }
      }
      __syncthreads();
    }
  } else if (g == 0) {
    for (int q = 1; q < rg; ++q) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { sa[j] += red[0][q * tpr + ch][j]; sb[j] += red[1][q * tpr + ch][j]; }
    }
  }
  if (g == 0) {  // always one row per block (the partial pass is followed by bn_final in either mode)
    float* pa = part + (size_t)blockIdx.x * 2 * C;
#pragma unroll
    for (int j = 0; j < 8; ++j) { pa[c0 + j] = sa[j]; pa[C + c0 + j] = sb[j]; }
  }
}

// per-channel finalize, block = 32 channels x 32 partial-row groups (1024 threads: coalesced 128-B
// rows, 4 independent loads in flight per thread, fixed summation order, so deterministic).
// mode 0: mean/invstd (+running stats); mode 1: dbeta/dgamma. It is one dependent chain between
// the partial and apply kernels, so it is latency-bound: more rows in flight, fewer trips.
constexpr int FIN_G = 32, FIN_NT = 32 * FIN_G;
__global__ __launch_bounds__(FIN_NT) void bn_final_kernel(int mode, const float* __restrict__ part, int nblk, int M,
                                                          int C, float eps, float momentum, float* __restrict__ o0,
                                                          float* __restrict__ o1, float* __restrict__ rmean,
                                                          float* __restrict__ rvar) {
  __shared__ float red[2][FIN_G][33];
  const int cl = threadIdx.x & 31, q = threadIdx.x >> 5, c = blockIdx.x * 32 + cl;
  float a = 0.f, b = 0.f;
  if (c < C) {
    const size_t st = (size_t)FIN_G * 2 * C;
    int k = q;
    for (; k + 3 * FIN_G < nblk; k += 4 * FIN_G) {
      const float* p0 = part + (size_t)k * 2 * C + c;
      a += (p0[0] + p0[st]) + (p0[2 * st] + p0[3 * st]);
      b += (p0[C] + p0[st + C]) + (p0[2 * st + C] + p0[3 * st + C]);
    }
    for (; k < nblk; k += FIN_G) {
      a += part[(size_t)k * 2 * C + c];
      b += part[(size_t)k * 2 * C + C + c];
    }
  }
  red[0][q][cl] = a;
  red[1][q][cl] = b;
  __syncthreads();
  if (q != 0 || c >= C) return;
  a = 0.f;
  b = 0.f;
#pragma unroll
  for (int j = 0; j < FIN_G; ++j) { a += red[0][j][cl]; b += red[1][j][cl]; }
  if (mode == 0) {
    const float mu = a / (float)M;
    const float var = fmaxf(b / (float)M - mu * mu, 0.f);
    o0[c] = mu;
    o1[c] = rsqrtf(var + eps);
    if (rmean) {
      rmean[c] = rmean[c] * momentum + mu * (1.f - momentum);
      rvar[c] = rvar[c] * momentum + var * ((float)M / (float)max(M - 1, 1)) * (1.f - momentum);
    }
  } else {
    o0[c] = a;  // dbeta
    o1[c] = b;  // dgamma
  }
}

// Inline finalize (slot mode, bn_slots() > 0): the apply passes read the S slot sums of a zeroed
// [S][2][C] buffer that the producer filled with atomics, instead of waiting on a bn_final launch.
// Threads g == 0 (one per 8-channel chunk) sum the slots of their chunk, hand the block's per-channel
// constants to the other row groups through LDS; block 0 also writes the statistics out (mean /
// invstd + running stats forward, dbeta / dgamma backward) with bn_final_kernel's formulas.
struct BnFin {
  const float* part;  // [slots][2][C]
  int slots;
  float eps, momentum;
  float *o0, *o1;       // forward: mean, invstd; backward: dbeta, dgamma (written by block 0)
  float *rmean, *rvar;  // forward running statistics (optional)
};
constexpr int FIN_MAXC = 2048;
constexpr int FIN_MAXS = 8;  // slot counts the inline finalize takes (set_bn_slots bounds it)
// Stage 1 (before the barrier): row group g < G = min(rg, S) sums slots g, g + G, ... of its thread's
// 8 channels and parks the pair in LDS [G][2][C] (rg * C = 2048, so at most 16 KB); stage 2 (after
// it): every thread sums the G parked pairs of its channels. Fixed order, so every block of the
// launch forms bit-identical statistics.
__device__ __forceinline__ void fin_stage(const BnFin& f, int C, int c0, int g, int rg, float* lds) {
  const int G = min(rg, f.slots);
  if (g >= G) return;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, b0 = a0, b1 = a0;
  for (int q = g; q < f.slots; q += G) {
    const f32x4* pa = reinterpret_cast<const f32x4*>(f.part + (size_t)q * 2 * C + c0);
    const f32x4* pb = reinterpret_cast<const f32x4*>(f.part + (size_t)q * 2 * C + C + c0);
    a0 += pa[0];
    a1 += pa[1];
    b0 += pb[0];
    b1 += pb[1];
  }
  f32x4* la = reinterpret_cast<f32x4*>(lds + (size_t)g * 2 * C + c0);
  f32x4* lb = reinterpret_cast<f32x4*>(lds + (size_t)g * 2 * C + C + c0);
  la[0] = a0;
  la[1] = a1;
  lb[0] = b0;
  lb[1] = b1;
}
__device__ __forceinline__ void fin_sums(const BnFin& f, int C, int c0, int rg, const float* lds, float (&a)[8],
                                         float (&b)[8]) {
  const int G = min(rg, f.slots);
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = 0.f; b[j] = 0.f; }
  for (int q = 0; q < G; ++q) {
    const f32x4* la = reinterpret_cast<const f32x4*>(lds + (size_t)q * 2 * C + c0);
    const f32x4* lb = reinterpret_cast<const f32x4*>(lds + (size_t)q * 2 * C + C + c0);
    const f32x4 a0 = la[0], a1 = la[1], b0 = lb[0], b1 = lb[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] += a0[j];
      a[4 + j] += a1[j];
      b[j] += b0[j];
      b[4 + j] += b1[j];
    }
  }
}

// Elementwise passes walk the same row split as the partial kernel: thread = (8-channel chunk,
// row group); its 8 channels' constants stay in registers for every row it touches; RU rows' loads
// per batch are issued before the first use (branch-free buffer loads, see bn_partial_kernel).
// HAS_RES / RELU are compile-time so no load sits under a branch.
template <bool HAS_RES, bool RELU, bool FIN = false>
__global__ __launch_bounds__(NT) void bn_apply_kernel(const uint16_t* __restrict__ y, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, const float* __restrict__ mean,
                                                      const float* __restrict__ invstd,
                                                      const uint16_t* __restrict__ res,
                                                      uint16_t* __restrict__ out, int M, int C, int tpr, int rg, int rb,
                                                      uint8_t* __restrict__ mbits, BnFin fin = BnFin{}) {
  const int t = threadIdx.x, ch = t % tpr, g = t / tpr, c0 = ch * 8;
  const uint32_t nbytes = (uint32_t)M * (uint32_t)C * 2u;
  const int r0 = blockIdx.x * rb, r1 = min(M, r0 + rb);
  uint4 Y[RU], Q[RU];
  auto load = [&](int rs) {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      Y[u] = row_ld(y, nbytes, rs + u * rg, r1, C, c0);
      if (HAS_RES) Q[u] = row_ld(res, nbytes, rs + u * rg, r1, C, c0);
    }
  };
  int rbase = r0 + g;
  float sc[8], sh[8];
  if constexpr (FIN) {
    // the finalize's operands (gamma, beta, the slot sums) and the block's first row batch are in
    // flight together: one memory latency before the barrier
    float gm[8], bt[8];
    __shared__ float fl[FIN_MAXC * 2];
#pragma unroll
    for (int j = 0; j < 8; ++j) { gm[j] = gamma[c0 + j]; bt[j] = beta[c0 + j]; }
    fin_stage(fin, C, c0, g, rg, fl);
    if (g < rg) load(rbase);
    __syncthreads();
    if (g >= rg) return;
    float a[8], b[8];
    fin_sums(fin, C, c0, rg, fl, a, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      const float mu = a[j] / (float)M;
      const float var = fmaxf(b[j] / (float)M - mu * mu, 0.f);
      const float is = rsqrtf(var + fin.eps);
      if (blockIdx.x == 0 && g == 0) {
        fin.o0[c] = mu;
        fin.o1[c] = is;
        if (fin.rmean) {
          fin.rmean[c] = fin.rmean[c] * fin.momentum + mu * (1.f - fin.momentum);
          fin.rvar[c] = fin.rvar[c] * fin.momentum + var * ((float)M / (float)max(M - 1, 1)) * (1.f - fin.momentum);
        }
      }
      bn_affine(mu, is, gm[j], bt[j], sc[j], sh[j]);
    }
  } else {
    if (g >= rg) return;
#pragma unroll
    for (int j = 0; j < 8; ++j) bn_affine(mean[c0 + j], invstd[c0 + j], gamma[c0 + j], beta[c0 + j], sc[j], sh[j]);
    load(rbase);
  }
  for (; rbase < r1; rbase += RU * rg) {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = rbase + u * rg;
      uint4 o;
      if constexpr (RELU && !HAS_RES) {  // the folded conv loaders' form (bn_relu2), bit for bit
        o.x = bn_relu2(Y[u].x, (bn_f32x2){sc[0], sc[1]}, (bn_f32x2){sh[0], sh[1]});
        o.y = bn_relu2(Y[u].y, (bn_f32x2){sc[2], sc[3]}, (bn_f32x2){sh[2], sh[3]});
        o.z = bn_relu2(Y[u].z, (bn_f32x2){sc[4], sc[5]}, (bn_f32x2){sh[4], sh[5]});
        o.w = bn_relu2(Y[u].w, (bn_f32x2){sc[6], sc[7]}, (bn_f32x2){sh[6], sh[7]});
      } else {
        float v[8], q[8];
        unpack8(Y[u], v);
        if (HAS_RES) unpack8(Q[u], q);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float z = fmaf(v[j], sc[j], sh[j]);
          if (HAS_RES) z += q[j];
          v[j] = RELU ? fmaxf(z, 0.f) : z;
        }
        o = pack8(v);
      }
      if (r < r1) {
        *reinterpret_cast<uint4*>(out + (size_t)r * C + c0) = o;
        if (RELU && mbits) {  // bit j: the stored bf16 output of channel c0 + j is > 0
          const uint32_t w[4] = {o.x, o.y, o.z, o.w};
          uint32_t b = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) b |= ((w[k] & 0xFFFFu) ? 1u : 0u) << (2 * k) | ((w[k] >> 16) ? 1u : 0u) << (2 * k + 1);
          mbits[(size_t)r * tpr + ch] = (uint8_t)b;
        }
      }
    }
    if (rbase + RU * rg < r1) load(rbase + RU * rg);
  }
}

// MASK: 0 no relu, 1 mask = out > 0, 2 mask recomputed from y
template <int MASK, bool FIN = false>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(const uint16_t* __restrict__ dout,
                                                          const uint16_t* __restrict__ out, const uint16_t* __restrict__ y,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, const float* __restrict__ dbeta,
                                                          const float* __restrict__ dgamma,
                                                          uint16_t* __restrict__ dy, uint16_t* __restrict__ dres,
                                                          int M, int C, int tpr, int rg, int rb, float invM,
                                                          const uint8_t* __restrict__ mbits, BnFin fin = BnFin{}) {
  const int t = threadIdx.x, ch = t % tpr, g = t / tpr, c0 = ch * 8;
  const uint32_t nbytes = (uint32_t)M * (uint32_t)C * 2u;
  const int r0 = blockIdx.x * rb, r1 = min(M, r0 + rb);
  uint4 D[RU], Y[RU], O[RU];
  uint32_t MB[RU];
  auto load = [&](int rs) {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = rs + u * rg;
      D[u] = row_ld(dout, nbytes, r, r1, C, c0);
      Y[u] = row_ld(y, nbytes, r, r1, C, c0);
      if (MASK == 1) O[u] = row_ld(out, nbytes, r, r1, C, c0);
      if (MASK == 3) MB[u] = mask_byte(mbits, r, r1, tpr, ch);
    }
  };
  int rbase = r0 + g;
  float db[8], dg[8];
  // the per-channel operands, issued before any wait (the FIN barrier included)
  float gm[8], is8[8], mu8[8], bt8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    gm[j] = gamma[c0 + j];
    is8[j] = invstd[c0 + j];
    mu8[j] = mean[c0 + j];
    if (MASK == 2) bt8[j] = beta[c0 + j];
  }
  if constexpr (FIN) {  // dbeta / dgamma from the slot sums (block 0 writes them out)
    __shared__ float fl[FIN_MAXC * 2];
    fin_stage(fin, C, c0, g, rg, fl);
    if (g < rg) load(rbase);  // the first batch is in flight while the sums are read
    __syncthreads();
    if (g >= rg) return;
    fin_sums(fin, C, c0, rg, fl, db, dg);
    if (blockIdx.x == 0 && g == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        fin.o0[c0 + j] = db[j];
        fin.o1[c0 + j] = dg[j];
      }
    }
  } else {
    if (g >= rg) return;
#pragma unroll
    for (int j = 0; j < 8; ++j) { db[j] = dbeta[c0 + j]; dg[j] = dgamma[c0 + j]; }
    load(rbase);
  }
  // dy = k1 * dz + k2 * y + k3 with k1 = gamma*invstd, k2 = -k1*invstd*dgamma/M,
  // k3 = -k1*(dbeta/M - mean*invstd^2*dgamma/M)
  float k1[8], k2[8], k3[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float is = is8[j];
    k1[j] = gm[j] * is;
    k2[j] = -k1[j] * is * dg[j] * invM;
    k3[j] = -k1[j] * (db[j] * invM - mu8[j] * is * dg[j] * invM);
    if (MASK == 2) bn_affine(mu8[j], is, gm[j], bt8[j], sc[j], sh[j]);  // the forward's constants (mask from y)
  }
  for (; rbase < r1; rbase += RU * rg) {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = rbase + u * rg;
      float d[8], v[8];
      unpack8(D[u], d);
      unpack8(Y[u], v);
      if (MASK == 1) {
        float ov[8];
        unpack8(O[u], ov);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = ov[j] > 0.f ? d[j] : 0.f;
      } else if (MASK == 2) {
        relu_mask_from_y(v, sc, sh, d);
      } else if (MASK == 3) {
        apply_mask_bits(MB[u], d);
      }
      float w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = fmaf(k1[j], d[j], fmaf(k2[j], v[j], k3[j]));
      if (r < r1) {
        const size_t o = (size_t)r * C + c0;
        if (dres) *reinterpret_cast<uint4*>(dres + o) = pack8(d);
        *reinterpret_cast<uint4*>(dy + o) = pack8(w);
      }
    }
    if (rbase + RU * rg < r1) load(rbase + RU * rg);
  }
}

__global__ __launch_bounds__(NT) void bn_infer_kernel(const uint16_t* __restrict__ y, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, const float* __restrict__ rm,
                                                      const float* __restrict__ rv, float eps, int relu,
                                                      uint16_t* __restrict__ out, int64_t nchunks, int C) {
  const int64_t stride = (int64_t)gridDim.x * NT;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < nchunks; i += stride) {
    const int c0 = (int)((i * 8) % C);
    float v[8];
    unpack8(reinterpret_cast<const uint4*>(y)[i], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      const float z = (v[j] - rm[c]) * rsqrtf(rv[c] + eps) * gamma[c] + beta[c];
      v[j] = relu ? fmaxf(z, 0.f) : z;
    }
    reinterpret_cast<uint4*>(out)[i] = pack8(v);
  }
}

// ---- pooling ----
__global__ __launch_bounds__(NT) void maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                         uint8_t* __restrict__ am, int N, int H, int W, int C, int k,
                                                         int st, int pad, int Ho, int Wo) {
  const int64_t total = (int64_t)N * Ho * Wo * (C / 8);
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= total) return;
  const int cc = (int)(i % (C / 8));
  int64_t p = i / (C / 8);
  const int wo = (int)(p % Wo);
  p /= Wo;
  const int ho = (int)(p % Ho);
  const int n = (int)(p / Ho);
  float best[8];
  uint8_t arg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
  for (int r = 0; r < k; ++r) {
    const int h = ho * st - pad + r;
    if ((unsigned)h >= (unsigned)H) continue;
    for (int s = 0; s < k; ++s) {
      const int w = wo * st - pad + s;
      if ((unsigned)w >= (unsigned)W) continue;
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(x + ((size_t)(n * H + h) * W + w) * C + cc * 8), v);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (v[j] > best[j]) { best[j] = v[j]; arg[j] = (uint8_t)(r * k + s); }
    }
  }
  reinterpret_cast<uint4*>(y)[i] = pack8(best);
  uint32_t lo = arg[0] | arg[1] << 8 | arg[2] << 16 | (uint32_t)arg[3] << 24;
  uint32_t hi = arg[4] | arg[5] << 8 | arg[6] << 16 | (uint32_t)arg[7] << 24;
  reinterpret_cast<uint2*>(am)[i] = make_uint2(lo, hi);
}

// gather form: every input element sums the output windows whose argmax points at it
// The stem's relu(bn(y)) -> max pool in one pass: the BN output (the largest activation of a ResNet,
// 112x112x64 per image) is never written or re-read. Thread = (8-channel chunk, row group) as in the
// apply passes, so the inline finalize (FIN, slot mode) is bn_apply_kernel's; each thread then walks
// pooled pixels grid-stride. A window's KMAX^2 16-B loads are issued together (range-checked buffer
// loads, no branch); every tap goes through bn_relu2 -- bn_apply's packed form, bit for bit -- before
// the max, so output and argmax equal bn_apply + maxpool_fwd_kernel's (strict >, taps in r, s order).
constexpr int POOL_KMAX = 3;
template <bool FIN>
__global__ __launch_bounds__(NT) void bn_relu_maxpool_kernel(const uint16_t* __restrict__ y, const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, const float* __restrict__ mean,
                                                             const float* __restrict__ invstd, uint16_t* __restrict__ out,
                                                             uint8_t* __restrict__ am, int N, int H, int W, int C, int k,
                                                             int st, int pad, int Ho, int Wo, BnFin fin) {
  const int tpr = C / 8, t = threadIdx.x, ch = t % tpr, g = t / tpr, rg = NT / tpr, c0 = ch * 8;
  const int M = N * H * W;
  bn_f32x2 sc2[4], sh2[4];
  float sc[8], sh[8];
  if constexpr (FIN) {
    __shared__ float fl[FIN_MAXC * 2];
    float gm[8], bt[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { gm[j] = gamma[c0 + j]; bt[j] = beta[c0 + j]; }
    fin_stage(fin, C, c0, g, rg, fl);
    __syncthreads();
    if (g >= rg) return;
    float a[8], b[8];
    fin_sums(fin, C, c0, rg, fl, a, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      const float mu = a[j] / (float)M;
      const float var = fmaxf(b[j] / (float)M - mu * mu, 0.f);
      const float is = rsqrtf(var + fin.eps);
      if (blockIdx.x == 0 && g == 0) {
        fin.o0[c] = mu;
        fin.o1[c] = is;
        if (fin.rmean) {
          fin.rmean[c] = fin.rmean[c] * fin.momentum + mu * (1.f - fin.momentum);
          fin.rvar[c] = fin.rvar[c] * fin.momentum + var * ((float)M / (float)max(M - 1, 1)) * (1.f - fin.momentum);
        }
      }
      bn_affine(mu, is, gm[j], bt[j], sc[j], sh[j]);
    }
  } else {
    if (g >= rg) return;
#pragma unroll
    for (int j = 0; j < 8; ++j) bn_affine(mean[c0 + j], invstd[c0 + j], gamma[c0 + j], beta[c0 + j], sc[j], sh[j]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    sc2[q] = (bn_f32x2){sc[2 * q], sc[2 * q + 1]};
    sh2[q] = (bn_f32x2){sh[2 * q], sh[2 * q + 1]};
  }
  const uint32_t ybytes = (uint32_t)M * (uint32_t)C * 2u;
  // blocks walk output rows (n, ho), the row groups its pixels: no per-pixel integer division
  for (int row = blockIdx.x; row < N * Ho; row += gridDim.x) {
   const int n = row / Ho, ho = row - n * Ho;
   for (int wo = g; wo < Wo; wo += rg) {
    const int64_t px = (int64_t)row * Wo + wo;
    uint4 v[POOL_KMAX * POOL_KMAX];
    bool ok[POOL_KMAX * POOL_KMAX];
#pragma unroll
    for (int r = 0; r < POOL_KMAX; ++r)
#pragma unroll
      for (int s = 0; s < POOL_KMAX; ++s) {
        const int h = ho * st - pad + r, w = wo * st - pad + s;
        const bool in = r < k && s < k && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        ok[r * POOL_KMAX + s] = in;
        v[r * POOL_KMAX + s] = buf_ld(y, ybytes, ((uint32_t)(n * H + h) * (uint32_t)W + (uint32_t)w) * (uint32_t)C + c0, in);
      }
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
#pragma unroll
    for (int r = 0; r < POOL_KMAX; ++r)
#pragma unroll
      for (int s = 0; s < POOL_KMAX; ++s) {
        if (!ok[r * POOL_KMAX + s]) continue;
        const uint4 q = v[r * POOL_KMAX + s];
        const uint32_t o[4] = {bn_relu2(q.x, sc2[0], sh2[0]), bn_relu2(q.y, sc2[1], sh2[1]), bn_relu2(q.z, sc2[2], sh2[2]),
                               bn_relu2(q.w, sc2[3], sh2[3])};
        float f[8];
        unpack8(make_uint4(o[0], o[1], o[2], o[3]), f);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f[j] > best[j]) { best[j] = f[j]; arg[j] = (uint8_t)(r * k + s); }
      }
    const size_t oi = (size_t)px * C + c0;
    *reinterpret_cast<uint4*>(out + oi) = pack8(best);
    const uint32_t lo = arg[0] | arg[1] << 8 | arg[2] << 16 | (uint32_t)arg[3] << 24;
    const uint32_t hi = arg[4] | arg[5] << 8 | arg[6] << 16 | (uint32_t)arg[7] << 24;
    *reinterpret_cast<uint2*>(am + oi) = make_uint2(lo, hi);
   }
  }
}

// Max-pool backward at most 2x2 windows per input pixel (ceil(k / st) <= 2: the ResNet stem's 3x3/2)
// with every window's dy / argmax loads issued together (range-checked buffer loads), and -- STATS --
// the backward statistics of the relu BN in front of the pool summed on the way (bn_partial_kernel<1,
// 2>'s math: d = dx through the relu mask recomputed from y, sums of d and d * xhat), so that BN's
// backward needs no partial pass over dx and y. Thread = (8-channel chunk, row group), walking input
// pixels grid-stride; windows in maxpool_bwd_kernel's order, so dx is the same bit for bit.
// Max-pool backward for at most 2x2 windows per input pixel (ceil(k / st) <= 2: the ResNet stem's
// 3x3/2): blocks walk input rows (n, h) -- no per-pixel division by runtime sizes -- and a pixel's
// window loads (dy, argmax) are issued together as range-checked buffer loads, so no load waits
// behind a branch. Windows in maxpool_bwd_kernel's order: the same dx bit for bit. ResNet-50 stem
// (128 x 112 x 112 x 64): 109 -> 84-88 us. (Summing the stem BN's backward statistics here as well
// measured 150-158 us in row mode and 173-273 in slot mode against 87 + the 79-us partial pass:
// not kept, tools/debug/pool_probe.py.)
__global__ __launch_bounds__(NT) void maxpool2_bwd_kernel(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ am,
                                                          uint16_t* __restrict__ dx, int N, int H, int W, int C, int k,
                                                          int st, int pad, int Ho, int Wo) {
  const int tpr = C / 8, t = threadIdx.x, ch = t % tpr, g = t / tpr, rg = NT / tpr, c0 = ch * 8;
  if (g >= rg) return;
  const uint32_t dybytes = (uint32_t)N * Ho * Wo * C * 2u, ambytes = dybytes / 2u;
  for (int row = blockIdx.x; row < N * H; row += gridDim.x) {
    const int n = row / H, h = row - n * H;
    const int ho_lo = max(0, (h + pad - k + st) / st), ho_hi = min(Ho - 1, (h + pad) / st);
    for (int w = g; w < W; w += rg) {
      const int wo_lo = max(0, (w + pad - k + st) / st), wo_hi = min(Wo - 1, (w + pad) / st);
      uint4 G[2][2];
      uint2 A[2][2];
      int tap[2][2];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int ho = ho_lo + a, wo = wo_lo + b, r = h + pad - ho * st, s = w + pad - wo * st;
          const bool ok = ho <= ho_hi && wo <= wo_hi && r >= 0 && r < k && s >= 0 && s < k;
          tap[a][b] = ok ? r * k + s : -1;
          const uint32_t o = ((uint32_t)(n * Ho + ho) * (uint32_t)Wo + (uint32_t)wo) * (uint32_t)C + (uint32_t)c0;
          G[a][b] = buf_ld(dy, dybytes, o, ok);
          // the chunk's 8 argmax bytes (a 16-B load whose upper half is ignored; the range check
          // zero-fills a last chunk's overhang)
          const uint4 q = buf_ld(reinterpret_cast<const uint16_t*>(am), ambytes, o / 2u, ok);
          A[a][b] = make_uint2(q.x, q.y);
        }
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          if (tap[a][b] < 0) continue;
          float gv[8];
          unpack8(G[a][b], gv);
          const uint8_t* ab = reinterpret_cast<const uint8_t*>(&A[a][b]);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (ab[j] == (uint8_t)tap[a][b]) acc[j] += gv[j];
        }
      *reinterpret_cast<uint4*>(dx + ((size_t)row * W + w) * C + c0) = pack8(acc);
    }
  }
}

__global__ __launch_bounds__(NT) void maxpool_bwd_kernel(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ am,
                                                         uint16_t* __restrict__ dx, int N, int H, int W, int C, int k,
                                                         int st, int pad, int Ho, int Wo) {
  const int64_t total = (int64_t)N * H * W * (C / 8);
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= total) return;
  const int cc = (int)(i % (C / 8));
  int64_t p = i / (C / 8);
  const int w = (int)(p % W);
  p /= W;
  const int h = (int)(p % H);
  const int n = (int)(p / H);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const int ho_lo = max(0, (h + pad - k + st) / st), ho_hi = min(Ho - 1, (h + pad) / st);
  const int wo_lo = max(0, (w + pad - k + st) / st), wo_hi = min(Wo - 1, (w + pad) / st);
  for (int ho = ho_lo; ho <= ho_hi; ++ho) {
    const int r = h + pad - ho * st;
    if (r < 0 || r >= k) continue;
    for (int wo = wo_lo; wo <= wo_hi; ++wo) {
      const int s = w + pad - wo * st;
      if (s < 0 || s >= k) continue;
      const size_t o = ((size_t)(n * Ho + ho) * Wo + wo) * C + cc * 8;
      float g[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + o), g);
      const uint2 a = *reinterpret_cast<const uint2*>(am + o);
      const uint8_t* ab = reinterpret_cast<const uint8_t*>(&a);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (ab[j] == (uint8_t)(r * k + s)) acc[j] += g[j];
    }
  }
  reinterpret_cast<uint4*>(dx)[i] = pack8(acc);
}

__global__ __launch_bounds__(NT) void avgpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                         int N, int HW, int C) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - n * C;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += bf2f(x[((size_t)n * HW + p) * C + c]);
  y[i] = f2bf_bits(s / (float)HW);
}

// 8-channel chunk forms (C % 8 == 0): 16-B loads / stores, the same per-channel sums in the same
// order and the same rounding as the scalar kernels
__global__ __launch_bounds__(NT) void avgpool_fwd8_kernel(const uint4* __restrict__ x, uint4* __restrict__ y, int N,
                                                          int HW, int C8) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= N * C8) return;
  const int n = i / C8, c = i - n * C8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, v[8];
  const uint4* p = x + (size_t)n * HW * C8 + c;
#pragma unroll 7
  for (int q = 0; q < HW; ++q) {
    unpack8(p[(size_t)q * C8], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += v[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = s[j] / (float)HW;
  y[i] = pack8(s);
}

__global__ __launch_bounds__(NT) void avgpool_bwd8_kernel(const uint4* __restrict__ dy, uint4* __restrict__ dx, int N,
                                                          int HW, int C8) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= (int64_t)N * HW * C8) return;
  const int c = (int)(i % C8);
  const int n = (int)(i / ((int64_t)HW * C8));
  float v[8];
  unpack8(dy[(size_t)n * C8 + c], v);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = v[j] / (float)HW;
  dx[i] = pack8(v);
}

__global__ __launch_bounds__(NT) void avgpool_bwd_kernel(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx,
                                                         int N, int HW, int C) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= (int64_t)N * HW * C) return;
  const int c = (int)(i % C);
  const int n = (int)(i / ((int64_t)HW * C));
  dx[i] = f2bf_bits(bf2f(dy[(size_t)n * C + c]) / (float)HW);
}

__global__ __launch_bounds__(NT) void softmax_xent_kernel(const float* __restrict__ logits, const int* __restrict__ labels,
                                                          float* __restrict__ loss, float* __restrict__ correct,
                                                          uint16_t* __restrict__ dl, int N, int K) {
  __shared__ float red[NT / 64];
  __shared__ int redi[NT / 64];
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const float* z = logits + (size_t)row * K;
  float mx = -INFINITY;
  int am = 0;
  for (int k = t; k < K; k += NT)
    if (z[k] > mx) { mx = z[k]; am = k; }
  // argmax (first index on ties) and max
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  if (lane == 0) { red[wv] = mx; redi[wv] = am; }
  __syncthreads();
  mx = red[0];
  am = redi[0];
  for (int q = 1; q < NT / 64; ++q)
    if (red[q] > mx || (red[q] == mx && redi[q] < am)) { mx = red[q]; am = redi[q]; }
  __syncthreads();
  float se = 0.f;
  for (int k = t; k < K; k += NT) se += __expf(z[k] - mx);
  se = wave_sum(se);
  if (lane == 0) red[wv] = se;
  __syncthreads();
  se = 0.f;
  for (int q = 0; q < NT / 64; ++q) se += red[q];
  const float lse = mx + __logf(se);
  const int lbl = labels[row];
  if (t == 0) {
    loss[row] = lse - z[lbl];
    correct[row] = (am == lbl) ? 1.f : 0.f;
  }
  const float invN = 1.f / (float)N;
  for (int k = t; k < K; k += NT)
    dl[(size_t)row * K + k] = f2bf_bits((__expf(z[k] - lse) - (k == lbl ? 1.f : 0.f)) * invN);
}

// one thread per 8-channel output chunk (16-B store; Cout % 8 == 0): the stem input [P][3] fp32 ->
// [P][8] bf16 is one pixel per thread
__global__ __launch_bounds__(NT) void pad_channels_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                          int64_t P, int Cin, int Cout) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x, nch = Cout / 8;
  if (i >= P * nch) return;
  const int c0 = (int)(i % nch) * 8;
  const int64_t p = i / nch;
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = c0 + j < Cin ? x[p * Cin + c0 + j] : 0.f;
  reinterpret_cast<uint4*>(y)[i] = pack8(f);
}

// one thread per output pixel pair: 6 contiguous floats in, one 16-B chunk out (same rounding as pad_channels)
__global__ __launch_bounds__(NT) void stem_pack_w2_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                          int64_t pairs) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (i >= pairs) return;
  const float2* p = reinterpret_cast<const float2*>(x + i * 6);
  const float2 a = p[0], b = p[1], c = p[2];
  float f[8] = {a.x, a.y, b.x, b.y, c.x, c.y, 0.f, 0.f};
  reinterpret_cast<uint4*>(y)[i] = pack8(f);
}

inline int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(4096, (n + NT - 1) / NT)); }

void launch_apply(const uint16_t* y, const float* gamma, const float* beta, const float* mean, const float* invstd,
                  const uint16_t* res, int relu, uint16_t* out, int M, int C, const RowSplit& r, hipStream_t st,
                  uint8_t* mb = nullptr, const BnFin* fin = nullptr) {
#define TFD_BN_APPLY(R, U)                                                                                          \
  if (fin)                                                                                                        \
    bn_apply_kernel<R, U, true><<<r.nblk, NT, 0, st>>>(y, gamma, beta, mean, invstd, res, out, M, C, r.tpr, r.rg,  \
                                                       r.rb, mb, *fin);                                           \
  else                                                                                                            \
    bn_apply_kernel<R, U><<<r.nblk, NT, 0, st>>>(y, gamma, beta, mean, invstd, res, out, M, C, r.tpr, r.rg, r.rb, mb);
  if (res && relu) { TFD_BN_APPLY(true, true) }
  else if (res) { TFD_BN_APPLY(true, false) }
  else if (relu) { TFD_BN_APPLY(false, true) }
  else { TFD_BN_APPLY(false, false) }
#undef TFD_BN_APPLY
}

template <int MK>
void launch_bwd_apply(const uint16_t* dout, const uint16_t* out, const uint16_t* y, const float* gamma,
                      const float* beta, const float* mean, const float* invstd, uint16_t* dy, uint16_t* dres,
                      float* dgamma, float* dbeta, int M, int C, const RowSplit& r, hipStream_t st,
                      const uint8_t* mb, const BnFin* fin) {
  if (fin)
    bn_bwd_apply_kernel<MK, true><<<r.nblk, NT, 0, st>>>(dout, out, y, gamma, beta, mean, invstd, dbeta, dgamma, dy, dres,
                                                         M, C, r.tpr, r.rg, r.rb, 1.f / (float)M, mb, *fin);
  else
    bn_bwd_apply_kernel<MK><<<r.nblk, NT, 0, st>>>(dout, out, y, gamma, beta, mean, invstd, dbeta, dgamma, dy, dres, M, C,
                                                   r.tpr, r.rg, r.rb, 1.f / (float)M, mb);
}

// backward: bn_final over the partial rows, then the apply pass; slots (a slot-mode buffer of nrows
// slots from a dgrad epilogue): the apply pass finalizes inline
void backward_apply(const uint16_t* dout, const uint16_t* out, const uint16_t* y, const float* gamma, const float* beta,
                    const float* mean, const float* invstd, int relu, uint16_t* dy, uint16_t* dres, float* dgamma,
                    float* dbeta, int M, int C, const float* partials, int nrows, hipStream_t st,
                    const uint8_t* mask_bits, bool slots) {
  const RowSplit r = row_split(M, C);
  // beta given (no residual in the forward): the relu mask is recomputed from y, `out` is not read;
  // mask_bits given: the forward's relu bits, `out` is not read
  const int mask = !relu ? 0 : (mask_bits ? 3 : (beta ? 2 : 1));
  BnFin f{partials, nrows, 0.f, 0.f, dbeta, dgamma, nullptr, nullptr};
  const BnFin* fin = slots ? &f : nullptr;
  if (!fin)
    bn_final_kernel<<<(C + 31) / 32, FIN_NT, 0, st>>>(1, partials, nrows, M, C, 0.f, 0.f, dbeta, dgamma, nullptr, nullptr);
  if (mask == 0) launch_bwd_apply<0>(dout, out, y, gamma, beta, mean, invstd, dy, dres, dgamma, dbeta, M, C, r, st, mask_bits, fin);
  else if (mask == 1) launch_bwd_apply<1>(dout, out, y, gamma, beta, mean, invstd, dy, dres, dgamma, dbeta, M, C, r, st, mask_bits, fin);
  else if (mask == 2) launch_bwd_apply<2>(dout, out, y, gamma, beta, mean, invstd, dy, dres, dgamma, dbeta, M, C, r, st, mask_bits, fin);
  else launch_bwd_apply<3>(dout, out, y, gamma, beta, mean, invstd, dy, dres, dgamma, dbeta, M, C, r, st, mask_bits, fin);
}

}  // namespace

static int g_bn_slots = kBnSlotsDefault;
int bn_slots() { return g_bn_slots; }
void set_bn_slots(int s) {
  if (s < 0 || s > FIN_MAXS) throw std::runtime_error("set_bn_slots: 0 (row mode) or 1..8 slots");
  g_bn_slots = s;  // read at launch time: every kernel takes the mode as an argument (BnPart, BnFin)
}

int bn_partials_size(int M, int C) {  // the partial pass's rows (row layout in either mode)
  const RowSplit r = row_split(M, C);
  return r.nblk * 2 * C;
}

namespace {
void forward_apply(const uint16_t* y, const float* gamma, const float* beta, const uint16_t* residual, int relu,
                   uint16_t* out, float* mean, float* invstd, float* running_mean, float* running_var, float momentum,
                   float eps, int M, int C, const float* partials, int nrows, hipStream_t st, uint8_t* mask_bits,
                   bool slots) {
  const RowSplit r = row_split(M, C);
  if (slots) {
    const BnFin f{partials, nrows, eps, momentum, mean, invstd, running_mean, running_var};
    launch_apply(y, gamma, beta, mean, invstd, residual, relu, out, M, C, r, st, mask_bits, &f);
    return;
  }
  bn_final_kernel<<<(C + 31) / 32, FIN_NT, 0, st>>>(0, partials, nrows, M, C, eps, momentum, mean, invstd,
                                                running_mean, running_var);
  launch_apply(y, gamma, beta, mean, invstd, residual, relu, out, M, C, r, st, mask_bits);
}
}  // namespace

// partials from conv_fwd_stats: [nrows][2][C] rows (row mode) or zeroed slots filled by atomics (slot mode)
void bn_forward_partials(const uint16_t* y, const float* gamma, const float* beta, const uint16_t* residual, int relu,
                         uint16_t* out, float* mean, float* invstd, float* running_mean, float* running_var,
                         float momentum, float eps, int M, int C, const float* partials, int nrows, hipStream_t st,
                         uint8_t* mask_bits) {
  forward_apply(y, gamma, beta, residual, relu, out, mean, invstd, running_mean, running_var, momentum, eps, M, C,
                partials, nrows, st, mask_bits, bn_slots() > 0);
}

// the partial pass writes one row per block in either mode (its blocks all end together, so slot
// atomics there serialised into a tail: ResNet-50 bn_partial 46 -> 92 us), then bn_final
void bn_forward(const uint16_t* y, const float* gamma, const float* beta, const uint16_t* residual, int relu,
                uint16_t* out, float* mean, float* invstd, float* running_mean, float* running_var, float momentum,
                float eps, int M, int C, float* partials, hipStream_t st, uint8_t* mask_bits) {
  const RowSplit r = row_split(M, C);
  bn_partial_kernel<0, 0><<<r.nblk, NT, 0, st>>>(y, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, M, C, r.tpr,
                                                 r.rg, r.rb, partials, nullptr);
  forward_apply(y, gamma, beta, residual, relu, out, mean, invstd, running_mean, running_var, momentum, eps, M, C,
                partials, r.nblk, st, mask_bits, false);
}

void bn_stats_partials(float* mean, float* invstd, float* running_mean, float* running_var, float momentum, float eps,
                       int M, int C, const float* partials, int nrows, hipStream_t st) {
  bn_final_kernel<<<(C + 31) / 32, FIN_NT, 0, st>>>(0, partials, nrows, M, C, eps, momentum, mean, invstd,
                                                running_mean, running_var);
}

void bn_backward(const uint16_t* dout, const uint16_t* out, const uint16_t* y, const float* gamma, const float* beta,
                 const float* mean, const float* invstd, int relu, uint16_t* dy, uint16_t* dres, float* dgamma,
                 float* dbeta, int M, int C, float* partials, hipStream_t st, const uint8_t* mask_bits) {
  const RowSplit r = row_split(M, C);
  const int mask = !relu ? 0 : (mask_bits ? 3 : (beta ? 2 : 1));
#define TFD_BN_PART(MK)                                                                                       \
  bn_partial_kernel<1, MK><<<r.nblk, NT, 0, st>>>(y, dout, out, mean, invstd, gamma, beta, M, C, r.tpr, r.rg, \
                                                  r.rb, partials, mask_bits);
  if (mask == 0) { TFD_BN_PART(0) }
  else if (mask == 1) { TFD_BN_PART(1) }
  else if (mask == 2) { TFD_BN_PART(2) }
  else { TFD_BN_PART(3) }
#undef TFD_BN_PART
  backward_apply(dout, out, y, gamma, beta, mean, invstd, relu, dy, dres, dgamma, dbeta, M, C, partials, r.nblk, st,
                 mask_bits, false);
}

void bn_backward_partials(const uint16_t* dout, const uint16_t* out, const uint16_t* y, const float* gamma,
                          const float* beta, const float* mean, const float* invstd, int relu, uint16_t* dy,
                          uint16_t* dres, float* dgamma, float* dbeta, int M, int C, const float* partials, int nblk,
                          hipStream_t st, const uint8_t* mask_bits) {
  backward_apply(dout, out, y, gamma, beta, mean, invstd, relu, dy, dres, dgamma, dbeta, M, C, partials, nblk, st,
                 mask_bits, bn_slots() > 0);
}

void bn_infer(const uint16_t* y, const float* gamma, const float* beta, const float* rmean, const float* rvar,
              float eps, int relu, uint16_t* out, int M, int C, hipStream_t st) {
  const int64_t nch = (int64_t)M * C / 8;
  bn_infer_kernel<<<grid_for(nch), NT, 0, st>>>(y, gamma, beta, rmean, rvar, eps, relu, out, nch, C);
}

void maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* argmax, int N, int H, int W, int C, int k, int st, int pad,
                 int Ho, int Wo, hipStream_t s) {
  const int64_t total = (int64_t)N * Ho * Wo * (C / 8);
  maxpool_fwd_kernel<<<(int)((total + NT - 1) / NT), NT, 0, s>>>(x, y, argmax, N, H, W, C, k, st, pad, Ho, Wo);
}

void maxpool_bwd(const uint16_t* dy, const uint8_t* argmax, uint16_t* dx, int N, int H, int W, int C, int k, int st,
                 int pad, int Ho, int Wo, hipStream_t s) {
  if ((k + st - 1) / st <= 2) {  // every window's loads in flight together
    const int grid = std::max(1, std::min(8192, N * H));
    maxpool2_bwd_kernel<<<grid, NT, 0, s>>>(dy, argmax, dx, N, H, W, C, k, st, pad, Ho, Wo);
    return;
  }
  const int64_t total = (int64_t)N * H * W * (C / 8);
  maxpool_bwd_kernel<<<(int)((total + NT - 1) / NT), NT, 0, s>>>(dy, argmax, dx, N, H, W, C, k, st, pad, Ho, Wo);
}

void bn_relu_maxpool(const uint16_t* y, const float* gamma, const float* beta, float* mean, float* invstd,
                     float* running_mean, float* running_var, float momentum, float eps, const float* partials,
                     int nrows, uint16_t* out, uint8_t* argmax, int N, int H, int W, int C, int k, int st, int pad,
                     int Ho, int Wo, hipStream_t s) {
  if (k > POOL_KMAX || C % 8 || C > 2048) throw std::runtime_error("bn_relu_maxpool: k <= 3, C % 8 == 0, C <= 2048");
  const int grid = std::max(1, std::min(2048, N * Ho));  // blocks walk output rows
  if (bn_slots() > 0) {
    const BnFin f{partials, nrows, eps, momentum, mean, invstd, running_mean, running_var};
    bn_relu_maxpool_kernel<true><<<grid, NT, 0, s>>>(y, gamma, beta, mean, invstd, out, argmax, N, H, W, C, k, st, pad,
                                                     Ho, Wo, f);
    return;
  }
  bn_final_kernel<<<(C + 31) / 32, FIN_NT, 0, s>>>(0, partials, nrows, N * H * W, C, eps, momentum, mean, invstd,
                                               running_mean, running_var);
  bn_relu_maxpool_kernel<false><<<grid, NT, 0, s>>>(y, gamma, beta, mean, invstd, out, argmax, N, H, W, C, k, st, pad, Ho,
                                                    Wo, BnFin{});
}

void avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t s) {
  if (C % 8 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(y) % 16 == 0) {
    avgpool_fwd8_kernel<<<(N * (C / 8) + NT - 1) / NT, NT, 0, s>>>(reinterpret_cast<const uint4*>(x),
                                                                   reinterpret_cast<uint4*>(y), N, HW, C / 8);
    return;
  }
  avgpool_fwd_kernel<<<(N * C + NT - 1) / NT, NT, 0, s>>>(x, y, N, HW, C);
}

void avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t s) {
  if (C % 8 == 0 && reinterpret_cast<uintptr_t>(dy) % 16 == 0 && reinterpret_cast<uintptr_t>(dx) % 16 == 0) {
    const int64_t chunks = (int64_t)N * HW * (C / 8);
    avgpool_bwd8_kernel<<<(int)((chunks + NT - 1) / NT), NT, 0, s>>>(reinterpret_cast<const uint4*>(dy),
                                                                     reinterpret_cast<uint4*>(dx), N, HW, C / 8);
    return;
  }
  const int64_t total = (int64_t)N * HW * C;
  avgpool_bwd_kernel<<<(int)((total + NT - 1) / NT), NT, 0, s>>>(dy, dx, N, HW, C);
}

void softmax_xent(const float* logits, const int* labels, float* loss_rows, float* correct, uint16_t* dlogits, int N,
                  int K, hipStream_t s) {
  softmax_xent_kernel<<<N, NT, 0, s>>>(logits, labels, loss_rows, correct, dlogits, N, K);
}

void stem_pack_w2(const float* x, uint16_t* y, int64_t pairs, hipStream_t s) {
  stem_pack_w2_kernel<<<(int)((pairs + NT - 1) / NT), NT, 0, s>>>(x, y, pairs);
}

void pad_channels(const float* x, uint16_t* y, int P, int Cin, int Cout, hipStream_t s) {
  const int64_t total = (int64_t)P * (Cout / 8);
  pad_channels_kernel<<<(int)((total + NT - 1) / NT), NT, 0, s>>>(x, y, P, Cin, Cout);
}

}  // namespace tfd
