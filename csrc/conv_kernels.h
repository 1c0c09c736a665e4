// Host API of the generic NHWC convolution / dense / normalisation kernel library
// (csrc/kernels/conv_nhwc.hip, csrc/kernels/norm.hip) used by the ResNet-style models.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <algorithm>

namespace tfd {

struct ConvShape {
  int N, H, W, C;   // input NHWC
  int K, R, S;      // output channels, filter rows/cols (HWIO filter [R][S][C][K])
  int stride, pad;  // symmetric zero padding
  // width-only overrides (forward and weight gradient only; the width-paired stem, conv2d_*_w2):
  // stride_w 0 = stride, pad_w -1 = pad (left pad; the right edge is the input's end), wo_out 0 = derived
  int stride_w = 0, pad_w = -1, wo_out = 0;
  int sw() const { return stride_w ? stride_w : stride; }
  int pw() const { return pad_w >= 0 ? pad_w : pad; }
  bool w_override() const { return stride_w != 0 || pad_w >= 0 || wo_out != 0; }
  int Ho() const { return (H + 2 * pad - R) / stride + 1; }
  int Wo() const { return wo_out ? wo_out : (W + 2 * pw() - S) / sw() + 1; }
};

// Forward BN fold: the conv input is relu(bn(x)) of the producing layer (training-mode statistics
// mean / invstd, affine gamma / beta, all fp32 [C]), applied by the operand loader while it stages x --
// the normalised activation is never materialised. C <= kBnReluMaxC. nullptr: x is the input as is.
constexpr int kBnReluMaxC = 512;
struct BnReluIn {
  const float *mean, *invstd, *gamma, *beta;
};
void conv_fwd(const ConvShape& c, const uint16_t* x, const uint16_t* w, uint16_t* y, hipStream_t st,
              const BnReluIn* act = nullptr);
// conv forward that also emits the batch-norm statistics of its (bf16) output: part is fp32
// [conv_fwd_stats_rows(c, folded)][2][K] (per-row-block sums and sums of squares), consumed by
// bn_forward_partials / bn_stats_partials -- the forward BN then never re-reads the conv output for
// its statistics
int conv_fwd_stats_rows(const ConvShape& c, bool folded = false);
void conv_fwd_stats(const ConvShape& c, const uint16_t* x, const uint16_t* w, uint16_t* y, float* part,
                    hipStream_t st, const BnReluIn* act = nullptr);
// add (optional, must not alias dx): dx = add + dgrad in the epilogue -- the residual-join sum of
// two gradient paths without a separate add kernel
// add_bits (stride 1, with add): add is a residual BN's dout and add_bits its forward relu bits
// ([M][C/8]): the epilogue adds dout masked by the bits -- the dres that BN's backward then need not
// write
// add_sub2 (stride 1, with add): add is [N][ceil(H/2)][ceil(W/2)][C], added at the even (h, w)
// pixels only -- a downsample block's 1x1 stride-2 shortcut dgrad computed on its own grid
void conv_dgrad(const ConvShape& c, const uint16_t* dy, const uint16_t* w, uint16_t* dx, hipStream_t st,
                const uint16_t* add = nullptr, const uint8_t* add_bits = nullptr, bool add_sub2 = false);
// dgrad whose epilogue also emits the backward statistics partials of the batch norm whose output
// was this conv's input (its dout is the dgrad output): part fp32 [conv_dgrad_bn_rows(c)][2][C] of
// per-row-block sums of d and d * (y - mean) * invstd, d = dout through the BN's relu mask -- what
// bn_backward's partial pass would read back; bn_backward_partials consumes them. mode: 0 no relu,
// 2 mask recomputed from y (gamma, beta: the forward's constants), 3 relu bits. Stride 1 only.
struct BnBwdStats {
  const uint16_t* y;
  const float *mean, *invstd, *gamma, *beta;
  const uint8_t* bits;
  int mode;
};
bool conv_dgrad_bn_supported(const ConvShape& c);
int conv_dgrad_bn_rows(const ConvShape& c);
void conv_dgrad_bn(const ConvShape& c, const uint16_t* dy, const uint16_t* w, uint16_t* dx, hipStream_t st,
                   const uint16_t* add, const BnBwdStats& b, float* part, const uint8_t* add_bits = nullptr,
                   bool add_sub2 = false);
// dw: fp32 [R*S*C][K]; overwritten (zeroed first when split)
// zeroed: dw is known to be zero already (the model zeroes its flat gradient buffer once per
// step), so split-K needs no per-layer memset
// act: x is the pre-BN input of a folded conv (see BnReluIn), the X operand is rebuilt while staging
void conv_wgrad(const ConvShape& c, const uint16_t* x, const uint16_t* dy, float* dw, int splits, hipStream_t st,
                bool zeroed = false, const BnReluIn* act = nullptr);
int conv_wgrad_splits(const ConvShape& c, bool folded = false);

void linear_fwd(const uint16_t* x, const uint16_t* w, const float* bias, float* y, int M, int Kin, int N,
                hipStream_t st);
void linear_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int M, int Kin, int N, hipStream_t st);
void linear_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int M, int Kin, int N, hipStream_t st);
// GEMM core of the conv ops: 0 = the 128-row core, 1 = the 256-row core where its tiles fill the
// chip (default; env TFD_G256 at the first call), 2 = the 256-row core wherever it applies. Returns the
// previous mode; -1 only queries. (A/B switch for tests and the per-layer probe.)
int conv_gemm_core(int mode);
// 3x3 stride-1 convs on LDS halo tiles: 0 off, 1 (default) maps >= 14 wide, 2 every eligible shape;
// returns the previous mode (-1: query only)
int conv_halo_mode(int mode);
// how a split-K weight gradient clears its own accumulator (zeroed = false): 0 a fill kernel (default),
// 1 hipMemsetAsync (tools/debug/memset_capture_probe.py: the diagnosis of the round-5 replay fault);
// -1 queries. Returns the previous mode.
int conv_wgrad_clear_mode(int mode);
// C[M][N] bf16 = A[M][K] . Bt[N][K]^T on the 256 x 256 core (csrc/kernels/gemm256.hip)
void gemm_nt_bf16(const uint16_t* a, const uint16_t* bt, uint16_t* c, int M, int N, int K, hipStream_t st);

// ---- batch norm (training mode, per-channel over the M = N*H*W rows of a [M][C] bf16 tensor) ----
// Statistics partials ([rows][2][C] fp32: per-channel sums of a and b over row blocks -- y and y^2
// forward, d and d*xhat backward). Slot mode, bn_slots() = S > 0: every producer (the conv
// epilogues, the partial pass) ADDS its row block's column sums into slot (row block % S) with fp32
// atomics, so a buffer has S rows and MUST BE ZEROED before its producer runs (the ResNet model
// zeroes one arena per forward); the apply passes then finalize the statistics inline from the S
// slots -- no bn_final launch between producer and apply (106 per ResNet-50 step). S only spreads
// same-address atomics. The fp32 sums' order is then not fixed (like the split-K weight gradients).
// Row mode, S = 0: one row per producer block (fixed order, bit-reproducible) reduced by
// bn_final_kernel -- what the bit-exact race tests and --deterministic runs select (set_bn_slots(0)).
// The mode is read at launch and passed to every kernel (BnPart / BnFin arguments), so a captured
// graph keeps the mode it was built with. S = 4 by default (S = 1 15.4, 2 13.37, 4 and 8 13.22,
// 16 13.70 ms/step for ResNet-50 b128, profiles/resnet50_bn_slots_ab_r4.log).
constexpr int kBnSlotsDefault = 4;
int bn_slots();
void set_bn_slots(int s);
// partials: fp32 workspace of bn_partials_size(M, C) floats for the partial pass (one row per block
// in either mode; only producer epilogues use the slots).
int bn_partials_size(int M, int C);
// mean/invstd [C]; running stats updated with `momentum` (TF decay semantics: r = r*m + x*(1-m)).
void bn_forward(const uint16_t* y, const float* gamma, const float* beta, const uint16_t* residual, int relu,
                uint16_t* out, float* mean, float* invstd, float* running_mean, float* running_var, float momentum,
                float eps, int M, int C, float* partials, hipStream_t st, uint8_t* mask_bits = nullptr);
// mask_bits (optional, relu only): [M][C/8] bytes, bit j of byte (m, c/8) = out[m][c/8*8 + j] > 0;
// the backward takes them instead of `out` (bn_backward mask_bits)
// same, with the statistics partials already produced by conv_fwd_stats ([nblk][2][C])
void bn_forward_partials(const uint16_t* y, const float* gamma, const float* beta, const uint16_t* residual, int relu,
                         uint16_t* out, float* mean, float* invstd, float* running_mean, float* running_var,
                         float momentum, float eps, int M, int C, const float* partials, int nblk, hipStream_t st,
                         uint8_t* mask_bits = nullptr);
// statistics only (mean / invstd + running stats) from conv_fwd_stats partials: the BN of a folded
// conv input, whose normalisation is applied by the consumer's loader (BnReluIn)
void bn_stats_partials(float* mean, float* invstd, float* running_mean, float* running_var, float momentum, float eps,
                       int M, int C, const float* partials, int nrows, hipStream_t st);
// dout -> dy (through relu/bn), writes dgamma/dbeta (fp32, overwritten) and, when dres != null, the
// gradient of the residual input (== gradient after the relu mask).
// beta != nullptr (only valid when the forward had no residual): the relu mask is recomputed from y
// with the forward's constants instead of reading `out`.
void bn_backward(const uint16_t* dout, const uint16_t* out, const uint16_t* y, const float* gamma, const float* beta,
                 const float* mean, const float* invstd, int relu, uint16_t* dy, uint16_t* dres, float* dgamma,
                 float* dbeta, int M, int C, float* partials, hipStream_t st, const uint8_t* mask_bits = nullptr);
// same, with the partials already summed by the producing dgrad's epilogue (conv_dgrad_bn, [nblk][2][C])
void bn_backward_partials(const uint16_t* dout, const uint16_t* out, const uint16_t* y, const float* gamma,
                          const float* beta, const float* mean, const float* invstd, int relu, uint16_t* dy,
                          uint16_t* dres, float* dgamma, float* dbeta, int M, int C, const float* partials, int nblk,
                          hipStream_t st, const uint8_t* mask_bits = nullptr);
// inference-mode BN (running statistics), optional relu
void bn_infer(const uint16_t* y, const float* gamma, const float* beta, const float* rmean, const float* rvar,
              float eps, int relu, uint16_t* out, int M, int C, hipStream_t st);

// the stem's training-mode relu(bn(y)) + max pool in one pass (the BN output is never written):
// statistics from conv_fwd_stats partials (finalized inline in slot mode), mean / invstd / running
// stats as bn_forward_partials; out / argmax exactly those of bn_forward_partials + maxpool_fwd
void bn_relu_maxpool(const uint16_t* y, const float* gamma, const float* beta, float* mean, float* invstd,
                     float* running_mean, float* running_var, float momentum, float eps, const float* partials,
                     int nrows, uint16_t* out, uint8_t* argmax, int N, int H, int W, int C, int k, int st, int pad,
                     int Ho, int Wo, hipStream_t s);

// ---- pooling / head ----
void maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* argmax, int N, int H, int W, int C, int k, int st, int pad,
                 int Ho, int Wo, hipStream_t s);
void maxpool_bwd(const uint16_t* dy, const uint8_t* argmax, uint16_t* dx, int N, int H, int W, int C, int k, int st,
                 int pad, int Ho, int Wo, hipStream_t s);
void avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t s);   // global average
void avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t s);
// softmax cross-entropy over fp32 logits [N][K], int labels: loss_rows [N], dlogits bf16 [N][K] (mean
// over N folded in), correct [N]
void softmax_xent(const float* logits, const int* labels, float* loss_rows, float* correct, uint16_t* dlogits, int N,
                  int K, hipStream_t s);
void pad_channels(const float* x, uint16_t* y, int P, int Cin, int Cout, hipStream_t s);
// fp32 NHWC [N][H][W][3] -> bf16 [N][H][W/2][8]: each 8-channel pixel holds two horizontally adjacent
// input pixels' 3 channels, then 2 zeros (the width-paired stem input)
void stem_pack_w2(const float* x, uint16_t* y, int64_t pairs, hipStream_t s);  // fp32 NHWC -> bf16, zero-pad C

}  // namespace tfd
