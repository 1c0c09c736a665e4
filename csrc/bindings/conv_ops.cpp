// Torch op bindings (torch.ops.tfd.*) of the NHWC conv / dense / batch-norm / pooling kernel library
// (csrc/conv_kernels.h). All ops run on the caller's current HIP stream (graph-capturable); shapes
// are checked on the host before any launch (the kernels assume C % 8 == 0 etc.).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <tuple>
#include <vector>

#include "../conv_kernels.h"

namespace tfd {
namespace {

hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }
uint16_t* bp(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
float* fp(const at::Tensor& t) { return t.defined() ? reinterpret_cast<float*>(t.data_ptr()) : nullptr; }

void check_bf16(const at::Tensor& t, const char* name, int dim) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), name,
              ": contiguous bf16 GPU tensor required");
  TORCH_CHECK(dim < 0 || t.dim() == dim, name, ": expected ", dim, " dims");
}
void check_f32(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name, ": contiguous fp32 GPU tensor");
}

ConvShape shape_of(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad) {
  ConvShape c;
  c.N = (int)x.size(0); c.H = (int)x.size(1); c.W = (int)x.size(2); c.C = (int)x.size(3);
  c.R = (int)w.size(0); c.S = (int)w.size(1); c.K = (int)w.size(3);
  c.stride = (int)stride; c.pad = (int)pad;
  TORCH_CHECK(w.size(2) == c.C, "conv: filter C ", w.size(2), " != input C ", c.C);
  TORCH_CHECK(c.C % 8 == 0 && c.K % 8 == 0, "conv: C and K must be multiples of 8 (pad the input channels)");
  TORCH_CHECK(c.Ho() > 0 && c.Wo() > 0 && stride >= 1 && pad >= 0, "conv: bad geometry");
  // the GEMM loaders address operands through 32-bit buffer descriptors (byte ranges < 2 GiB)
  TORCH_CHECK((int64_t)c.N * c.H * c.W * c.C < (1ll << 30) && (int64_t)c.N * c.Ho() * c.Wo() * c.K < (1ll << 30),
              "conv: tensor too large for 32-bit buffer addressing");
  return c;
}

// Folded BN input (BnReluIn): mean, invstd, gamma, beta all given (fp32 [C]) or none
struct Act {
  BnReluIn in{};
  bool on = false;
  const BnReluIn* ptr() const { return on ? &in : nullptr; }
};
Act act_of(const c10::optional<at::Tensor>& mean, const c10::optional<at::Tensor>& invstd,
           const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta, int C) {
  Act a;
  const int n = (int)mean.has_value() + (int)invstd.has_value() + (int)gamma.has_value() + (int)beta.has_value();
  if (n == 0) return a;
  TORCH_CHECK(n == 4, "conv: a folded BN input needs mean, invstd, gamma and beta");
  for (const auto* t : {&*mean, &*invstd, &*gamma, &*beta}) {
    check_f32(*t, "bn");
    TORCH_CHECK(t->numel() == C, "conv: folded BN vectors must have C elements");
  }
  TORCH_CHECK(C <= kBnReluMaxC, "conv: folded BN input with C > ", kBnReluMaxC);
  a.in = BnReluIn{fp(*mean), fp(*invstd), fp(*gamma), fp(*beta)};
  a.on = true;
  return a;
}

// A statistics-partials buffer [rows][2][C]: the caller's (slot mode: zeroed by the caller, the
// ResNet model's per-forward arena) or a fresh one (zero-filled in slot mode).
at::Tensor part_buffer(const c10::optional<at::Tensor>& given, int64_t rows, int64_t C, const at::TensorOptions& o,
                       const char* what) {
  if (given.has_value()) {
    TORCH_CHECK(given->is_cuda() && given->scalar_type() == at::kFloat && given->is_contiguous() && given->dim() == 3 &&
                    given->size(0) == rows && given->size(1) == 2 && given->size(2) == C &&
                    reinterpret_cast<uintptr_t>(given->data_ptr()) % 16 == 0,
                what, ": partials buffer must be contiguous 16-B aligned fp32 [", rows, ", 2, ", C, "]");
    return *given;
  }
  auto f = o.dtype(at::kFloat);
  return bn_slots() > 0 ? at::zeros({rows, 2, C}, f) : at::empty({rows, 2, C}, f);
}

at::Tensor conv2d_fwd(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad,
                      const c10::optional<at::Tensor>& mean, const c10::optional<at::Tensor>& invstd,
                      const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta) {
  check_bf16(x, "x", 4);
  check_bf16(w, "w", 4);
  const ConvShape c = shape_of(x, w, stride, pad);
  const Act a = act_of(mean, invstd, gamma, beta, c.C);
  auto y = at::empty({c.N, c.Ho(), c.Wo(), c.K}, x.options());
  conv_fwd(c, bp(x), bp(w), bp(y), cur(), a.ptr());
  return y;
}

std::tuple<at::Tensor, at::Tensor> conv2d_fwd_stats(const at::Tensor& x, const at::Tensor& w, int64_t stride,
                                                    int64_t pad, const c10::optional<at::Tensor>& mean,
                                                    const c10::optional<at::Tensor>& invstd,
                                                    const c10::optional<at::Tensor>& gamma,
                                                    const c10::optional<at::Tensor>& beta,
                                                    const c10::optional<at::Tensor>& part_out) {
  check_bf16(x, "x", 4);
  check_bf16(w, "w", 4);
  const ConvShape c = shape_of(x, w, stride, pad);
  const Act a = act_of(mean, invstd, gamma, beta, c.C);
  auto y = at::empty({c.N, c.Ho(), c.Wo(), c.K}, x.options());
  auto part = part_buffer(part_out, conv_fwd_stats_rows(c, a.on), c.K, x.options(), "conv2d_fwd_stats");
  conv_fwd_stats(c, bp(x), bp(w), bp(y), fp(part), cur(), a.ptr());
  return {y, part};
}

// acc_bits: acc is a residual BN's dout, the add is dout masked by that BN's forward relu bits
const uint8_t* acc_bits_of(const c10::optional<at::Tensor>& acc_bits, const c10::optional<at::Tensor>& acc,
                           at::IntArrayRef xshape) {
  if (!acc_bits.has_value()) return nullptr;
  TORCH_CHECK(acc.has_value(), "dgrad: acc_bits needs acc");
  const int64_t C = xshape.back(), M = acc->numel() / C;
  TORCH_CHECK(acc_bits->is_cuda() && acc_bits->scalar_type() == at::kByte && acc_bits->is_contiguous() &&
                  acc_bits->numel() == M * (C / 8), "dgrad: acc_bits must be uint8 [M, C/8] relu bits");
  return acc_bits->data_ptr<uint8_t>();
}

// acc_sub2: acc is [N, ceil(H/2), ceil(W/2), C], added at the even pixels (AddSrc)
void check_acc(const at::Tensor& acc, at::IntArrayRef xshape, bool sub2, const char* what) {
  check_bf16(acc, "acc", 4);
  if (sub2) {
    const std::vector<int64_t> s2{xshape[0], (xshape[1] + 1) / 2, (xshape[2] + 1) / 2, xshape[3]};
    TORCH_CHECK(acc.sizes() == at::IntArrayRef(s2), what, ": a stride-2 acc must be [N, ceil(H/2), ceil(W/2), C]");
  } else {
    TORCH_CHECK(acc.sizes() == xshape, what, ": acc shape must equal xshape");
  }
}

at::Tensor conv2d_dgrad(const at::Tensor& dy, const at::Tensor& w, at::IntArrayRef xshape, int64_t stride, int64_t pad,
                        const c10::optional<at::Tensor>& acc, const c10::optional<at::Tensor>& acc_bits, bool acc_sub2) {
  check_bf16(dy, "dy", 4);
  check_bf16(w, "w", 4);
  TORCH_CHECK(xshape.size() == 4, "xshape [N,H,W,C]");
  auto x = at::empty(xshape, dy.options());
  TORCH_CHECK(!acc_sub2 || acc.has_value(), "dgrad: acc_sub2 needs acc");
  if (acc.has_value()) check_acc(*acc, xshape, acc_sub2, "dgrad");  // dx = acc + dgrad
  const ConvShape c = shape_of(x, w, stride, pad);
  TORCH_CHECK(dy.size(1) == c.Ho() && dy.size(2) == c.Wo() && dy.size(3) == c.K, "dgrad: dy shape mismatch");
  conv_dgrad(c, bp(dy), bp(w), bp(x), cur(), acc.has_value() ? bp(*acc) : nullptr, acc_bits_of(acc_bits, acc, xshape),
             acc_sub2);
  return x;
}

// dgrad + the BN-backward statistics partials of its output (conv_dgrad_bn): the conv's input was
// the output of a batch norm (y, mean, invstd, gamma; beta for a residual-free relu BN, whose mask
// is recomputed from y; mask = the forward's relu bits for a residual BN; neither: no relu)
std::tuple<at::Tensor, at::Tensor> conv2d_dgrad_bn(const at::Tensor& dy, const at::Tensor& w, at::IntArrayRef xshape,
                                                   int64_t stride, int64_t pad, const c10::optional<at::Tensor>& acc,
                                                   const at::Tensor& y, const at::Tensor& mean, const at::Tensor& invstd,
                                                   const at::Tensor& gamma, const c10::optional<at::Tensor>& beta,
                                                   const c10::optional<at::Tensor>& mask, bool relu,
                                                   const c10::optional<at::Tensor>& acc_bits,
                                                   const c10::optional<at::Tensor>& part_out, bool acc_sub2) {
  check_bf16(dy, "dy", 4);
  check_bf16(w, "w", 4);
  check_bf16(y, "y", 4);
  TORCH_CHECK(xshape.size() == 4 && y.sizes() == xshape, "dgrad_bn: y must have the conv input's shape");
  auto x = at::empty(xshape, dy.options());
  TORCH_CHECK(!acc_sub2 || acc.has_value(), "dgrad_bn: acc_sub2 needs acc");
  if (acc.has_value()) check_acc(*acc, xshape, acc_sub2, "dgrad_bn");
  const ConvShape c = shape_of(x, w, stride, pad);
  TORCH_CHECK(dy.size(1) == c.Ho() && dy.size(2) == c.Wo() && dy.size(3) == c.K, "dgrad_bn: dy shape mismatch");
  TORCH_CHECK(conv_dgrad_bn_supported(c), "dgrad_bn: unsupported conv (C % 8, or a strided dgrad with tap-less phases)");
  TORCH_CHECK(y.numel() < (1ll << 30), "dgrad_bn: < 2^30 elements (buffer addressing)");
  check_f32(mean, "mean");
  check_f32(invstd, "invstd");
  check_f32(gamma, "gamma");
  const int C = (int)c.C, M = (int)(y.numel() / C);
  BnBwdStats b{bp(y), fp(mean), fp(invstd), fp(gamma), nullptr, nullptr, 0};
  if (relu) {
    if (mask.has_value()) {
      TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                      mask->numel() == (int64_t)M * (C / 8), "dgrad_bn: mask must be the forward's uint8 [M, C/8] relu bits");
      b.bits = mask->data_ptr<uint8_t>();
      b.mode = 3;
    } else {
      TORCH_CHECK(beta.has_value(), "dgrad_bn: a relu BN needs beta (mask from y) or its relu bits");
      check_f32(*beta, "beta");
      b.beta = fp(*beta);
      b.mode = 2;
    }
  }
  auto part = part_buffer(part_out, conv_dgrad_bn_rows(c), C, dy.options(), "conv2d_dgrad_bn");
  conv_dgrad_bn(c, bp(dy), bp(w), bp(x), cur(), acc.has_value() ? bp(*acc) : nullptr, b, fp(part),
                acc_sub2 ? nullptr : acc_bits_of(acc_bits, acc, xshape), acc_sub2);
  return {x, part};
}

void conv2d_wgrad(const at::Tensor& x, const at::Tensor& dy, at::Tensor dw, int64_t stride, int64_t pad, bool zeroed,
                  const c10::optional<at::Tensor>& mean, const c10::optional<at::Tensor>& invstd,
                  const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta) {
  check_bf16(x, "x", 4);
  check_bf16(dy, "dy", 4);
  check_f32(dw, "dw");
  TORCH_CHECK(dw.dim() == 4, "dw [R,S,C,K]");
  auto wfake = at::empty({dw.size(0), dw.size(1), dw.size(2), dw.size(3)}, x.options().device(at::kCPU));
  const ConvShape c = shape_of(x, wfake, stride, pad);
  TORCH_CHECK(dy.size(0) == c.N && dy.size(1) == c.Ho() && dy.size(2) == c.Wo() && dy.size(3) == c.K,
              "wgrad: dy shape mismatch");
  const Act a = act_of(mean, invstd, gamma, beta, c.C);
  conv_wgrad(c, bp(x), bp(dy), fp(dw), conv_wgrad_splits(c, a.on), cur(), zeroed, a.ptr());
}

at::Tensor gemm_nt_op(const at::Tensor& a, const at::Tensor& bt) {
  check_bf16(a, "a", 2);
  check_bf16(bt, "bt", 2);
  TORCH_CHECK(a.size(1) == bt.size(1) && a.size(1) % 8 == 0 && bt.size(0) % 8 == 0, "gemm_nt: shapes / multiples of 8");
  auto c = at::empty({a.size(0), bt.size(0)}, a.options());
  gemm_nt_bf16(bp(a), bp(bt), bp(c), (int)a.size(0), (int)bt.size(0), (int)a.size(1), cur());
  return c;
}

at::Tensor linear_fwd_op(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias) {
  check_bf16(x, "x", 2);
  check_bf16(w, "w", 2);
  TORCH_CHECK(x.size(1) == w.size(0) && x.size(1) % 8 == 0 && w.size(1) % 8 == 0, "linear: shapes / multiples of 8");
  if (bias) check_f32(*bias, "bias");
  auto y = at::empty({x.size(0), w.size(1)}, x.options().dtype(at::kFloat));
  linear_fwd(bp(x), bp(w), bias ? fp(*bias) : nullptr, fp(y), (int)x.size(0), (int)x.size(1), (int)w.size(1), cur());
  return y;
}

at::Tensor linear_dgrad_op(const at::Tensor& dy, const at::Tensor& w) {
  check_bf16(dy, "dy", 2);
  check_bf16(w, "w", 2);
  TORCH_CHECK(dy.size(1) == w.size(1), "linear_dgrad: shapes");
  auto dx = at::empty({dy.size(0), w.size(0)}, dy.options());
  linear_dgrad(bp(dy), bp(w), bp(dx), (int)dy.size(0), (int)w.size(0), (int)w.size(1), cur());
  return dx;
}

void linear_wgrad_op(const at::Tensor& x, const at::Tensor& dy, at::Tensor dw) {
  check_bf16(x, "x", 2);
  check_bf16(dy, "dy", 2);
  check_f32(dw, "dw");
  TORCH_CHECK(dw.size(0) == x.size(1) && dw.size(1) == dy.size(1) && x.size(0) == dy.size(0), "linear_wgrad: shapes");
  linear_wgrad(bp(x), bp(dy), fp(dw), (int)x.size(0), (int)x.size(1), (int)dy.size(1), cur());
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> bn_fwd(const at::Tensor& y, const at::Tensor& gamma,
                                                      const at::Tensor& beta, const c10::optional<at::Tensor>& res,
                                                      bool relu, at::Tensor running_mean, at::Tensor running_var,
                                                      double momentum, double eps,
                                                      const c10::optional<at::Tensor>& partials,
                                                      const c10::optional<at::Tensor>& mask) {
  check_bf16(y, "y", -1);
  const int C = (int)y.size(-1);
  const int M = (int)(y.numel() / C);
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn: C must be a multiple of 8 and <= 2048");
  TORCH_CHECK(y.numel() < (1ll << 30), "bn: tensor too large for 32-bit buffer addressing");
  check_f32(gamma, "gamma");
  check_f32(beta, "beta");
  if (res) {
    check_bf16(*res, "residual", -1);
    TORCH_CHECK(res->numel() == y.numel(), "bn: residual shape");
  }
  auto out = at::empty_like(y);
  auto f = y.options().dtype(at::kFloat);
  auto mean = at::empty({C}, f), invstd = at::empty({C}, f);
  float* rm = running_mean.defined() && running_mean.numel() ? fp(running_mean) : nullptr;
  float* rv = running_var.defined() && running_var.numel() ? fp(running_var) : nullptr;
  uint8_t* mb = nullptr;
  if (mask.has_value()) {  // relu bits for the backward ([M][C/8] uint8)
    TORCH_CHECK(relu && mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() == (int64_t)M * (C / 8), "bn: mask must be contiguous uint8 [M, C/8] (relu only)");
    mb = mask->data_ptr<uint8_t>();
  }
  if (partials.has_value()) {  // statistics already summed by the producing conv (conv2d_fwd_stats)
    check_f32(*partials, "partials");
    TORCH_CHECK(partials->dim() == 3 && partials->size(1) == 2 && partials->size(2) == C, "bn: partials [nblk,2,C]");
    bn_forward_partials(bp(y), fp(gamma), fp(beta), res ? bp(*res) : nullptr, relu ? 1 : 0, bp(out), fp(mean),
                        fp(invstd), rm, rv, (float)momentum, (float)eps, M, C, fp(*partials),
                        (int)partials->size(0), cur(), mb);
    return {out, mean, invstd};
  }
  auto part = at::empty({bn_partials_size(M, C)}, f);  // the partial pass's rows
  bn_forward(bp(y), fp(gamma), fp(beta), res ? bp(*res) : nullptr, relu ? 1 : 0, bp(out), fp(mean), fp(invstd), rm, rv,
             (float)momentum, (float)eps, M, C, fp(part), cur(), mb);
  return {out, mean, invstd};
}

// training-mode statistics only (the BN of a folded conv input: its consumer applies it while staging)
std::tuple<at::Tensor, at::Tensor> bn_stats(const at::Tensor& y, const at::Tensor& partials, at::Tensor running_mean,
                                            at::Tensor running_var, double momentum, double eps) {
  check_bf16(y, "y", -1);
  check_f32(partials, "partials");
  const int C = (int)y.size(-1);
  TORCH_CHECK(partials.dim() == 3 && partials.size(1) == 2 && partials.size(2) == C, "bn_stats: partials [nblk,2,C]");
  auto f = y.options().dtype(at::kFloat);
  auto mean = at::empty({C}, f), invstd = at::empty({C}, f);
  float* rm = running_mean.defined() && running_mean.numel() ? fp(running_mean) : nullptr;
  float* rv = running_var.defined() && running_var.numel() ? fp(running_var) : nullptr;
  bn_stats_partials(fp(mean), fp(invstd), rm, rv, (float)momentum, (float)eps, (int)(y.numel() / C), C, fp(partials),
                    (int)partials.size(0), cur());
  return {mean, invstd};
}

std::tuple<at::Tensor, at::Tensor> bn_bwd(const at::Tensor& dout, const at::Tensor& out, const at::Tensor& y,
                                          const at::Tensor& gamma, const at::Tensor& mean, const at::Tensor& invstd,
                                          bool relu, bool want_dres, at::Tensor dgamma, at::Tensor dbeta,
                                          const c10::optional<at::Tensor>& beta, const c10::optional<at::Tensor>& mask,
                                          const c10::optional<at::Tensor>& partials) {
  check_bf16(dout, "dout", -1);
  check_bf16(out, "out", -1);
  check_bf16(y, "y", -1);
  check_f32(dgamma, "dgamma");
  check_f32(dbeta, "dbeta");
  const int C = (int)y.size(-1);
  const int M = (int)(y.numel() / C);
  TORCH_CHECK(y.numel() < (1ll << 30) && C % 8 == 0, "bn_bwd: C % 8 and < 2^30 elements (buffer addressing)");
  auto dy = at::empty_like(y);
  at::Tensor dres = want_dres ? at::empty_like(y) : at::Tensor();
  if (beta) check_f32(*beta, "beta");
  const uint8_t* mb = nullptr;
  if (mask.has_value()) {
    TORCH_CHECK(relu && mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() == (int64_t)M * (C / 8), "bn_bwd: mask must be the forward's uint8 [M, C/8] relu bits");
    mb = mask->data_ptr<uint8_t>();
  }
  if (partials.has_value()) {  // statistics partials from the producing dgrad (conv2d_dgrad_bn)
    check_f32(*partials, "partials");
    TORCH_CHECK(partials->dim() == 3 && partials->size(1) == 2 && partials->size(2) == C, "bn_bwd: partials [nblk,2,C]");
    bn_backward_partials(bp(dout), bp(out), bp(y), fp(gamma), beta ? fp(*beta) : nullptr, fp(mean), fp(invstd),
                         relu ? 1 : 0, bp(dy), want_dres ? bp(dres) : nullptr, fp(dgamma), fp(dbeta), M, C,
                         fp(*partials), (int)partials->size(0), cur(), mb);
    return {dy, dres};
  }
  auto part = at::empty({bn_partials_size(M, C)}, y.options().dtype(at::kFloat));
  bn_backward(bp(dout), bp(out), bp(y), fp(gamma), beta ? fp(*beta) : nullptr, fp(mean), fp(invstd), relu ? 1 : 0,
              bp(dy), want_dres ? bp(dres) : nullptr, fp(dgamma), fp(dbeta), M, C, fp(part), cur(), mb);
  return {dy, dres};
}

at::Tensor bn_infer_op(const at::Tensor& y, const at::Tensor& gamma, const at::Tensor& beta, const at::Tensor& rm,
                       const at::Tensor& rv, double eps, bool relu) {
  check_bf16(y, "y", -1);
  const int C = (int)y.size(-1);
  auto out = at::empty_like(y);
  bn_infer(bp(y), fp(gamma), fp(beta), fp(rm), fp(rv), (float)eps, relu ? 1 : 0, bp(out), (int)(y.numel() / C), C,
           cur());
  return out;
}

std::tuple<at::Tensor, at::Tensor> maxpool2d_fwd(const at::Tensor& x, int64_t k, int64_t st, int64_t pad) {
  check_bf16(x, "x", 4);
  const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), C = (int)x.size(3);
  TORCH_CHECK(C % 8 == 0 && k <= 15, "maxpool: C % 8, k <= 15");
  const int Ho = (H + 2 * (int)pad - (int)k) / (int)st + 1, Wo = (W + 2 * (int)pad - (int)k) / (int)st + 1;
  auto y = at::empty({N, Ho, Wo, C}, x.options());
  auto am = at::empty({N, Ho, Wo, C}, x.options().dtype(at::kByte));
  maxpool_fwd(bp(x), bp(y), am.data_ptr<uint8_t>(), N, H, W, C, (int)k, (int)st, (int)pad, Ho, Wo, cur());
  return {y, am};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_relu_maxpool_op(
    const at::Tensor& y, const at::Tensor& gamma, const at::Tensor& beta, at::Tensor running_mean, at::Tensor running_var,
    double momentum, double eps, const at::Tensor& partials, int64_t k, int64_t st, int64_t pad) {
  check_bf16(y, "y", 4);
  check_f32(gamma, "gamma");
  check_f32(beta, "beta");
  check_f32(partials, "partials");
  const int N = (int)y.size(0), H = (int)y.size(1), W = (int)y.size(2), C = (int)y.size(3);
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && k <= 3 && y.numel() < (1ll << 30), "bn_relu_maxpool: C % 8, C <= 2048, k <= 3");
  TORCH_CHECK(partials.dim() == 3 && partials.size(1) == 2 && partials.size(2) == C, "bn_relu_maxpool: partials [rows,2,C]");
  const int Ho = (H + 2 * (int)pad - (int)k) / (int)st + 1, Wo = (W + 2 * (int)pad - (int)k) / (int)st + 1;
  auto out = at::empty({N, Ho, Wo, C}, y.options());
  auto am = at::empty({N, Ho, Wo, C}, y.options().dtype(at::kByte));
  auto f = y.options().dtype(at::kFloat);
  auto mean = at::empty({C}, f), invstd = at::empty({C}, f);
  float* rm = running_mean.defined() && running_mean.numel() ? fp(running_mean) : nullptr;
  float* rv = running_var.defined() && running_var.numel() ? fp(running_var) : nullptr;
  bn_relu_maxpool(bp(y), fp(gamma), fp(beta), fp(mean), fp(invstd), rm, rv, (float)momentum, (float)eps, fp(partials),
                  (int)partials.size(0), bp(out), am.data_ptr<uint8_t>(), N, H, W, C, (int)k, (int)st, (int)pad, Ho, Wo,
                  cur());
  return {out, am, mean, invstd};
}

at::Tensor maxpool2d_bwd(const at::Tensor& dy, const at::Tensor& am, at::IntArrayRef xshape, int64_t k, int64_t st,
                         int64_t pad) {
  check_bf16(dy, "dy", 4);
  auto dx = at::empty(xshape, dy.options());
  maxpool_bwd(bp(dy), am.data_ptr<uint8_t>(), bp(dx), (int)xshape[0], (int)xshape[1], (int)xshape[2], (int)xshape[3],
              (int)k, (int)st, (int)pad, (int)dy.size(1), (int)dy.size(2), cur());
  return dx;
}

at::Tensor avgpool_fwd_op(const at::Tensor& x) {
  check_bf16(x, "x", 4);
  const int N = (int)x.size(0), HW = (int)(x.size(1) * x.size(2)), C = (int)x.size(3);
  auto y = at::empty({N, C}, x.options());
  avgpool_fwd(bp(x), bp(y), N, HW, C, cur());
  return y;
}

at::Tensor avgpool_bwd_op(const at::Tensor& dy, at::IntArrayRef xshape) {
  check_bf16(dy, "dy", 2);
  auto dx = at::empty(xshape, dy.options());
  avgpool_bwd(bp(dy), bp(dx), (int)xshape[0], (int)(xshape[1] * xshape[2]), (int)xshape[3], cur());
  return dx;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> softmax_xent_op(const at::Tensor& logits, const at::Tensor& labels) {
  check_f32(logits, "logits");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kInt && labels.numel() == logits.size(0), "labels int32");
  const int N = (int)logits.size(0), K = (int)logits.size(1);
  auto loss = at::empty({N}, logits.options());
  auto corr = at::empty({N}, logits.options());
  auto dl = at::empty({N, K}, logits.options().dtype(at::kBFloat16));
  softmax_xent(fp(logits), labels.data_ptr<int>(), fp(loss), fp(corr), bp(dl), N, K, cur());
  return {loss, corr, dl};
}

// The width-paired stem (ResNet conv1: 7x7, stride 2, pad 3, 3 input channels). stem_pack pairs
// horizontally adjacent input pixels into one 8-channel pixel ({p0 c0..2, p1 c0..2, 0, 0}); the filter
// [R][S'][8][K] holds at channel p*3+c of column s' the original tap s = 2s' + p + pad - 2*pw (pw = (pad+1)/2:
// s = 2s' + p - 1 at pad 3, tap -1 zero). The conv is then R x S' x 8 with the height stride / pad and width
// stride 1, left pad pw: 7 x 4 x 8 = 224 MACs per output element instead of 7 x 7 x 8 = 392 over the
// channel-padded input, and the packed input is half the bytes.
ConvShape w2_shape(const at::Tensor& xp, const at::Tensor& wp, int64_t stride, int64_t pad) {
  ConvShape c = shape_of(xp, wp, stride, pad);
  TORCH_CHECK(c.C == 8 && stride == 2 && pad % 2 == 1, "w2 conv: paired input [N, H, W/2, 8], stride 2, odd pad");
  c.stride_w = 1;
  c.pad_w = (int)(pad + 1) / 2;
  c.wo_out = (2 * c.W + 2 * (int)pad - (2 * c.S - 1)) / (int)stride + 1;
  return c;
}

at::Tensor stem_pack_op(const at::Tensor& x) {
  check_f32(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 3 && x.size(2) % 2 == 0 && x.is_contiguous(),
              "stem_pack: x must be contiguous fp32 [N, H, W (even), 3]");
  auto y = at::empty({x.size(0), x.size(1), x.size(2) / 2, 8}, x.options().dtype(at::kBFloat16));
  stem_pack_w2(fp(x), bp(y), x.numel() / 6, cur());
  return y;
}

std::tuple<at::Tensor, at::Tensor> conv2d_fwd_stats_w2(const at::Tensor& xp, const at::Tensor& wp, int64_t stride,
                                                       int64_t pad, const c10::optional<at::Tensor>& part_out) {
  check_bf16(xp, "x", 4);
  check_bf16(wp, "w", 4);
  const ConvShape c = w2_shape(xp, wp, stride, pad);
  auto y = at::empty({c.N, c.Ho(), c.Wo(), c.K}, xp.options());
  auto part = part_buffer(part_out, conv_fwd_stats_rows(c, false), c.K, xp.options(), "conv2d_fwd_stats_w2");
  conv_fwd_stats(c, bp(xp), bp(wp), bp(y), fp(part), cur(), nullptr);
  return {y, part};
}

void conv2d_wgrad_w2(const at::Tensor& xp, const at::Tensor& dy, at::Tensor dwp, int64_t stride, int64_t pad,
                     bool zeroed) {
  check_bf16(xp, "x", 4);
  check_bf16(dy, "dy", 4);
  check_f32(dwp, "dw");
  TORCH_CHECK(dwp.dim() == 4, "dw [R,S',8,K]");
  auto wfake = at::empty({dwp.size(0), dwp.size(1), dwp.size(2), dwp.size(3)}, xp.options().device(at::kCPU));
  const ConvShape c = w2_shape(xp, wfake, stride, pad);
  TORCH_CHECK(dy.size(0) == c.N && dy.size(1) == c.Ho() && dy.size(2) == c.Wo() && dy.size(3) == c.K,
              "wgrad_w2: dy shape mismatch");
  conv_wgrad(c, bp(xp), bp(dy), fp(dwp), conv_wgrad_splits(c, false), cur(), zeroed, nullptr);
}

at::Tensor pad_channels_op(const at::Tensor& x, int64_t cout) {
  check_f32(x, "x");
  const int cin = (int)x.size(-1);
  TORCH_CHECK(cout >= cin && cout % 8 == 0, "pad_channels: need cout >= cin and cout % 8 == 0");
  std::vector<int64_t> sh(x.sizes().begin(), x.sizes().end());
  sh.back() = cout;
  auto y = at::empty(sh, x.options().dtype(at::kBFloat16));
  pad_channels(fp(x), bp(y), (int)(x.numel() / cin), cin, (int)cout, cur());
  return y;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(tfd, m) {
  m.def("conv2d_fwd(Tensor x, Tensor w, int stride, int pad, Tensor? mean=None, Tensor? invstd=None, "
        "Tensor? gamma=None, Tensor? beta=None) -> Tensor");
  m.impl("conv2d_fwd", c10::DispatchKey::CUDA, &conv2d_fwd);
  // part_out: the caller's partials buffer (slot mode: zeroed), returned as the second output
  m.def("conv2d_fwd_stats(Tensor x, Tensor w, int stride, int pad, Tensor? mean=None, Tensor? invstd=None, "
        "Tensor? gamma=None, Tensor? beta=None, Tensor? part_out=None) -> (Tensor, Tensor)");
  m.impl("conv2d_fwd_stats", c10::DispatchKey::CUDA, &conv2d_fwd_stats);
  m.def("conv2d_dgrad(Tensor dy, Tensor w, int[] xshape, int stride, int pad, Tensor? acc=None, Tensor? acc_bits=None, "
        "bool acc_sub2=False) -> Tensor");
  m.impl("conv2d_dgrad", c10::DispatchKey::CUDA, &conv2d_dgrad);
  m.def("conv2d_dgrad_bn(Tensor dy, Tensor w, int[] xshape, int stride, int pad, Tensor? acc, Tensor y, Tensor mean, "
        "Tensor invstd, Tensor gamma, Tensor? beta, Tensor? mask, bool relu, Tensor? acc_bits=None, "
        "Tensor? part_out=None, bool acc_sub2=False) -> (Tensor, Tensor)");
  m.impl("conv2d_dgrad_bn", c10::DispatchKey::CUDA, &conv2d_dgrad_bn);
  m.def("conv2d_wgrad(Tensor x, Tensor dy, Tensor(a!) dw, int stride, int pad, bool zeroed=False, Tensor? mean=None, "
        "Tensor? invstd=None, Tensor? gamma=None, Tensor? beta=None) -> ()");
  m.def("bn_relu_max_channels() -> int", []() -> int64_t { return kBnReluMaxC; });
  m.impl("conv2d_wgrad", c10::DispatchKey::CUDA, &conv2d_wgrad);
  m.def("conv_gemm_core(int mode) -> int", [](int64_t mode) -> int64_t { return conv_gemm_core((int)mode); });
  m.def("conv_halo_mode(int mode) -> int", [](int64_t mode) -> int64_t { return conv_halo_mode((int)mode); });
  m.def("conv_wgrad_clear_mode(int mode) -> int", [](int64_t mode) -> int64_t { return conv_wgrad_clear_mode((int)mode); });
  m.def("gemm_nt(Tensor a, Tensor bt) -> Tensor");
  m.impl("gemm_nt", c10::DispatchKey::CUDA, &gemm_nt_op);
  m.def("linear_fwd(Tensor x, Tensor w, Tensor? bias) -> Tensor");
  m.impl("linear_fwd", c10::DispatchKey::CUDA, &linear_fwd_op);
  m.def("linear_dgrad(Tensor dy, Tensor w) -> Tensor");
  m.impl("linear_dgrad", c10::DispatchKey::CUDA, &linear_dgrad_op);
  m.def("linear_wgrad(Tensor x, Tensor dy, Tensor(a!) dw) -> ()");
  m.impl("linear_wgrad", c10::DispatchKey::CUDA, &linear_wgrad_op);
  m.def("bn_fwd(Tensor y, Tensor gamma, Tensor beta, Tensor? residual, bool relu, Tensor(a!) running_mean, "
        "Tensor(b!) running_var, float momentum, float eps, Tensor? partials=None, Tensor(c!)? mask=None) -> "
        "(Tensor, Tensor, Tensor)");
  m.impl("bn_fwd", c10::DispatchKey::CUDA, &bn_fwd);
  m.def("bn_stats(Tensor y, Tensor partials, Tensor(a!) running_mean, Tensor(b!) running_var, float momentum, "
        "float eps) -> (Tensor, Tensor)");
  m.impl("bn_stats", c10::DispatchKey::CUDA, &bn_stats);
  m.def("bn_bwd(Tensor dout, Tensor out, Tensor y, Tensor gamma, Tensor mean, Tensor invstd, bool relu, "
        "bool want_dres, Tensor(a!) dgamma, Tensor(b!) dbeta, Tensor? beta=None, Tensor? mask=None, "
        "Tensor? partials=None) -> (Tensor, Tensor)");
  // rows of a statistics-partials buffer in slot mode (TFD_BN_SLOTS; 0: one row per producer block)
  m.def("bn_part_slots() -> int", []() -> int64_t { return bn_slots(); });
  // switch the mode (between steps only; returns the previous one) -- the bit-exact tests take row mode
  m.def("set_bn_part_slots(int slots) -> int", [](int64_t s) -> int64_t {
    const int old = bn_slots();
    set_bn_slots((int)s);
    return old;
  });
  m.impl("bn_bwd", c10::DispatchKey::CUDA, &bn_bwd);
  m.def("bn_infer(Tensor y, Tensor gamma, Tensor beta, Tensor rm, Tensor rv, float eps, bool relu) -> Tensor");
  m.impl("bn_infer", c10::DispatchKey::CUDA, &bn_infer_op);
  m.def("maxpool2d_fwd(Tensor x, int k, int stride, int pad) -> (Tensor, Tensor)");
  m.impl("maxpool2d_fwd", c10::DispatchKey::CUDA, &maxpool2d_fwd);
  m.def("bn_relu_maxpool(Tensor y, Tensor gamma, Tensor beta, Tensor(a!) running_mean, Tensor(b!) running_var, "
        "float momentum, float eps, Tensor partials, int k, int stride, int pad) -> (Tensor, Tensor, Tensor, Tensor)");
  m.impl("bn_relu_maxpool", c10::DispatchKey::CUDA, &bn_relu_maxpool_op);
  m.def("maxpool2d_bwd(Tensor dy, Tensor argmax, int[] xshape, int k, int stride, int pad) -> Tensor");
  m.impl("maxpool2d_bwd", c10::DispatchKey::CUDA, &maxpool2d_bwd);
  m.def("avgpool_fwd(Tensor x) -> Tensor");
  m.impl("avgpool_fwd", c10::DispatchKey::CUDA, &avgpool_fwd_op);
  m.def("avgpool_bwd(Tensor dy, int[] xshape) -> Tensor");
  m.impl("avgpool_bwd", c10::DispatchKey::CUDA, &avgpool_bwd_op);
  m.def("softmax_xent(Tensor logits, Tensor labels) -> (Tensor, Tensor, Tensor)");
  m.impl("softmax_xent", c10::DispatchKey::CUDA, &softmax_xent_op);
  m.def("pad_channels(Tensor x, int cout) -> Tensor");
  m.impl("pad_channels", c10::DispatchKey::CUDA, &pad_channels_op);
  m.def("stem_pack(Tensor x) -> Tensor");
  m.impl("stem_pack", c10::DispatchKey::CUDA, &stem_pack_op);
  m.def("conv2d_fwd_stats_w2(Tensor x, Tensor w, int stride, int pad, Tensor? part_out=None) -> (Tensor, Tensor)");
  m.impl("conv2d_fwd_stats_w2", c10::DispatchKey::CUDA, &conv2d_fwd_stats_w2);
  m.def("conv2d_wgrad_w2(Tensor x, Tensor dy, Tensor(a!) dw, int stride, int pad, bool zeroed=False) -> ()");
  m.impl("conv2d_wgrad_w2", c10::DispatchKey::CUDA, &conv2d_wgrad_w2);
}

}  // namespace tfd
