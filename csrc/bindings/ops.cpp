// Torch custom-op registration for the native library (namespace `tfd`, see torch.ops.tfd.*).
// Ops run on the caller's current HIP stream so they compose with torch stream/graph semantics.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "../tfd_kernels.h"

namespace tfd {
uint32_t crc32c_extend(uint32_t init, const void* data, size_t n);

namespace {
hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }

int64_t crc32c_op(const at::Tensor& bytes, int64_t init) {
  TORCH_CHECK(!bytes.is_cuda() && bytes.is_contiguous(), "crc32c: contiguous CPU tensor");
  return (int64_t)crc32c_extend((uint32_t)init, bytes.data_ptr(), (size_t)bytes.nbytes());
}

void adam_flat(at::Tensor p, at::Tensor m, at::Tensor v, at::Tensor g, c10::optional<at::Tensor> pbf, double lr,
               double b1, double b2, double eps, at::Tensor step, double grad_scale) {
  TORCH_CHECK(p.is_cuda() && p.scalar_type() == at::kFloat && p.is_contiguous(), "adam_flat: fp32 GPU params");
  TORCH_CHECK(m.numel() == p.numel() && v.numel() == p.numel() && g.numel() == p.numel(), "adam_flat: sizes");
  TORCH_CHECK(step.scalar_type() == at::kLong && step.is_cuda(), "adam_flat: int64 GPU step");
  const bool gb = g.scalar_type() == at::kBFloat16;
  AdamArgs a{(float*)p.data_ptr(), (float*)m.data_ptr(), (float*)v.data_ptr(), gb ? nullptr : (const float*)g.data_ptr(),
             pbf ? (uint16_t*)pbf->data_ptr() : nullptr, gb ? (const uint16_t*)g.data_ptr() : nullptr, p.numel(),
             (float)lr, (float)b1, (float)b2, (float)eps, (const int64_t*)step.data_ptr(), 1, (float)grad_scale};
  adam_apply(a, cur());
}

void momentum_flat(at::Tensor p, c10::optional<at::Tensor> mom, at::Tensor g, c10::optional<at::Tensor> pbf,
                   double lr, double momentum, double weight_decay, bool nesterov, double grad_scale) {
  TORCH_CHECK(p.is_cuda() && p.scalar_type() == at::kFloat && p.is_contiguous(), "momentum_flat: fp32 GPU params");
  const bool gb = g.scalar_type() == at::kBFloat16;
  SgdArgs a{(float*)p.data_ptr(), mom ? (float*)mom->data_ptr() : nullptr, gb ? nullptr : (const float*)g.data_ptr(),
            pbf ? (uint16_t*)pbf->data_ptr() : nullptr, gb ? (const uint16_t*)g.data_ptr() : nullptr, p.numel(),
            (float)lr, (float)momentum, (float)weight_decay, (float)grad_scale, nesterov ? 1 : 0};
  sgd_apply(a, cur());
}

void roofline_stream(at::Tensor p, at::Tensor m, at::Tensor v, const at::Tensor& g, at::Tensor pbf,
                     c10::optional<at::Tensor> x, int64_t blocks, int64_t unroll) {
  const int64_t n = p.numel();
  TORCH_CHECK(p.is_cuda() && p.scalar_type() == at::kFloat && p.is_contiguous() && n % 4 == 0, "roofline_stream: p");
  TORCH_CHECK(m.numel() == n && v.numel() == n && g.numel() == n && pbf.numel() == n, "roofline_stream: sizes");
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 && pbf.scalar_type() == at::kBFloat16, "roofline_stream: bf16 g / pbf");
  const int64_t nx = x ? x->numel() : 0;
  TORCH_CHECK(nx % 4 == 0 && nx <= n && (!x || x->scalar_type() == at::kFloat), "roofline_stream: x");
  stream_floor((float*)p.data_ptr(), (float*)m.data_ptr(), (float*)v.data_ptr(), (const uint16_t*)g.data_ptr(),
               (uint16_t*)pbf.data_ptr(), x ? (const float*)x->data_ptr() : nullptr, n / 4, nx / 4, (int)blocks,
               (int)unroll, cur());
}

void noop_op(int64_t blocks) { noop_launch((int)blocks, cur()); }

at::Tensor to_bf16(const at::Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat, "to_bf16: fp32 GPU");
  auto xc = x.contiguous();
  auto y = at::empty(xc.sizes(), xc.options().dtype(at::kBFloat16));
  cast_f32_bf16((const float*)xc.data_ptr(), (uint16_t*)y.data_ptr(), xc.numel(), cur());
  return y;
}
}  // namespace

TORCH_LIBRARY(tfd, m) {
  m.def("crc32c(Tensor bytes, int init=0) -> int");
  m.impl("crc32c", c10::DispatchKey::CPU, &crc32c_op);
  m.def("adam_flat(Tensor(a!) p, Tensor(b!) m, Tensor(c!) v, Tensor g, Tensor(d!)? pbf, float lr, float b1, float b2, "
        "float eps, Tensor(e!) step, float grad_scale=1.0) -> ()");
  m.impl("adam_flat", c10::DispatchKey::CUDA, &adam_flat);
  m.def("momentum_flat(Tensor(a!) p, Tensor(b!)? mom, Tensor g, Tensor(d!)? pbf, float lr, float momentum, "
        "float weight_decay, bool nesterov, float grad_scale=1.0) -> ()");
  m.impl("momentum_flat", c10::DispatchKey::CUDA, &momentum_flat);
  m.def("roofline_stream(Tensor(a!) p, Tensor(b!) m, Tensor(c!) v, Tensor g, Tensor(d!) pbf, Tensor? x, int blocks, "
        "int unroll) -> ()");
  m.impl("roofline_stream", c10::DispatchKey::CUDA, &roofline_stream);
  m.def("noop(int blocks) -> ()");
  m.impl("noop", c10::DispatchKey::CompositeExplicitAutograd, &noop_op);
  m.def("to_bf16(Tensor x) -> Tensor");
  m.impl("to_bf16", c10::DispatchKey::CUDA, &to_bf16);
}

}  // namespace tfd
