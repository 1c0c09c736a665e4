// IpcComm: peer-to-peer (IPC-mapped) communicator for latency-bound small collectives
// (SURVEY.md §2.2 N3, §5.8 item 3). One process per GPU; each rank exports a staging buffer
// (coarse-grained device memory) and an uncached signal region with hipIpcGetMemHandle; the
// 2 x 64-byte handles are exchanged over the control plane (Gloo) and opened in every peer.
// all_reduce() is one kernel (csrc/comm/ipc_allreduce.hip) and can be captured into a hipGraph.
// Ranks may share one GPU (two processes, same device): that is how the protocol is tested on a
// one-GPU box, where RCCL refuses duplicate devices.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <cstdlib>
#include <cstring>
#include <algorithm>

#include "../ipc_kernels.h"
#include "ipc_comm.h"

namespace tfd {

#define HIP_OK2(x)                                                                         \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    TORCH_CHECK(e_ == hipSuccess, #x, " failed: ", hipGetErrorString(e_));                 \
  } while (0)

IpcComm::IpcComm(int64_t world, int64_t rank, int64_t device, int64_t capacity_elems)
    : world_(world), rank_(rank), device_(device), cap_(capacity_elems) {
  TORCH_CHECK(world >= 1 && world <= kIpcMaxRanks, "IpcComm: world must be in [1, ", kIpcMaxRanks, "]");
  TORCH_CHECK(rank >= 0 && rank < world, "IpcComm: bad rank");
  TORCH_CHECK(capacity_elems > 0, "IpcComm: capacity");
  HIP_OK2(hipSetDevice((int)device));
  // two halves of cap_ fp32 (call v stages into half v & 1: double buffering instead of an END barrier)
  HIP_OK2(hipMalloc(&stage_, 2 * (size_t)cap_ * sizeof(float)));
  HIP_OK2(hipExtMallocWithFlags(&sig_, kIpcSigInts * sizeof(int), hipDeviceMallocUncached));
  HIP_OK2(hipMemset(sig_, 0, kIpcSigInts * sizeof(int)));
  HIP_OK2(hipMemset(stage_, 0, 2 * (size_t)cap_ * sizeof(float)));
  HIP_OK2(hipDeviceSynchronize());
  HIP_OK2(hipEventCreateWithFlags(&last_ev_, hipEventDisableTiming));
  for (int i = 0; i < kIpcMaxRanks; ++i) {
    peer_stage_[i] = nullptr;
    peer_sig_[i] = nullptr;
  }
  peer_stage_[rank] = stage_;
  peer_sig_[rank] = (int*)sig_;
}

IpcComm::~IpcComm() { close(); }

at::Tensor IpcComm::handle() {
  hipIpcMemHandle_t h[2];
  HIP_OK2(hipIpcGetMemHandle(&h[0], stage_));
  HIP_OK2(hipIpcGetMemHandle(&h[1], sig_));
  auto t = at::empty({2 * (int64_t)sizeof(hipIpcMemHandle_t)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), h, sizeof(h));
  return t;
}

void IpcComm::open(const at::Tensor& all) {
  TORCH_CHECK(!opened_, "IpcComm: already opened");
  const int64_t hb = 2 * (int64_t)sizeof(hipIpcMemHandle_t);
  TORCH_CHECK(all.numel() == world_ * hb && all.scalar_type() == at::kByte, "IpcComm.open: [world, 128] uint8");
  auto c = all.contiguous().cpu();
  const uint8_t* base = c.data_ptr<uint8_t>();
  HIP_OK2(hipSetDevice((int)device_));
  for (int p = 0; p < world_; ++p) {
    if (p == rank_) continue;
    hipIpcMemHandle_t h[2];
    std::memcpy(h, base + p * hb, sizeof(h));
    HIP_OK2(hipIpcOpenMemHandle(&peer_stage_[p], h[0], hipIpcMemLazyEnablePeerAccess));
    HIP_OK2(hipIpcOpenMemHandle((void**)&peer_sig_[p], h[1], hipIpcMemLazyEnablePeerAccess));
  }
  opened_ = true;
}

void IpcComm::close() {
  if (opened_) {
    for (int p = 0; p < world_; ++p) {
      if (p == rank_) continue;
      if (peer_stage_[p]) hipIpcCloseMemHandle(peer_stage_[p]);
      if (peer_sig_[p]) hipIpcCloseMemHandle(peer_sig_[p]);
      peer_stage_[p] = nullptr;
      peer_sig_[p] = nullptr;
    }
    opened_ = false;
  }
  if (stage_) {
    hipFree(stage_);
    stage_ = nullptr;
  }
  if (sig_) {
    hipFree(sig_);
    sig_ = nullptr;
  }
  if (last_ev_) {
    hipEventDestroy(last_ev_);
    last_ev_ = nullptr;
  }
}

static bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  HIP_OK2(hipStreamIsCapturing(s, &st));
  return st != hipStreamCaptureStatusNone;
}

void IpcComm::order(hipStream_t s) {
  if (last_recorded_ && s != last_stream_ && !capturing(s)) HIP_OK2(hipStreamWaitEvent(s, last_ev_, 0));
}

void IpcComm::mark(hipStream_t s) {
  last_stream_ = s;
  last_recorded_ = !capturing(s);
  if (last_recorded_) HIP_OK2(hipEventRecord(last_ev_, s));
}

// Grid of a spinning collective: every block of it must become resident while the peers' blocks
// are resident too. Ranks that share one GPU compete for its CUs with two spinning kernels plus
// their other streams' work; grids of up to 256 blocks there hung in 2 of 4 DP runs (a block
// spinning for a peer block that could not be dispatched), 8-block grids in none
// (scripts/gpu_diag_ipc.sh). set_max_blocks() caps it; TFD_IPC_MAX_BLOCKS overrides.
int IpcComm::blocks(int64_t n) const {
  static const int env_cap = [] {
    const char* e = std::getenv("TFD_IPC_MAX_BLOCKS");
    return e ? std::max(1, std::atoi(e)) : 0;
  }();
  return std::min(ipc_blocks_for(n), env_cap ? env_cap : max_blocks_);
}
void IpcComm::set_max_blocks(int64_t b) { max_blocks_ = (int)std::max<int64_t>(1, std::min<int64_t>(b, kIpcMaxBlocks)); }

void IpcComm::all_reduce_raw(const void* in, bool in_bf16, void* out, bool out_bf16, int64_t n, double scale,
                             hipStream_t s) {
  TORCH_CHECK(opened_ || world_ == 1, "IpcComm: open() the peer handles first");
  TORCH_CHECK(n <= cap_, "IpcComm: ", n, " elements exceed the staging capacity ", cap_);
  IpcAllReduceArgs a{};
  a.in = in;
  a.out = out;
  for (int p = 0; p < world_; ++p) {
    a.stage[p] = peer_stage_[p];
    a.sig[p] = peer_sig_[p];
  }
  a.n = n;
  a.rank = (int)rank_;
  a.world = (int)world_;
  a.in_bf16 = in_bf16 ? 1 : 0;
  a.out_bf16 = out_bf16 ? 1 : 0;
  a.scale = (float)scale;
  a.spin_limit_ticks = spin_ticks_;
  a.half_bytes = cap_ * (int64_t)sizeof(float);
  order(s);
  ipc_allreduce(a, blocks(n), s);
  mark(s);
}

void IpcComm::all_reduce(const at::Tensor& t, double scale) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "IpcComm.all_reduce: contiguous GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "IpcComm: fp32/bf16 only");
  const bool bf = t.scalar_type() == at::kBFloat16;
  all_reduce_raw(t.data_ptr(), bf, t.data_ptr(), bf, t.numel(), scale, c10::hip::getCurrentHIPStream().stream());
}

void IpcComm::all_reduce_into(const at::Tensor& in, const at::Tensor& out, double scale) {
  for (const at::Tensor* t : {&in, &out}) {
    TORCH_CHECK(t->is_cuda() && t->is_contiguous(), "IpcComm.all_reduce_into: contiguous GPU tensors");
    TORCH_CHECK(t->scalar_type() == at::kFloat || t->scalar_type() == at::kBFloat16, "IpcComm: fp32/bf16 only");
  }
  TORCH_CHECK(in.numel() == out.numel(), "IpcComm.all_reduce_into: in and out sizes differ");
  all_reduce_raw(in.data_ptr(), in.scalar_type() == at::kBFloat16, out.data_ptr(), out.scalar_type() == at::kBFloat16,
                 in.numel(), scale, c10::hip::getCurrentHIPStream().stream());
}

void IpcComm::reduce_scatter_raw(const void* in, bool in_bf16, void* out, bool out_bf16, int64_t shard, double scale,
                                 hipStream_t s) {
  TORCH_CHECK(opened_ || world_ == 1, "IpcComm: open() the peer handles first");
  TORCH_CHECK(shard * world_ <= cap_, "IpcComm.reduce_scatter: ", shard * world_, " elements exceed capacity ", cap_);
  IpcAllReduceArgs a{};
  a.in = in;
  a.out = out;
  for (int p = 0; p < world_; ++p) {
    a.stage[p] = peer_stage_[p];
    a.sig[p] = peer_sig_[p];
  }
  a.n = shard;
  a.rank = (int)rank_;
  a.world = (int)world_;
  a.in_bf16 = in_bf16 ? 1 : 0;
  a.out_bf16 = out_bf16 ? 1 : 0;
  a.scale = (float)scale;
  a.spin_limit_ticks = spin_ticks_;
  a.half_bytes = cap_ * (int64_t)sizeof(float);
  TORCH_CHECK(shard % 8 == 0, "IpcComm.reduce_scatter: shard must be a multiple of 8 elements");
  order(s);
  ipc_reduce_scatter(a, blocks(shard), s);
  mark(s);
}

void IpcComm::all_gather_raw(void* buf, int elem_bytes, int64_t shard, hipStream_t s) {
  TORCH_CHECK(opened_ || world_ == 1, "IpcComm: open() the peer handles first");
  TORCH_CHECK(elem_bytes == 2 || elem_bytes == 4, "IpcComm.all_gather: 2- or 4-byte elements");
  TORCH_CHECK(shard * elem_bytes <= cap_ * 4, "IpcComm.all_gather: shard exceeds staging capacity");
  IpcAllReduceArgs a{};
  a.out = buf;
  for (int p = 0; p < world_; ++p) {
    a.stage[p] = peer_stage_[p];
    a.sig[p] = peer_sig_[p];
  }
  a.n = shard;
  a.rank = (int)rank_;
  a.world = (int)world_;
  a.spin_limit_ticks = spin_ticks_;
  a.half_bytes = cap_ * (int64_t)sizeof(float);
  TORCH_CHECK(shard % 8 == 0, "IpcComm.all_gather: shard must be a multiple of 8 elements");
  order(s);
  ipc_all_gather(a, elem_bytes, blocks(shard), s);
  mark(s);
}

void IpcComm::reduce_scatter(const at::Tensor& in, const at::Tensor& out, double scale) {
  TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.is_contiguous() && out.is_contiguous(), "reduce_scatter: GPU");
  TORCH_CHECK(in.numel() == out.numel() * world_, "reduce_scatter: in must be world * out elements");
  reduce_scatter_raw(in.data_ptr(), in.scalar_type() == at::kBFloat16, out.data_ptr(),
                     out.scalar_type() == at::kBFloat16, out.numel(), scale, c10::hip::getCurrentHIPStream().stream());
}

void IpcComm::all_gather(const at::Tensor& buf) {
  TORCH_CHECK(buf.is_cuda() && buf.is_contiguous() && buf.numel() % world_ == 0, "all_gather: GPU, divisible");
  all_gather_raw(buf.data_ptr(), (int)buf.element_size(), buf.numel() / world_,
                 c10::hip::getCurrentHIPStream().stream());
}

int64_t IpcComm::error() {
  int v = 0;
  HIP_OK2(hipMemcpy(&v, (int*)sig_ + kIpcSigFlags, sizeof(int), hipMemcpyDeviceToHost));
  return v;
}

void IpcComm::set_spin_limit_ms(double ms) { spin_ticks_ = (int64_t)(ms * 1e5); }  // 100 MHz clock

TORCH_LIBRARY_FRAGMENT(tfd, m) {
  m.class_<IpcComm>("IpcComm")
      .def(torch::init<int64_t, int64_t, int64_t, int64_t>())
      .def("handle", &IpcComm::handle)
      .def("open", &IpcComm::open)
      .def("close", &IpcComm::close)
      .def("all_reduce", &IpcComm::all_reduce)
      .def("all_reduce_into", &IpcComm::all_reduce_into)
      .def("reduce_scatter", &IpcComm::reduce_scatter)
      .def("all_gather", &IpcComm::all_gather)
      .def("error", &IpcComm::error)
      .def("set_spin_limit_ms", &IpcComm::set_spin_limit_ms)
      .def("set_max_blocks", &IpcComm::set_max_blocks)
      .def("world", &IpcComm::world)
      .def("rank", &IpcComm::rank);
}

}  // namespace tfd
