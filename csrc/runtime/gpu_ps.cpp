// GPU-resident parameter server (VERDICT r2 "next round" item 6).
//
// The reference keeps every variable and its Adam slots on the PS tasks' CPUs
// (replica_device_setter(ps_device="/job:ps/cpu:0"), /root/reference/mnist_python_m.py:164-177)
// and moves whole gradients / parameters over gRPC each step (:247-253 async, :210-222 sync with
// an accumulator). Here a PS task owns its shard on a GPU:
//
//   GpuPsShard (PS side): fp32 params + optimizer slots of the shard's variable ranges, one
//     gradient MAILBOX slot per worker (plain device memory exported with hipIpcGetMemHandle), and
//     IPC mappings of every worker's flat parameter buffer. apply()/accumulate() run the flat
//     optimizer kernels (csrc/kernels/optim.hip) on the mailbox; push() writes the updated ranges
//     straight into the worker's engine parameters (peer memory over xGMI, or the same GPU).
//   GpuPsPort (worker side): maps each PS's mailbox and copies the worker's gradient ranges into
//     its slot with device-to-device copies; exports the worker's own parameter buffer.
//
// No gradient or parameter byte goes through host memory; the control plane (who pushed, global
// step, token replies) stays a 32-byte Gloo message (parallel/gpu_ps.py). Ordering: every data
// operation ends in a stream synchronize BEFORE its control message is sent, so the receiver's
// next kernel (which starts with the kernel-boundary cache acquire) sees the bytes.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <vector>

#include "../tfd_kernels.h"

namespace tfd {

#define PS_OK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    TORCH_CHECK(e_ == hipSuccess, #x, " failed: ", hipGetErrorString(e_));                 \
  } while (0)

namespace {

constexpr int64_t kExportBytes = (int64_t)sizeof(hipIpcMemHandle_t) + 2 * (int64_t)sizeof(int64_t);

// IPC export of a device buffer: the handle of its whole allocation (tensors from the caching
// allocator live inside larger segments) + the byte offset of the buffer in it + its size.
at::Tensor export_ptr(void* p, int64_t nbytes) {
  void* base = nullptr;
  size_t size = 0;
  PS_OK(hipMemGetAddressRange(&base, &size, p));
  hipIpcMemHandle_t h;
  PS_OK(hipIpcGetMemHandle(&h, base));
  auto t = at::empty({kExportBytes}, at::TensorOptions().dtype(at::kByte));
  auto* o = (uint8_t*)t.data_ptr();
  std::memcpy(o, &h, sizeof(h));
  const int64_t off = (int64_t)((char*)p - (char*)base);
  std::memcpy(o + sizeof(h), &off, sizeof(off));
  std::memcpy(o + sizeof(h) + sizeof(off), &nbytes, sizeof(nbytes));
  return t;
}

struct Mapping {
  void* base = nullptr;  // hipIpcOpenMemHandle result (allocation base)
  char* ptr = nullptr;   // the exported buffer inside it
  int64_t nbytes = 0;
  void open(const at::Tensor& ex) {
    TORCH_CHECK(ex.numel() == kExportBytes && ex.scalar_type() == at::kByte && !ex.is_cuda(), "bad IPC export");
    auto t = ex.contiguous();
    const auto* o = (const uint8_t*)t.data_ptr();
    hipIpcMemHandle_t h;
    int64_t off = 0;
    std::memcpy(&h, o, sizeof(h));
    std::memcpy(&off, o + sizeof(h), sizeof(off));
    std::memcpy(&nbytes, o + sizeof(h) + sizeof(off), sizeof(nbytes));
    close();
    PS_OK(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess));
    ptr = (char*)base + off;
  }
  void close() {
    if (base) (void)hipIpcCloseMemHandle(base);
    base = nullptr;
    ptr = nullptr;
  }
};

// [R][2] int64 CPU tensor of (flat offset, length) -> vector; returns the total length
int64_t read_ranges(const at::Tensor& r, std::vector<std::pair<int64_t, int64_t>>* out) {
  TORCH_CHECK(!r.is_cuda() && r.scalar_type() == at::kLong && r.dim() == 2 && r.size(1) == 2,
              "ranges: [R][2] int64 CPU tensor of (offset, length)");
  auto c = r.contiguous();
  const int64_t* d = c.data_ptr<int64_t>();
  int64_t tot = 0;
  out->clear();
  for (int64_t i = 0; i < c.size(0); ++i) {
    TORCH_CHECK(d[2 * i] >= 0 && d[2 * i + 1] >= 0, "ranges: negative entry");
    out->emplace_back(d[2 * i], d[2 * i + 1]);
    tot += d[2 * i + 1];
  }
  return tot;
}

}  // namespace

class GpuPsShard : public torch::CustomClassHolder {
 public:
  // opt: 0 Adam (lr, b1, b2, eps), 1 GradientDescent (lr), 2 Momentum (lr, momentum), 3 Nesterov
  GpuPsShard(int64_t device, at::Tensor ranges, int64_t flat_total, int64_t n_workers, int64_t opt, double lr,
             double b1, double b2, double eps, double momentum, bool sync)
      : device_(device), total_(flat_total), nw_(n_workers), opt_(opt), lr_(lr), b1_(b1), b2_(b2), eps_(eps),
        mom_(momentum), sync_(sync) {
    n_ = read_ranges(ranges, &ranges_);
    for (auto& r : ranges_) TORCH_CHECK(r.first + r.second <= flat_total, "range past the flat buffer");
    TORCH_CHECK(n_workers >= 1 && n_workers <= 1024, "n_workers");
    TORCH_CHECK(opt >= 0 && opt <= 3, "opt kind");
    PS_OK(hipSetDevice((int)device));
    PS_OK(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
    auto f32 = at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device);
    const int64_t n = std::max<int64_t>(n_, 4);
    params_ = at::zeros({n}, f32);
    m_ = at::zeros({n}, f32);
    v_ = at::zeros({n}, f32);
    if (sync) acc_ = at::zeros({n}, f32);
    // mailbox: its own allocation (exported whole), one fp32 slot per worker, 16-B aligned slots
    slot_ = (n + 3) / 4 * 4;
    PS_OK(hipMalloc(&mail_, (size_t)nw_ * slot_ * sizeof(float)));
    PS_OK(hipMemset(mail_, 0, (size_t)nw_ * slot_ * sizeof(float)));
    PS_OK(hipDeviceSynchronize());
    workers_.resize(nw_);
  }
  ~GpuPsShard() override {
    for (auto& w : workers_) w.close();
    if (mail_) (void)hipFree(mail_);
    if (s_) (void)hipStreamDestroy(s_);
  }

  int64_t numel() const { return n_; }
  int64_t updates() const { return t_; }
  // 1 (default): peer-buffer copies by a copy kernel on the shard's stream; 0: hipMemcpyAsync
  void set_copy_kernel(bool on) { copy_kernel_ = on; }
  at::Tensor params() { return params_.narrow(0, 0, n_); }
  at::Tensor slot_m() { return m_.narrow(0, 0, n_); }
  at::Tensor slot_v() { return v_.narrow(0, 0, n_); }
  at::Tensor mailbox() { return export_ptr(mail_, nw_ * slot_ * (int64_t)sizeof(float)); }
  void open_worker(int64_t w, at::Tensor exported) {
    TORCH_CHECK(w >= 0 && w < nw_, "worker index");
    workers_[w].open(exported);
    TORCH_CHECK(workers_[w].nbytes >= total_ * (int64_t)sizeof(float), "worker buffer smaller than the flat params");
  }

  // chief's init: the shard's ranges of worker w's parameters (its engine buffer, peer memory)
  void pull_init(int64_t w, int64_t t) {
    copy_ranges(/*to_worker=*/false, w);
    PS_OK(hipMemsetAsync(m_.data_ptr(), 0, m_.numel() * sizeof(float), s_));
    PS_OK(hipMemsetAsync(v_.data_ptr(), 0, v_.numel() * sizeof(float), s_));
    if (sync_) PS_OK(hipMemsetAsync(acc_.data_ptr(), 0, acc_.numel() * sizeof(float), s_));
    PS_OK(hipStreamSynchronize(s_));
    t_ = t;
  }
  // restore: values (and slots, when given) in the shard's compact layout, any device
  void load_state(at::Tensor p, c10::optional<at::Tensor> m, c10::optional<at::Tensor> v, int64_t t) {
    TORCH_CHECK(p.numel() == n_, "load_state: shard size");
    params().copy_(p);
    if (m) slot_m().copy_(*m); else slot_m().zero_();
    if (v) slot_v().copy_(*v); else slot_v().zero_();
    if (sync_) acc_.zero_();
    PS_OK(hipDeviceSynchronize());
    t_ = t;
  }
  // async (Hogwild) update with worker w's mailbox gradient: TF ApplyAdam / SGD / Momentum, t += 1
  void apply(int64_t w, double scale) {
    TORCH_CHECK(w >= 0 && w < nw_, "worker index");
    step_with(mail_ + w * slot_, scale);
    PS_OK(hipStreamSynchronize(s_));
  }
  // sync (backup workers): acc += mailbox[w]
  void accumulate(int64_t w) {
    TORCH_CHECK(sync_ && w >= 0 && w < nw_, "accumulate: sync shard, worker index");
    vec_accumulate((float*)acc_.data_ptr(), mail_ + w * slot_, n_, 1.f, s_);
    PS_OK(hipStreamSynchronize(s_));
  }
  // sync: one averaged update from the accumulator (scale = 1/R), then acc = 0
  void apply_accumulated(double scale) {
    TORCH_CHECK(sync_, "apply_accumulated: sync shard");
    step_with((const float*)acc_.data_ptr(), scale);
    PS_OK(hipMemsetAsync(acc_.data_ptr(), 0, acc_.numel() * sizeof(float), s_));
    PS_OK(hipStreamSynchronize(s_));
  }
  // the shard's current values -> worker w's engine parameters (its ranges only)
  void push(int64_t w) {
    copy_ranges(/*to_worker=*/true, w);
    PS_OK(hipStreamSynchronize(s_));
  }

 private:
  void step_with(const float* g, double scale) {
    if (n_ == 0) { ++t_; return; }
    if (opt_ == 0) {
      AdamArgs a{(float*)params_.data_ptr(), (float*)m_.data_ptr(), (float*)v_.data_ptr(), g, nullptr, nullptr, n_,
                 (float)lr_, (float)b1_, (float)b2_, (float)eps_, nullptr, (int)(t_ + 1), (float)scale};
      adam_apply(a, s_);
    } else {
      SgdArgs a{(float*)params_.data_ptr(), opt_ >= 2 ? (float*)m_.data_ptr() : nullptr, g, nullptr, nullptr, n_,
                (float)lr_, opt_ >= 2 ? (float)mom_ : 0.f, 0.f, (float)scale, opt_ == 3 ? 1 : 0};
      sgd_apply(a, s_);
    }
    ++t_;
  }
  void copy_ranges(bool to_worker, int64_t w) {
    TORCH_CHECK(w >= 0 && w < nw_ && workers_[w].ptr, "worker ", w, " not opened");
    char* wb = workers_[w].ptr;
    char* pb = (char*)params_.data_ptr();
    int64_t o = 0;
    for (auto& r : ranges_) {
      char* wp = wb + r.first * (int64_t)sizeof(float);
      char* sp = pb + o * (int64_t)sizeof(float);
      const size_t bytes = (size_t)r.second * sizeof(float);
      if (bytes && copy_kernel_) copy_f32((float*)(to_worker ? wp : sp), (const float*)(to_worker ? sp : wp), r.second, s_);
      else if (bytes) PS_OK(hipMemcpyAsync(to_worker ? wp : sp, to_worker ? sp : wp, bytes, hipMemcpyDeviceToDevice, s_));
      o += r.second;
    }
  }

  int64_t device_, total_, nw_, opt_;
  double lr_, b1_, b2_, eps_, mom_;
  bool sync_;
  int64_t n_ = 0, slot_ = 0, t_ = 0;
  bool copy_kernel_ = true;
  std::vector<std::pair<int64_t, int64_t>> ranges_;
  at::Tensor params_, m_, v_, acc_;
  float* mail_ = nullptr;
  hipStream_t s_ = nullptr;
  std::vector<Mapping> workers_;
};

class GpuPsPort : public torch::CustomClassHolder {
 public:
  GpuPsPort(int64_t device, int64_t num_ps) : device_(device), ps_(num_ps), ranges_(num_ps) {
    TORCH_CHECK(num_ps >= 1 && num_ps <= 64, "num_ps");
    PS_OK(hipSetDevice((int)device));
    PS_OK(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
  }
  ~GpuPsPort() override {
    for (auto& m : ps_) m.close();
    if (s_) (void)hipStreamDestroy(s_);
  }
  // this worker's flat parameter buffer, for the PS tasks to push into
  at::Tensor export_buffer(at::Tensor t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "export_buffer: contiguous device tensor");
    return export_ptr(t.data_ptr(), t.numel() * t.element_size());
  }
  // PS p's mailbox and the (offset, length) ranges it owns, in its compact order
  void open_ps(int64_t p, at::Tensor mailbox, at::Tensor ranges, int64_t slot_elems) {
    TORCH_CHECK(p >= 0 && p < (int64_t)ps_.size(), "ps index");
    ps_[p].open(mailbox);
    read_ranges(ranges, &ranges_[p]);
    slot_[p] = slot_elems;
  }
  // the worker's fp32 flat gradient (ranges of PS p) -> its mailbox slot `w`; returns after the copy
  void set_copy_kernel(bool on) { copy_kernel_ = on; }
  void push_grad(int64_t p, int64_t w, at::Tensor grad) {
    TORCH_CHECK(grad.is_cuda() && grad.scalar_type() == at::kFloat && grad.is_contiguous(), "fp32 device grad");
    TORCH_CHECK(p >= 0 && p < (int64_t)ps_.size() && ps_[p].ptr, "PS ", p, " not opened");
    auto sl = slot_.find(p);
    TORCH_CHECK(sl != slot_.end(), "PS slot size unknown");
    TORCH_CHECK((w + 1) * sl->second * (int64_t)sizeof(float) <= ps_[p].nbytes, "mailbox slot past the export");
    // the gradient is produced on the caller's stream: order the copies behind it
    hipEvent_t ev;
    PS_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    PS_OK(hipEventRecord(ev, c10::hip::getCurrentHIPStream().stream()));
    PS_OK(hipStreamWaitEvent(s_, ev, 0));
    char* dst = ps_[p].ptr + w * sl->second * (int64_t)sizeof(float);
    const char* src = (const char*)grad.data_ptr();
    int64_t o = 0;
    for (auto& r : ranges_[p]) {
      TORCH_CHECK(r.first + r.second <= grad.numel(), "range past the gradient");
      if (r.second && copy_kernel_)
        copy_f32((float*)(dst + o * (int64_t)sizeof(float)), (const float*)(src + r.first * (int64_t)sizeof(float)),
                 r.second, s_);
      else if (r.second)
        PS_OK(hipMemcpyAsync(dst + o * (int64_t)sizeof(float), src + r.first * (int64_t)sizeof(float),
                             (size_t)r.second * sizeof(float), hipMemcpyDeviceToDevice, s_));
      o += r.second;
    }
    PS_OK(hipStreamSynchronize(s_));
    (void)hipEventDestroy(ev);
  }

 private:
  int64_t device_;
  std::vector<Mapping> ps_;
  std::vector<std::vector<std::pair<int64_t, int64_t>>> ranges_;
  std::map<int64_t, int64_t> slot_;
  bool copy_kernel_ = true;
  hipStream_t s_ = nullptr;
};

TORCH_LIBRARY_FRAGMENT(tfd, m) {
  m.class_<GpuPsShard>("GpuPsShard")
      .def(torch::init<int64_t, at::Tensor, int64_t, int64_t, int64_t, double, double, double, double, double, bool>())
      .def("numel", &GpuPsShard::numel)
      .def("updates", &GpuPsShard::updates)
      .def("params", &GpuPsShard::params)
      .def("slot_m", &GpuPsShard::slot_m)
      .def("slot_v", &GpuPsShard::slot_v)
      .def("mailbox", &GpuPsShard::mailbox)
      .def("open_worker", &GpuPsShard::open_worker)
      .def("pull_init", &GpuPsShard::pull_init)
      .def("load_state", &GpuPsShard::load_state)
      .def("apply", &GpuPsShard::apply)
      .def("accumulate", &GpuPsShard::accumulate)
      .def("apply_accumulated", &GpuPsShard::apply_accumulated)
      .def("push", &GpuPsShard::push)
      .def("set_copy_kernel", &GpuPsShard::set_copy_kernel);
  m.class_<GpuPsPort>("GpuPsPort")
      .def(torch::init<int64_t, int64_t>())
      .def("export_buffer", &GpuPsPort::export_buffer)
      .def("open_ps", &GpuPsPort::open_ps)
      .def("push_grad", &GpuPsPort::push_grad)
      .def("set_copy_kernel", &GpuPsPort::set_copy_kernel);
}

}  // namespace tfd
