// IpcComm class declaration (see ipc_comm.cpp).
#pragma once
#include <ATen/ATen.h>
#include <hip/hip_runtime_api.h>
#include <torch/custom_class.h>

namespace tfd {

class IpcComm : public torch::CustomClassHolder {
 public:
  IpcComm(int64_t world, int64_t rank, int64_t device, int64_t capacity_elems);
  ~IpcComm() override;
  at::Tensor handle();                       // this rank's [128] uint8 export (staging + signals)
  void open(const at::Tensor& all_handles);  // [world, 128]: open every peer's export
  void close();
  void all_reduce(const at::Tensor& t, double scale);  // in place, current HIP stream
  // out = scale * sum over ranks of in (fp32 / bf16 each, same numel; the staging keeps in's format):
  // e.g. fp32 gradients in, the bf16 sums out -- the wire cast fused into the collective
  void all_reduce_into(const at::Tensor& in, const at::Tensor& out, double scale);
  // in: fp32/bf16 -> fp32 staging -> reduced sum * scale -> out (fp32/bf16); n <= capacity
  void all_reduce_raw(const void* in, bool in_bf16, void* out, bool out_bf16, int64_t n, double scale,
                      hipStream_t s);
  // reduce-scatter of N*S elements (fp32/bf16 in) into this rank's S-element shard (fp32/bf16 out)
  void reduce_scatter_raw(const void* in, bool in_bf16, void* out, bool out_bf16, int64_t shard, double scale,
                          hipStream_t s);
  // in-place all-gather of N*S elements (2- or 4-byte) with this rank's shard at rank*S
  void all_gather_raw(void* buf, int elem_bytes, int64_t shard, hipStream_t s);
  void reduce_scatter(const at::Tensor& in, const at::Tensor& out, double scale);
  void all_gather(const at::Tensor& buf);
  int64_t error();                           // 1 once a barrier timed out (sticky)
  void set_spin_limit_ms(double ms);
  void set_max_blocks(int64_t b);          // grid cap of the spinning collectives
  int blocks(int64_t n) const;
  int64_t world() const { return world_; }
  int64_t rank() const { return rank_; }
  int64_t capacity() const { return cap_; }

 private:
  // Every collective of one IpcComm shares the staging halves and the call counter, so they must
  // execute one after another. order() makes a launch on a stream other than the previous
  // launch's wait for that launch (an event recorded after it); mark() records that event. Under
  // hipGraph capture the caller's capture order is the execution order (the engine captures all
  // of its collectives on one comm stream), so nothing is recorded there.
  void order(hipStream_t s);
  void mark(hipStream_t s);
  hipEvent_t last_ev_ = nullptr;
  hipStream_t last_stream_ = nullptr;
  bool last_recorded_ = false;
  int64_t world_, rank_, device_, cap_;
  void* stage_ = nullptr;
  void* sig_ = nullptr;
  void* peer_stage_[8];
  int* peer_sig_[8];
  bool opened_ = false;
  int64_t spin_ticks_ = 200000000;  // 2 s at 100 MHz
  int max_blocks_ = 64;
};

}  // namespace tfd
