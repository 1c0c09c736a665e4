// Native RCCL communicator (one process per GPU; xGMI transport chosen by RCCL).
//
// Replaces the reference's gRPC Send/Recv between worker and PS graph partitions
// (/root/reference/mnist_python_m.py:152-177, 216-233): gradients are averaged with a bucketed
// all-reduce / reduce-scatter on a dedicated comm stream, params are broadcast from the chief at
// init, and send/recv carry the async-PS protocol. Collectives are issued straight from C++ so
// they can sit inside a captured hipGraph next to the compute kernels (one replay per step).
#pragma once
#include <memory>
#include <ATen/ATen.h>
#include <torch/custom_class.h>
#include <rccl/rccl.h>
#include <string>

namespace tfd {

void rccl_check(ncclResult_t r, const char* what);

// The communicator itself, shared by its RcclComm and by every captured graph whose collectives use
// it (a reference per capture, held by a HIP user object of the graph): it is destroyed when the last
// holder lets go -- the Python object or the last graph, in whichever order they go.
struct CommHandle {
  ncclComm_t comm = nullptr;
  ~CommHandle();
};

class RcclComm : public torch::CustomClassHolder {
 public:
  // uid: 128-byte ncclUniqueId produced by unique_id() on rank 0 and distributed via the store.
  RcclComm(const at::Tensor& uid, int64_t world, int64_t rank, int64_t device);
  ~RcclComm() override;  // drops this object's reference (see comm.cpp)
  static at::Tensor unique_id();
  // destroy the communicators whose last reference was dropped on HIP's user-object thread (no HIP or
  // RCCL calls are allowed there); also run by every constructor / destructor
  static int64_t reap();
  static int64_t retired_count();
  // number of captured graphs (user objects) that currently hold this communicator
  int64_t graph_refs() const;

  int64_t world() const { return world_; }
  int64_t rank() const { return rank_; }

  // Tensor-level collectives on the current HIP stream (in place where it makes sense).
  void all_reduce(const at::Tensor& t, const std::string& op);
  void reduce_scatter(const at::Tensor& in, const at::Tensor& out, const std::string& op);
  void all_gather(const at::Tensor& in, const at::Tensor& out);
  void broadcast(const at::Tensor& t, int64_t root);
  void send(const at::Tensor& t, int64_t peer);
  void recv(const at::Tensor& t, int64_t peer);
  void abort();

  // Raw-pointer forms used by the C++ engines.
  void all_reduce_raw(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s);
  void reduce_scatter_raw(const void* in, void* out, size_t recvcount, ncclDataType_t dt, ncclRedOp_t op,
                          hipStream_t s);
  void all_gather_raw(const void* in, void* out, size_t sendcount, ncclDataType_t dt, hipStream_t s);
  ncclComm_t handle() const { return h_ ? h_->comm : nullptr; }

 private:
  ncclComm_t live(hipStream_t s);  // the handle for a collective on s (a capture takes a reference)
  std::shared_ptr<CommHandle> h_;
  int64_t world_, rank_, device_;
};

ncclDataType_t rccl_dtype(const at::Tensor& t);
ncclRedOp_t rccl_op(const std::string& op);

}  // namespace tfd
