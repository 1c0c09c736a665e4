#include "comm.h"

#include <c10/hip/HIPStream.h>
#include <c10/util/Exception.h>
#include <cstring>
#include <mutex>
#include <vector>

namespace tfd {

void rccl_check(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, "RCCL ", what, " failed: ", ncclGetErrorString(r));
}

ncclDataType_t rccl_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "RcclComm: unsupported dtype ", t.scalar_type());
  }
}

ncclRedOp_t rccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "avg" || op == "mean") return ncclAvg;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  TORCH_CHECK(false, "RcclComm: unknown reduce op ", op);
}

at::Tensor RcclComm::unique_id() {
  ncclUniqueId id;
  rccl_check(ncclGetUniqueId(&id), "GetUniqueId");
  auto t = at::empty({NCCL_UNIQUE_ID_BYTES}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &id, NCCL_UNIQUE_ID_BYTES);
  return t;
}

namespace {
std::mutex g_retired_mu;
std::vector<ncclComm_t>& retired() {
  static auto* v = new std::vector<ncclComm_t>();  // intentionally never destroyed (exit order)
  return *v;
}
thread_local bool t_user_object_thread = false;
// HIP user-object destructor: a captured graph that held a reference is gone
void release_graph_ref(void* p) {
  t_user_object_thread = true;
  delete static_cast<std::shared_ptr<CommHandle>*>(p);
  t_user_object_thread = false;
}
}  // namespace

// A collective captured into a hipGraph stays tied to its communicator until that graph is destroyed,
// and Python frees a job's objects in no fixed order (a test's locals, a model rebuilt between
// bucket-size probes): a communicator destroyed before a graph that captured it left that graph's
// replay / teardown on freed resources -- round 3's in-suite segfault in CUDAGraph.replay
// (profiles/pytest_gpu_r3_segv.log). So the handle is reference-counted: the RcclComm holds one
// reference and every capture that issues a collective hands one to its graph as a HIP user object
// (hipUserObjectCreate + hipGraphRetainUserObject; the instantiated graph keeps its graph's user
// objects). The last holder destroys the communicator -- on the caller's thread directly, or, when
// the last holder was a graph released on HIP's user-object thread (where no HIP/RCCL call is allowed),
// through the retired list that the next constructor, destructor or reap() drains.
CommHandle::~CommHandle() {
  if (!comm) return;
  if (t_user_object_thread) {
    std::lock_guard<std::mutex> g(g_retired_mu);
    retired().push_back(comm);
  } else {
    ncclCommDestroy(comm);
  }
}

RcclComm::RcclComm(const at::Tensor& uid, int64_t world, int64_t rank, int64_t device)
    : world_(world), rank_(rank), device_(device) {
  TORCH_CHECK(uid.numel() == NCCL_UNIQUE_ID_BYTES && uid.scalar_type() == at::kByte, "bad unique id");
  reap();
  ncclUniqueId id;
  auto c = uid.contiguous().cpu();
  std::memcpy(&id, c.data_ptr(), NCCL_UNIQUE_ID_BYTES);
  TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "hipSetDevice failed");
  h_ = std::make_shared<CommHandle>();
  rccl_check(ncclCommInitRank(&h_->comm, (int)world, id, (int)rank), "CommInitRank");
}

RcclComm::~RcclComm() {
  h_.reset();  // destroys the communicator now unless a live captured graph still holds it
  reap();
}

int64_t RcclComm::graph_refs() const { return h_ ? (int64_t)h_.use_count() - 1 : 0; }

int64_t RcclComm::reap() {
  std::vector<ncclComm_t> v;
  {
    std::lock_guard<std::mutex> g(g_retired_mu);
    v.swap(retired());
  }
  for (auto c : v) ncclCommDestroy(c);
  return (int64_t)v.size();
}

int64_t RcclComm::retired_count() {
  std::lock_guard<std::mutex> g(g_retired_mu);
  return (int64_t)retired().size();
}

void RcclComm::abort() {
  if (h_ && h_->comm) {
    ncclCommAbort(h_->comm);
    h_->comm = nullptr;
  }
}

ncclComm_t RcclComm::live(hipStream_t s) {
  TORCH_CHECK(h_ && h_->comm, "communicator aborted");
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  TORCH_CHECK(hipStreamGetCaptureInfo_v2(s, &st, &id, &g, nullptr, nullptr) == hipSuccess, "capture info");
  if (st == hipStreamCaptureStatusActive && g) {
    auto* ref = new std::shared_ptr<CommHandle>(h_);
    hipUserObject_t obj = nullptr;
    if (hipUserObjectCreate(&obj, ref, release_graph_ref, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
      delete ref;
      TORCH_CHECK(false, "hipUserObjectCreate failed");
    }
    TORCH_CHECK(hipGraphRetainUserObject(g, obj, 1, hipGraphUserObjectMove) == hipSuccess,
                "hipGraphRetainUserObject failed");
  }
  return h_->comm;
}

static hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void RcclComm::all_reduce_raw(void* buf, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t s) {
  rccl_check(ncclAllReduce(buf, buf, count, dt, op, live(s), s), "AllReduce");
}
void RcclComm::reduce_scatter_raw(const void* in, void* out, size_t recvcount, ncclDataType_t dt, ncclRedOp_t op,
                                  hipStream_t s) {
  rccl_check(ncclReduceScatter(in, out, recvcount, dt, op, live(s), s), "ReduceScatter");
}
void RcclComm::all_gather_raw(const void* in, void* out, size_t sendcount, ncclDataType_t dt, hipStream_t s) {
  rccl_check(ncclAllGather(in, out, sendcount, dt, live(s), s), "AllGather");
}

void RcclComm::all_reduce(const at::Tensor& t, const std::string& op) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "all_reduce: contiguous GPU tensor required");
  all_reduce_raw(t.data_ptr(), t.numel(), rccl_dtype(t), rccl_op(op), cur_stream());
}
void RcclComm::reduce_scatter(const at::Tensor& in, const at::Tensor& out, const std::string& op) {
  TORCH_CHECK(in.numel() == out.numel() * world_, "reduce_scatter: size mismatch");
  reduce_scatter_raw(in.data_ptr(), out.data_ptr(), out.numel(), rccl_dtype(in), rccl_op(op), cur_stream());
}
void RcclComm::all_gather(const at::Tensor& in, const at::Tensor& out) {
  TORCH_CHECK(out.numel() == in.numel() * world_, "all_gather: size mismatch");
  all_gather_raw(in.data_ptr(), out.data_ptr(), in.numel(), rccl_dtype(in), cur_stream());
}
void RcclComm::broadcast(const at::Tensor& t, int64_t root) {
  hipStream_t s = cur_stream();
  rccl_check(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), rccl_dtype(t), (int)root, live(s), s), "Broadcast");
}
void RcclComm::send(const at::Tensor& t, int64_t peer) {
  hipStream_t s = cur_stream();
  rccl_check(ncclSend(t.data_ptr(), t.numel(), rccl_dtype(t), (int)peer, live(s), s), "Send");
}
void RcclComm::recv(const at::Tensor& t, int64_t peer) {
  hipStream_t s = cur_stream();
  rccl_check(ncclRecv(t.data_ptr(), t.numel(), rccl_dtype(t), (int)peer, live(s), s), "Recv");
}

}  // namespace tfd
