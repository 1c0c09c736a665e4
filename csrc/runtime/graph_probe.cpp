// Captured hipMemsetAsync probe: does a hipMemsetAsync issued into a stream
// capture clear its buffer on every replay of the instantiated graph?
//
// The symptom it chases: ResNet's split-K weight-gradient accumulator was zeroed by hipMemsetAsync on
// the capturing stream, then accumulated with atomics; on graph replays the stem gradient grew to
// inf, as if the clear did not run (tools/debug/stem_mode_check.py). The engine now clears with a
// kernel (conv_nhwc.hip zero_f32). This probe captures the same pattern in isolation --
//     +1 (atomics)  ->  clear  ->  +1 (atomics)      (capture_mode bit 2: clear -> +1, the clear a root node)
// -- on a caller-given buffer (so a 4-B aligned view of a flat buffer can be tested against a
// 256-B aligned one), instantiates and replays it, and reports the graph's nodes (type, the memset
// node's parameters and dependency count) and the buffer after the replays (every element must be
// 1.0 if the clear ran on each replay; 1 + 2 x replays ... if it never did).
#include <hip/hip_runtime.h>

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

namespace tfd {
void probe_add_one(float* p, int64_t n, hipStream_t s);
void probe_fill(float* p, int64_t n, float v, hipStream_t s);

namespace {
#define GP_OK(x)                                                                            \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    TORCH_CHECK(e_ == hipSuccess, #x, " failed: ", hipGetErrorString(e_));                  \
  } while (0)

// info layout (int64): [0] nodes, [1] kernel nodes, [2] memset nodes, [3] other nodes,
// [4] memset dst - buffer (bytes), [5] memset elementSize, [6] memset width, [7] memset height,
// [8] memset value, [9] memset node dependency count, [10] elements != 1.0 after the replays,
// [11] buffer[0] bit pattern as float*1000, [12] buffer[n-1] * 1000, [13] memset nodes total width*elem
at::Tensor memset_capture_probe(at::Tensor buf, int64_t replays, int64_t clear_mode, int64_t capture_mode) {
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kFloat && buf.is_contiguous(), "fp32 contiguous GPU buffer");
  const int64_t n = buf.numel();
  float* p = (float*)buf.data_ptr();
  hipStream_t s;
  GP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  probe_fill(p, n, 5.f, s);
  GP_OK(hipStreamSynchronize(s));
  const int cm = (int)(capture_mode & 3);
  const hipStreamCaptureMode mode = cm == 0 ? hipStreamCaptureModeGlobal
                                    : cm == 1 ? hipStreamCaptureModeThreadLocal
                                              : hipStreamCaptureModeRelaxed;
  hipGraph_t g = nullptr;
  GP_OK(hipStreamBeginCapture(s, mode));
  if (!(capture_mode & 4)) probe_add_one(p, n, s);  // bit 2: the clear is the graph's root node
  if (clear_mode == 0) GP_OK(hipMemsetAsync(p, 0, n * sizeof(float), s));
  else if (clear_mode == 1) GP_OK(hipMemsetD32Async((hipDeviceptr_t)p, 0, (size_t)n, s));
  else probe_fill(p, n, 0.f, s);
  probe_add_one(p, n, s);
  GP_OK(hipStreamEndCapture(s, &g));
  std::vector<int64_t> info(14, 0);
  size_t nn = 0;
  GP_OK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  GP_OK(hipGraphGetNodes(g, nodes.data(), &nn));
  info[0] = (int64_t)nn;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    GP_OK(hipGraphNodeGetType(nd, &t));
    if (t == hipGraphNodeTypeKernel) {
      info[1]++;
    } else if (t == hipGraphNodeTypeMemset) {
      info[2]++;
      hipMemsetParams prm{};
      GP_OK(hipGraphMemsetNodeGetParams(nd, &prm));
      info[4] = (int64_t)((char*)prm.dst - (char*)p);
      info[5] = prm.elementSize;
      info[6] = (int64_t)prm.width;
      info[7] = (int64_t)prm.height;
      info[8] = prm.value;
      info[13] += (int64_t)prm.width * prm.elementSize * std::max<int64_t>(1, (int64_t)prm.height);
      size_t nd_deps = 0;
      GP_OK(hipGraphNodeGetDependencies(nd, nullptr, &nd_deps));
      info[9] = (int64_t)nd_deps;
    } else {
      info[3]++;
    }
  }
  hipGraphExec_t ge = nullptr;
  GP_OK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int64_t r = 0; r < replays; ++r) GP_OK(hipGraphLaunch(ge, s));
  GP_OK(hipStreamSynchronize(s));
  std::vector<float> h(n);
  GP_OK(hipMemcpy(h.data(), p, n * sizeof(float), hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < n; ++i) info[10] += h[i] != 1.f;
  info[11] = (int64_t)(h[0] * 1000.f);
  info[12] = (int64_t)(h[n - 1] * 1000.f);
  GP_OK(hipGraphExecDestroy(ge));
  GP_OK(hipGraphDestroy(g));
  GP_OK(hipStreamDestroy(s));
  return at::tensor(info, at::TensorOptions().dtype(at::kLong));
}

// The memset nodes of a captured graph (torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph()): one row
// per node [dst, elementSize, width, height, value, dependency count, dependent count]; row 0 holds the
// graph's node count and kernel-node count.
at::Tensor graph_memset_nodes(int64_t graph) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
  size_t nn = 0;
  GP_OK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  GP_OK(hipGraphGetNodes(g, nodes.data(), &nn));
  std::vector<int64_t> rows(7, 0);
  rows[0] = (int64_t)nn;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    GP_OK(hipGraphNodeGetType(nd, &t));
    if (t == hipGraphNodeTypeKernel) rows[1]++;
    if (t != hipGraphNodeTypeMemset) continue;
    hipMemsetParams prm{};
    GP_OK(hipGraphMemsetNodeGetParams(nd, &prm));
    size_t deps = 0, outs = 0;
    GP_OK(hipGraphNodeGetDependencies(nd, nullptr, &deps));
    GP_OK(hipGraphNodeGetDependentNodes(nd, nullptr, &outs));
    const int64_t r[7] = {(int64_t)(uintptr_t)prm.dst, prm.elementSize, (int64_t)prm.width, (int64_t)prm.height,
                          prm.value, (int64_t)deps, (int64_t)outs};
    rows.insert(rows.end(), r, r + 7);
  }
  return at::tensor(rows, at::TensorOptions().dtype(at::kLong)).view({-1, 7});
}

// Node count of a captured graph per hipGraphNodeType (index = the enum value: 0 kernel, 1 memcpy,
// 2 memset, 3 host, 4 child graph, 5 empty, 6 wait event, 7 event record, ...).
at::Tensor graph_node_types(int64_t graph) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
  size_t nn = 0;
  GP_OK(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  GP_OK(hipGraphGetNodes(g, nodes.data(), &nn));
  std::vector<int64_t> counts(16, 0);
  for (auto nd : nodes) {
    hipGraphNodeType t;
    GP_OK(hipGraphNodeGetType(nd, &t));
    counts[std::min<int>((int)t, 15)]++;
  }
  return at::tensor(counts, at::TensorOptions().dtype(at::kLong));
}

// hipMemsetAsync on the caller's current stream (inside a torch.cuda.graph capture: the path the
// ResNet wgrad took before the fill kernel replaced it)
void memset_zero_async(at::Tensor buf) {
  TORCH_CHECK(buf.is_cuda() && buf.is_contiguous(), "contiguous GPU buffer");
  GP_OK(hipMemsetAsync(buf.data_ptr(), 0, buf.nbytes(), c10::hip::getCurrentHIPStream().stream()));
}
void atomic_add_one(at::Tensor buf) {
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kFloat && buf.is_contiguous(), "fp32 contiguous GPU buffer");
  probe_add_one((float*)buf.data_ptr(), buf.numel(), c10::hip::getCurrentHIPStream().stream());
}
}  // namespace

TORCH_LIBRARY_FRAGMENT(tfd, m) {
  m.def("memset_capture_probe(Tensor buf, int replays, int clear_mode, int capture_mode) -> Tensor",
        &memset_capture_probe);
  m.def("graph_memset_nodes(int graph) -> Tensor", &graph_memset_nodes);
  m.def("graph_node_types(int graph) -> Tensor", &graph_node_types);
  m.def("memset_zero_async(Tensor(a!) buf) -> ()");
  m.impl("memset_zero_async", c10::DispatchKey::CUDA, &memset_zero_async);
  m.def("probe_atomic_add_one(Tensor(a!) buf) -> ()");
  m.impl("probe_atomic_add_one", c10::DispatchKey::CUDA, &atomic_add_one);
}
}  // namespace tfd
