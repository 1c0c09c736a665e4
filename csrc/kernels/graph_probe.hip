// Kernels of the captured-memset probe (csrc/runtime/graph_probe.cpp): an atomic "+1" over a buffer
// (the shape of the split-K accumulation that follows a zero fill) and a plain fill.
#include "../common.h"

namespace tfd {
namespace {
__global__ __launch_bounds__(256) void probe_add_one_kernel(float* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    atomicAdd(p + i, 1.f);
}
__global__ __launch_bounds__(256) void probe_fill_kernel(float* __restrict__ p, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}
int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 255) / 256)); }
}  // namespace

void probe_add_one(float* p, int64_t n, hipStream_t s) { probe_add_one_kernel<<<grid_for(n), 256, 0, s>>>(p, n); }
void probe_fill(float* p, int64_t n, float v, hipStream_t s) { probe_fill_kernel<<<grid_for(n), 256, 0, s>>>(p, n, v); }
}  // namespace tfd
