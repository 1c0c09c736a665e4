// One-shot peer-to-peer all-reduce over IPC-mapped staging buffers (see csrc/ipc_kernels.h).
//
// Block b of rank r owns the element slice S_b. Per call:
//   1. copy S_b of the local input into stage[r] (fp32), system-scope release;
//   2. START barrier: store epoch into sig[p][START][b][r] of every peer p, spin (bounded) until
//      every peer has stored it into our sig[r][START][b][*];
//   3. reduce S_b from all `world` staging buffers (remote reads; fp32 accumulate, rank order
//      0..world-1 on every rank so all ranks compute bit-identical sums) -> out;
//   4. END barrier (same protocol, other phase) so nobody rewrites its staging while peers read.
// Epochs are per block and monotonic (kept in the local signal region), so no reset is needed and
// the whole thing replays from a captured hipGraph. Signal memory is uncached (fine-grained) so
// polls see remote stores; staging reads happen after a system-scope acquire.
#include "../common.h"
#include "../ipc_kernels.h"

namespace tfd {
namespace {

__device__ __forceinline__ int64_t now_ticks() { return (int64_t)__builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void flag_store(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int flag_load(int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one lane does the cross-rank handshake for the whole block; returns false on timeout
__device__ bool block_barrier(const IpcAllReduceArgs& a, int phase, int epoch) {
  __shared__ int ok;
  // producer side (MI355X_MICROARCH.md, inter-workgroup visibility): every wave drains its own
  // stores, barrier, ONE lane releases at system scope, drains again (the compiler may drop the
  // fence's own wait), then publishes the flags.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int slot = (phase * kIpcMaxBlocks + (int)blockIdx.x) * kIpcMaxRanks + a.rank;
    for (int p = 0; p < a.world; ++p) flag_store(a.sig[p] + slot, epoch);
    int* mine = a.sig[a.rank] + (phase * kIpcMaxBlocks + (int)blockIdx.x) * kIpcMaxRanks;
    const int64_t t0 = now_ticks();
    int good = 1;
    for (int p = 0; p < a.world && good; ++p) {
      while (flag_load(mine + p) < epoch) {
        if (now_ticks() - t0 > a.spin_limit_ticks) { good = 0; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (!good) __hip_atomic_store(a.sig[a.rank] + kIpcSigFlags + kIpcMaxBlocks, 1, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
    // consumer side: one acquire (invalidates this CU's caches), drained before the barrier
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ok = good;
  }
  __syncthreads();
  return ok != 0;
}

__device__ __forceinline__ float load_in(const IpcAllReduceArgs& a, int64_t i) {
  return a.in_bf16 ? bf2f(reinterpret_cast<const uint16_t*>(a.in)[i]) : reinterpret_cast<const float*>(a.in)[i];
}

__global__ __launch_bounds__(256) void ipc_allreduce_kernel(IpcAllReduceArgs a) {
  const int64_t chunk = ((a.n + gridDim.x - 1) / gridDim.x + 3) & ~(int64_t)3;
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(a.n, lo + chunk);
  int* ep = a.sig[a.rank] + kIpcSigFlags + blockIdx.x;
  const int epoch = *ep + 1;  // only this block touches its epoch word
  float* my = reinterpret_cast<float*>(a.stage[a.rank]);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) my[i] = load_in(a, i);
  if (!block_barrier(a, 0, epoch)) return;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    float s = 0.f;
    for (int p = 0; p < a.world; ++p) s += reinterpret_cast<const float*>(a.stage[p])[i];
    s *= a.scale;
    if (a.out_bf16) reinterpret_cast<uint16_t*>(a.out)[i] = f2bf_bits(s);
    else reinterpret_cast<float*>(a.out)[i] = s;
  }
  block_barrier(a, 1, epoch);
  if (threadIdx.x == 0) *ep = epoch;
}

}  // namespace

void ipc_allreduce(const IpcAllReduceArgs& a, int blocks, hipStream_t s) {
  if (blocks < 1) blocks = 1;
  if (blocks > kIpcMaxBlocks) blocks = kIpcMaxBlocks;
  ipc_allreduce_kernel<<<blocks, 256, 0, s>>>(a);
}

}  // namespace tfd
