// Peer-to-peer collectives over IPC-mapped staging buffers (see csrc/ipc_kernels.h):
// one-shot all-reduce, reduce-scatter and in-place all-gather.
//
// Protocol (per call, value v = this communicator's call counter + 1, identical on every rank
// because every rank issues the same collective sequence):
//   1. block b publishes its slice(s) into this rank's staging buffer, system-scope release;
//   2. START: block b stores v into start[b][r] of every peer and spins (time-bounded) until
//      every peer has stored v into our start[b][*] -- after which the peers' slice-b data is
//      visible (system-scope acquire);
//   3. the block reads slice b from every peer (remote reads over xGMI; fp32 accumulate in rank
//      order 0..N-1, so all ranks compute bit-identical sums) and writes its local output;
//   4. END: every block stores v into end[b][r] of every peer; block 0 then waits until ALL blocks
//      of ALL ranks have done so, and only then bumps the call counter and lets the kernel
//      complete. So no rank can start the next collective -- which may decompose the staging
//      buffer into different block slices -- while a peer still reads this one's staging bytes.
// Counters are monotonic (no reset), so captured hipGraphs replay freely. Every spin is bounded
// (sticky error word instead of a hung GPU).
#include "../common.h"
#include "../ipc_kernels.h"

#include <algorithm>

namespace tfd {
namespace {

constexpr int kErrWord = kIpcSigFlags + kIpcMaxBlocks;
constexpr int kCallWord = kErrWord + 1;

__device__ __forceinline__ int64_t now_ticks() { return (int64_t)__builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void flag_store(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int flag_load(int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int* flag_slot(const IpcAllReduceArgs& a, int rank_sig, int phase, int block, int from) {
  return a.sig[rank_sig] + (phase * kIpcMaxBlocks + block) * kIpcMaxRanks + from;
}
__device__ void set_error(const IpcAllReduceArgs& a) {
  __hip_atomic_store(a.sig[a.rank] + kErrWord, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Producer side (MI355X_MICROARCH.md, inter-workgroup visibility): every wave drains its own
// stores, workgroup barrier, ONE lane releases at system scope and drains again (the compiler may
// drop the fence's own wait), then publishes the flag to every rank.
__device__ __forceinline__ void publish(const IpcAllReduceArgs& a, int phase, int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int p = 0; p < a.world; ++p) flag_store(flag_slot(a, p, phase, blockIdx.x, a.rank), v);
  }
}

// START: wait for every peer's block b (one lane), then one system-scope acquire for the block
__device__ bool start_barrier(const IpcAllReduceArgs& a, int v) {
  __shared__ int ok;
  publish(a, 0, v);
  if (threadIdx.x == 0) {
    const int64_t t0 = now_ticks();
    int good = 1;
    for (int p = 0; p < a.world && good; ++p) {
      while (flag_load(flag_slot(a, a.rank, 0, blockIdx.x, p)) < v) {
        if (now_ticks() - t0 > a.spin_limit_ticks) { good = 0; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (!good) set_error(a);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ok = good;
  }
  __syncthreads();
  return ok != 0;
}

// END: publish; block 0 waits for every (block, rank) pair with 64 polling lanes, then bumps the
// call counter (every block read it before publishing START, so nobody sees the new value early)
__device__ void end_barrier(const IpcAllReduceArgs& a, int v) {
  publish(a, 1, v);
  if (blockIdx.x != 0) return;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x, pairs = (int)gridDim.x * a.world;
    const int64_t t0 = now_ticks();
    int good = 1;
    for (int i = lane; i < pairs && good; i += 64) {
      const int blk = i / a.world, p = i - blk * a.world;
      while (flag_load(flag_slot(a, a.rank, 1, blk, p)) < v) {
        if (now_ticks() - t0 > a.spin_limit_ticks) { good = 0; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (!good) set_error(a);
  }
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(a.sig[a.rank] + kCallWord, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ int call_value(const IpcAllReduceArgs& a) {
  return __hip_atomic_load(a.sig[a.rank] + kCallWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
}

__device__ __forceinline__ float load_in(const IpcAllReduceArgs& a, int64_t i) {
  return a.in_bf16 ? bf2f(reinterpret_cast<const uint16_t*>(a.in)[i]) : reinterpret_cast<const float*>(a.in)[i];
}
__device__ __forceinline__ void store_out(const IpcAllReduceArgs& a, int64_t i, float s) {
  if (a.out_bf16) reinterpret_cast<uint16_t*>(a.out)[i] = f2bf_bits(s);
  else reinterpret_cast<float*>(a.out)[i] = s;
}

__global__ __launch_bounds__(256) void ipc_allreduce_kernel(IpcAllReduceArgs a) {
  const int v = call_value(a);
  const int64_t chunk = ((a.n + gridDim.x - 1) / gridDim.x + 3) & ~(int64_t)3;
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(a.n, lo + chunk);
  float* my = reinterpret_cast<float*>(a.stage[a.rank]);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) my[i] = load_in(a, i);
  if (start_barrier(a, v)) {
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      float s = 0.f;
      for (int p = 0; p < a.world; ++p) s += reinterpret_cast<const float*>(a.stage[p])[i];
      store_out(a, i, s * a.scale);
    }
  }
  end_barrier(a, v);
}

// Reduce-scatter: block b publishes slice b of EVERY shard (the bytes block b of every rank will
// read), then sums slice b of its own shard from all ranks. in: N*S local elements, out: S.
__global__ __launch_bounds__(256) void ipc_reduce_scatter_kernel(IpcAllReduceArgs a) {
  const int v = call_value(a);
  const int64_t S = a.n;
  const int64_t chunk = ((S + gridDim.x - 1) / gridDim.x + 3) & ~(int64_t)3;
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(S, lo + chunk);
  float* my = reinterpret_cast<float*>(a.stage[a.rank]);
  for (int q = 0; q < a.world; ++q)
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) my[q * S + i] = load_in(a, q * S + i);
  if (start_barrier(a, v)) {
    const int64_t base = (int64_t)a.rank * S;
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      float s = 0.f;
      for (int p = 0; p < a.world; ++p) s += reinterpret_cast<const float*>(a.stage[p])[base + i];
      store_out(a, i, s * a.scale);
    }
  }
  end_barrier(a, v);
}

// All-gather in place: buf holds N*S elements (2- or 4-byte raw), this rank's shard at r*S.
template <typename T>
__global__ __launch_bounds__(256) void ipc_all_gather_kernel(IpcAllReduceArgs a) {
  const int v = call_value(a);
  const int64_t S = a.n;
  const int64_t chunk = ((S + gridDim.x - 1) / gridDim.x + 7) & ~(int64_t)7;
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(S, lo + chunk);
  T* buf = reinterpret_cast<T*>(a.out);
  T* my = reinterpret_cast<T*>(a.stage[a.rank]);
  const int64_t own = (int64_t)a.rank * S;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) my[i] = buf[own + i];
  if (start_barrier(a, v)) {
    for (int p = 0; p < a.world; ++p) {
      if (p == a.rank) continue;
      const T* src = reinterpret_cast<const T*>(a.stage[p]);
      for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) buf[(int64_t)p * S + i] = src[i];
    }
  }
  end_barrier(a, v);
}

inline int clamp_blocks(int b) { return std::max(1, std::min(b, kIpcMaxBlocks)); }

}  // namespace

void ipc_allreduce(const IpcAllReduceArgs& a, int blocks, hipStream_t s) {
  ipc_allreduce_kernel<<<clamp_blocks(blocks), 256, 0, s>>>(a);
}
void ipc_reduce_scatter(const IpcAllReduceArgs& a, int blocks, hipStream_t s) {
  ipc_reduce_scatter_kernel<<<clamp_blocks(blocks), 256, 0, s>>>(a);
}
void ipc_all_gather(const IpcAllReduceArgs& a, int elem_bytes, int blocks, hipStream_t s) {
  if (elem_bytes == 2) ipc_all_gather_kernel<uint16_t><<<clamp_blocks(blocks), 256, 0, s>>>(a);
  else ipc_all_gather_kernel<float><<<clamp_blocks(blocks), 256, 0, s>>>(a);
}

}  // namespace tfd
