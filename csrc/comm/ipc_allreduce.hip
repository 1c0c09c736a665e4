// Peer-to-peer collectives over IPC-mapped staging buffers (see csrc/ipc_kernels.h):
// one-shot all-reduce, reduce-scatter and in-place all-gather, shaped for xGMI's point-to-point
// links: every rank reads its reduce slice from ALL peers at once, 16 B per lane per peer, with
// the peer loop unrolled by a compile-time world size so the W remote loads of a lane are all in
// flight before the first add.
//
// Protocol (per call; v = this communicator's call counter + 1, identical on every rank because
// every rank issues the same collective sequence):
//   1. block b copies its slice(s) into this rank's staging half (v & 1) in the wire dtype (bf16
//      stays bf16: half the xGMI bytes), then a system-scope release;
//   2. START: block b stores v into flag[b][r] of every peer and spins (time-bounded) until every
//      peer has stored >= v into our flag[b][*]; then a system-scope acquire;
//   3. the block reads slice b from every peer (remote 16-B loads over xGMI), accumulates in fp32
//      in rank order 0..W-1 (every rank computes bit-identical sums) and writes its local output;
//   4. the last block to finish (a device-scope arrival ticket) bumps the call counter.
// Double-buffered staging replaces an END barrier: a peer's START flag for call v+1 is published
// only after its whole call-v kernel has completed (same stream), so once a rank has passed
// START(v+1) every peer is done reading its call-v half, and call v+2 may overwrite it; no rank
// can run more than one call ahead of any peer. Counters are monotonic (no reset), so captured
// hipGraphs replay freely. Every spin is time-bounded: a missing peer sets a sticky error word
// (IpcComm::error(), checked by the trainers) instead of hanging the GPU.
#include "../common.h"
#include "../ipc_kernels.h"

#include <algorithm>

namespace tfd {
namespace {

constexpr int kErrWord = kIpcSigFlags;
constexpr int kCallWord = kIpcSigFlags + 1;
constexpr int kTicketWord = kIpcSigFlags + 2;
constexpr int kThreads = 256;
constexpr int kVec = 8;  // elements per lane per iteration (16 B of bf16, 32 B of fp32)

__device__ __forceinline__ int64_t now_ticks() { return (int64_t)__builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void flag_store(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int flag_load(int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int* flag_slot(const IpcAllReduceArgs& a, int rank_sig, int block, int from) {
  return a.sig[rank_sig] + block * kIpcMaxRanks + from;
}
__device__ void set_error(const IpcAllReduceArgs& a) {
  __hip_atomic_store(a.sig[a.rank] + kErrWord, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int call_value(const IpcAllReduceArgs& a) {
  return __hip_atomic_load(a.sig[a.rank] + kCallWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
}

// START: drain this block's staging stores, release at system scope, publish v to every rank,
// then one lane per peer (lanes 0..W-1 poll in parallel) waits for the peers' flags.
template <int W>
__device__ bool start_barrier(const IpcAllReduceArgs& a, int v) {
  __shared__ int ok;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) ok = 1;
  if (threadIdx.x < W) {
    const int p = threadIdx.x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    flag_store(flag_slot(a, p, blockIdx.x, a.rank), v);
    const int64_t t0 = now_ticks();
    int good = 1;
    while (flag_load(flag_slot(a, a.rank, blockIdx.x, p)) < v) {
      if (now_ticks() - t0 > a.spin_limit_ticks) { good = 0; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!good) {
      set_error(a);
      ok = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return ok != 0;
}

// the last block to arrive bumps the call counter (every block read it at its start)
__device__ void finish(const IpcAllReduceArgs& a) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(a.sig[a.rank] + kTicketWord, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (int)gridDim.x - 1) {
      __hip_atomic_store(a.sig[a.rank] + kTicketWord, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(a.sig[a.rank] + kCallWord, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// 8 elements <-> fp32 registers
struct V8 {
  float f[kVec];
};
__device__ __forceinline__ V8 load8(const void* base, bool bf, int64_t i) {
  V8 r;
  if (bf) {
    const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(base) + i);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r.f[2 * j] = __uint_as_float(w[j] << 16);
      r.f[2 * j + 1] = __uint_as_float(w[j] & 0xFFFF0000u);
    }
  } else {
    const f32x4 x0 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(base) + i);
    const f32x4 x1 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(base) + i + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r.f[j] = x0[j];
      r.f[4 + j] = x1[j];
    }
  }
  return r;
}
__device__ __forceinline__ void store8(void* base, bool bf, int64_t i, const V8& r) {
  if (bf) {
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(base) + i) =
        make_uint4(pack_bf2(r.f[0], r.f[1]), pack_bf2(r.f[2], r.f[3]), pack_bf2(r.f[4], r.f[5]), pack_bf2(r.f[6], r.f[7]));
  } else {
    float* p = reinterpret_cast<float*>(base) + i;
    *reinterpret_cast<f32x4*>(p) = f32x4{r.f[0], r.f[1], r.f[2], r.f[3]};
    *reinterpret_cast<f32x4*>(p + 4) = f32x4{r.f[4], r.f[5], r.f[6], r.f[7]};
  }
}
// raw 16-B or 32-B copy (staging keeps the input's dtype)
__device__ __forceinline__ void copy8(void* dst, const void* src, bool bf, int64_t i) {
  if (bf) {
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(dst) + i) =
        *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(src) + i);
  } else {
    const f32x4 x0 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(src) + i);
    const f32x4 x1 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(src) + i + 4);
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(dst) + i) = x0;
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(dst) + i + 4) = x1;
  }
}
__device__ __forceinline__ void* stage_half(const IpcAllReduceArgs& a, int p, int v) {
  return reinterpret_cast<char*>(a.stage[p]) + (size_t)(v & 1) * a.half_bytes;
}

// sum over the W peers' staging (rank order), 16 B loads of all peers issued before the adds
template <int W>
__device__ __forceinline__ V8 peer_sum(const IpcAllReduceArgs& a, int v, bool bf, int64_t i) {
  V8 x[W];
#pragma unroll
  for (int p = 0; p < W; ++p) x[p] = load8(stage_half(a, p, v), bf, i);
  V8 s = x[0];
#pragma unroll
  for (int p = 1; p < W; ++p)
#pragma unroll
    for (int j = 0; j < kVec; ++j) s.f[j] += x[p].f[j];
  return s;
}

// chunk of block b: multiples of kVec elements (n % kVec == 0 is required by the host)
__device__ __forceinline__ void block_range(int64_t n, int64_t& lo, int64_t& hi) {
  const int64_t chunk = ((n + gridDim.x - 1) / gridDim.x + kVec - 1) / kVec * kVec;
  lo = (int64_t)blockIdx.x * chunk;
  hi = min(n, lo + chunk);
}

__device__ __forceinline__ float load1(const void* base, bool bf, int64_t i) {
  return bf ? bf2f(reinterpret_cast<const uint16_t*>(base)[i]) : reinterpret_cast<const float*>(base)[i];
}

template <int W>
__global__ __launch_bounds__(kThreads) void ipc_allreduce_kernel(IpcAllReduceArgs a) {
  const int v = call_value(a);
  const int64_t n8 = a.n & ~(int64_t)(kVec - 1);
  int64_t lo, hi;
  block_range(n8, lo, hi);
  const bool ib = a.in_bf16, ob = a.out_bf16;
  // the < 8 tail elements belong to the last block (scalar)
  const bool tail = blockIdx.x == gridDim.x - 1 && threadIdx.x < a.n - n8;
  const int64_t it = n8 + threadIdx.x;
  void* my = stage_half(a, a.rank, v);
  for (int64_t i = lo + (int64_t)threadIdx.x * kVec; i < hi; i += kThreads * kVec) copy8(my, a.in, ib, i);
  if (tail) {
    if (ib) reinterpret_cast<uint16_t*>(my)[it] = reinterpret_cast<const uint16_t*>(a.in)[it];
    else reinterpret_cast<float*>(my)[it] = reinterpret_cast<const float*>(a.in)[it];
  }
  if (start_barrier<W>(a, v)) {
    for (int64_t i = lo + (int64_t)threadIdx.x * kVec; i < hi; i += kThreads * kVec) {
      V8 s = peer_sum<W>(a, v, ib, i);
#pragma unroll
      for (int j = 0; j < kVec; ++j) s.f[j] *= a.scale;
      store8(a.out, ob, i, s);
    }
    if (tail) {
      float s = 0.f;
#pragma unroll
      for (int p = 0; p < W; ++p) s += load1(stage_half(a, p, v), ib, it);
      s *= a.scale;
      if (ob) reinterpret_cast<uint16_t*>(a.out)[it] = f2bf_bits(s);
      else reinterpret_cast<float*>(a.out)[it] = s;
    }
  }
  finish(a);
}

// Reduce-scatter: block b publishes slice b of EVERY shard (the bytes block b of every rank will
// read), then sums slice b of its own shard from all ranks. in: W*S local elements, out: S.
template <int W>
__global__ __launch_bounds__(kThreads) void ipc_reduce_scatter_kernel(IpcAllReduceArgs a) {
  const int v = call_value(a);
  const int64_t S = a.n;
  int64_t lo, hi;
  block_range(S, lo, hi);
  const bool ib = a.in_bf16, ob = a.out_bf16;
  void* my = stage_half(a, a.rank, v);
#pragma unroll
  for (int q = 0; q < W; ++q)
    for (int64_t i = lo + (int64_t)threadIdx.x * kVec; i < hi; i += kThreads * kVec) copy8(my, a.in, ib, q * S + i);
  if (start_barrier<W>(a, v)) {
    const int64_t base = (int64_t)a.rank * S;
    for (int64_t i = lo + (int64_t)threadIdx.x * kVec; i < hi; i += kThreads * kVec) {
      V8 s = peer_sum<W>(a, v, ib, base + i);
#pragma unroll
      for (int j = 0; j < kVec; ++j) s.f[j] *= a.scale;
      store8(a.out, ob, i, s);
    }
  }
  finish(a);
}

// All-gather in place: buf holds W*S elements (2- or 4-byte raw), this rank's shard at r*S.
template <int W>
__global__ __launch_bounds__(kThreads) void ipc_all_gather_kernel(IpcAllReduceArgs a) {
  const int v = call_value(a);
  const int64_t S = a.n;
  int64_t lo, hi;
  block_range(S, lo, hi);
  const bool bf = a.out_bf16;  // element size 2 (raw 16-bit) or 4
  void* my = stage_half(a, a.rank, v);
  const int64_t own = (int64_t)a.rank * S;
  for (int64_t i = lo + (int64_t)threadIdx.x * kVec; i < hi; i += kThreads * kVec) {
    const int64_t e = own + i;
    if (bf) *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(my) + i) = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(a.out) + e);
    else {
      const float* src = reinterpret_cast<const float*>(a.out) + e;
      float* d = reinterpret_cast<float*>(my) + i;
      *reinterpret_cast<f32x4*>(d) = *reinterpret_cast<const f32x4*>(src);
      *reinterpret_cast<f32x4*>(d + 4) = *reinterpret_cast<const f32x4*>(src + 4);
    }
  }
  if (start_barrier<W>(a, v)) {
    for (int64_t i = lo + (int64_t)threadIdx.x * kVec; i < hi; i += kThreads * kVec) {
      // all W-1 remote 16/32-B loads in flight before the local stores
      if (bf) {
        uint4 x[W];
#pragma unroll
        for (int p = 0; p < W; ++p)
          if (p != a.rank) x[p] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(stage_half(a, p, v)) + i);
#pragma unroll
        for (int p = 0; p < W; ++p)
          if (p != a.rank) *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(a.out) + (int64_t)p * S + i) = x[p];
      } else {
        f32x4 x[W][2];
#pragma unroll
        for (int p = 0; p < W; ++p)
          if (p != a.rank) {
            const float* src = reinterpret_cast<const float*>(stage_half(a, p, v)) + i;
            x[p][0] = *reinterpret_cast<const f32x4*>(src);
            x[p][1] = *reinterpret_cast<const f32x4*>(src + 4);
          }
#pragma unroll
        for (int p = 0; p < W; ++p)
          if (p != a.rank) {
            float* d = reinterpret_cast<float*>(a.out) + (int64_t)p * S + i;
            *reinterpret_cast<f32x4*>(d) = x[p][0];
            *reinterpret_cast<f32x4*>(d + 4) = x[p][1];
          }
      }
    }
  }
  finish(a);
}

inline int clamp_blocks(int b) { return std::max(1, std::min(b, kIpcMaxBlocks)); }

#define TFD_IPC_DISPATCH(KERNEL)                                                                  \
  switch (a.world) {                                                                              \
    case 1: KERNEL<1><<<nb, kThreads, 0, s>>>(a); break;                                         \
    case 2: KERNEL<2><<<nb, kThreads, 0, s>>>(a); break;                                         \
    case 3: KERNEL<3><<<nb, kThreads, 0, s>>>(a); break;                                         \
    case 4: KERNEL<4><<<nb, kThreads, 0, s>>>(a); break;                                         \
    case 5: KERNEL<5><<<nb, kThreads, 0, s>>>(a); break;                                         \
    case 6: KERNEL<6><<<nb, kThreads, 0, s>>>(a); break;                                         \
    case 7: KERNEL<7><<<nb, kThreads, 0, s>>>(a); break;                                         \
    default: KERNEL<8><<<nb, kThreads, 0, s>>>(a); break;                                        \
  }

}  // namespace

// blocks: enough that every block has >= ~1 K elements (64 lanes x 16 B per peer in flight per
// wave), never more than the signal layout holds
int ipc_blocks_for(int64_t n) { return clamp_blocks((int)((n + 1023) / 1024)); }

void ipc_allreduce(const IpcAllReduceArgs& a, int blocks, hipStream_t s) {
  const int nb = clamp_blocks(blocks);
  TFD_IPC_DISPATCH(ipc_allreduce_kernel)
}
void ipc_reduce_scatter(const IpcAllReduceArgs& a, int blocks, hipStream_t s) {
  const int nb = clamp_blocks(blocks);
  TFD_IPC_DISPATCH(ipc_reduce_scatter_kernel)
}
void ipc_all_gather(const IpcAllReduceArgs& a, int elem_bytes, int blocks, hipStream_t s) {
  IpcAllReduceArgs b = a;
  b.out_bf16 = elem_bytes == 2 ? 1 : 0;
  const int nb = clamp_blocks(blocks);
  {
    const IpcAllReduceArgs& a = b;
    TFD_IPC_DISPATCH(ipc_all_gather_kernel)
  }
}

}  // namespace tfd
