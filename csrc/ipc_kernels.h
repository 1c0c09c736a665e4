// Host-side API of the one-shot peer-to-peer (IPC) all-reduce (csrc/comm/ipc_allreduce.hip).
//
// for small gradient buckets the latency of a ring dominates, so
// every rank's kernel reads its slice from ALL peers' staging buffers at once (on MI355X: over all
// 7 xGMI links in parallel), reduces in fp32 registers and writes the result locally. Cross-rank
// ordering uses per-block START/END flag barriers in uncached (fine-grained) signal memory with
// system-scope release/acquire; every spin is time-bounded (error flag instead of a hang).
//
// Single-stream requirement: the collectives of one communicator share its two staging halves,
// its call counter and its arrival ticket, so two of them must never be in flight at once. The
// host side (IpcComm::order/mark, csrc/runtime/ipc_comm.cpp) makes a launch on a new stream wait
// for the previous launch; inside a captured graph the capture order on the engine's one comm
// stream provides it.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace tfd {

constexpr int kIpcMaxRanks = 8;
constexpr int kIpcMaxBlocks = 256;
// signal region layout (int32): [kIpcMaxBlocks][kIpcMaxRanks] START flags, then the sticky error
// word, the call counter and the per-call block-arrival ticket.
constexpr int kIpcSigFlags = kIpcMaxBlocks * kIpcMaxRanks;
constexpr int kIpcSigInts = kIpcSigFlags + 8;

struct IpcAllReduceArgs {
  const void* in;               // local input (fp32 or bf16)
  void* out;                    // local output (may alias in)
  void* stage[kIpcMaxRanks];    // staging buffer of every rank (two halves of half_bytes), mapped here
  int* sig[kIpcMaxRanks];       // signal region of every rank, mapped here
  int64_t n;                    // elements
  int rank, world;
  int in_bf16, out_bf16;
  float scale;                  // applied to the reduced sum
  int64_t spin_limit_ticks;     // s_memrealtime (100 MHz) ticks before a barrier gives up
  int64_t half_bytes;           // bytes per staging half (call v uses half v & 1)
};

int ipc_blocks_for(int64_t n);  // grid size for an n-element collective
void ipc_allreduce(const IpcAllReduceArgs& a, int blocks, hipStream_t s);
// n = shard size S. reduce-scatter: in = N*S local elements, out = this rank's S-element shard.
void ipc_reduce_scatter(const IpcAllReduceArgs& a, int blocks, hipStream_t s);
// all-gather in place: out = N*S elements of elem_bytes (2 or 4) with this rank's shard at rank*S.
void ipc_all_gather(const IpcAllReduceArgs& a, int elem_bytes, int blocks, hipStream_t s);

}  // namespace tfd
