// Grid-wide per-column sums in the producing launch ("last arriver" reduction), so the batch-norm
// statistics / parameter gradients need no separate finalize launch (bn_final_kernel: 106 launches
// of 5-7 us per ResNet-50 step, each a latency-bound island between two bandwidth kernels).
//
// Every row-block `row` of a grid of `nrows` has written its partial row part[row][2][ld] with
// tot_store (write-through; columns
// c0 .. c0+nc of the pair a, b). The last block of each group of G consecutive rows (a ticket per
// (column tile, group)) sums its group's rows in row order into row g*G; the last group of the
// column tile sums the group rows in group order and writes tot_a / tot_b[c0 .. c0+nc). Fixed
// summation order: deterministic. Publication follows the write-through hand-off recipe
// (/opt/skills/guides/cdna_hip_programming.md, Guideline 16 R1 / "In-launch split-K reduction"):
// sc1 payload stores, s_waitcnt vmcnt(0) in every storing wave, barrier, relaxed agent-scope ticket
// add by one lane; the last arriver reads the handed-off words with sc1 loads (no acquire fence) --
// valid whichever XCDs the blocks ran on. Counters are reset by their last
// arriver, so a workspace slot is reusable by the next launch (zeroed once at allocation).
#pragma once
#include <hip/hip_runtime.h>

namespace tfd {

constexpr int kTotMaxGroups = 128;              // groups per column tile (+1 final counter)
constexpr int kTotCntPerTile = kTotMaxGroups + 1;
constexpr int kTotMaxTiles = 64;                // column tiles per launch
constexpr int kTotSlots = 64;                   // launches rotate over slots (no reuse by neighbours)

// Workspace of kTotSlots x kTotMaxTiles x kTotCntPerTile zeroed counters on the current device;
// each call returns the next slot (host side, csrc/kernels/norm.hip).
int* bn_ticket_slot();
bool bn_totals_enabled();          // built with TFD_BN_TOTALS (norm.hip)
int bn_totals_group(int nrows);    // rows per group of the two-level reduction

// Handed-off words are stored write-through (sc1: an agent-scope relaxed atomic store), so the
// producer needs no release fence -- an agent-scope release writes back the whole L2 of its XCD,
// which in EVERY block of a GEMM that just stored its output tile cost 1.5-3x the kernel time.
typedef __attribute__((address_space(1))) float tot_gf32;
typedef __attribute__((address_space(1))) int tot_gi32;
__device__ __forceinline__ void tot_store(float* p, float v) {
  __hip_atomic_store((tot_gf32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The last arriver reads every handed-off word with an sc1 load (agent-scope relaxed atomic load)
// instead of taking an acquire fence: an agent-scope acquire invalidates the XCD's L2, which in a
// streaming kernel full of dirty output lines cost far more than the finalize launch it replaces.
__device__ __forceinline__ float tot_load(const float* p) {
  return __hip_atomic_load((const tot_gf32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every storing wave drains its sc1 stores, the barrier orders them before lane 0's ticket add
__device__ __forceinline__ bool tot_ticket(int* cnt, int expected, int* lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add((tot_gi32*)cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == expected - 1;
    if (last) __hip_atomic_store((tot_gi32*)cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}

// cnt: this column tile's kTotCntPerTile counters. NT threads. lds_flag: one int of LDS.
template <int NT>
__device__ void totals_last_arriver(float* __restrict__ part, int nrows, int row, int ld, int c0, int nc, int G,
                                    int* cnt, float* __restrict__ tot_a, float* __restrict__ tot_b, int* lds_flag) {
  const int g = row / G, ng = (nrows + G - 1) / G, r0 = g * G, gsize = min(G, nrows - r0);
  if (!tot_ticket(cnt + g, gsize, lds_flag)) return;
  for (int j = threadIdx.x; j < 2 * nc; j += NT) {
    const int off = (j < nc ? 0 : ld) + c0 + (j < nc ? j : j - nc);
    float s = 0.f;
    for (int r = r0; r < r0 + gsize; ++r) s += tot_load(part + (size_t)r * 2 * ld + off);
    tot_store(part + (size_t)r0 * 2 * ld + off, s);
  }
  if (!tot_ticket(cnt + kTotMaxGroups, ng, lds_flag)) return;
  for (int j = threadIdx.x; j < 2 * nc; j += NT) {
    const int col = c0 + (j < nc ? j : j - nc), off = (j < nc ? 0 : ld) + col;
    float s = 0.f;
    for (int q = 0; q < ng; ++q) s += tot_load(part + (size_t)q * G * 2 * ld + off);
    (j < nc ? tot_a : tot_b)[col] = s;
  }
}

}  // namespace tfd
