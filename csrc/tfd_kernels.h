// Host-side launcher API of the HIP kernel library (no HIP kernel syntax here: this header is
// included by the g++-compiled torch binding / runtime layer).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace tfd {

// ---------------- fused MNIST CNN train step ----------------
struct MnistStepArgs {
  int B;                       // per-rank batch
  // data: rows of `data` ([n_data][784] fp32) are taken as perm[(step*B + b) % n_data] when perm
  // is non-null, else row b directly (a fed batch). labels likewise ([n_data] int32 class ids).
  const float* data;
  const int* labels;
  const int* perm;
  int n_data;
  const int64_t* step;         // device global_step (read by every kernel of the step)
  int64_t* t_out;              // if set, the head kernel writes *step + 1 here: Adam's t for the fused
                               // one-GPU optimizer tail, which bumps *step itself (mnist_adam_fused)
  int64_t* step_bump;          // if set, the last conv-grad reduce kernel increments *step (it is the
                               // first kernel of the step that no longer reads it; the optimizer after it
                               // then sees t = global_step + 1 directly)
  // params
  const float* p32;            // flat fp32 master params (mnist_layout.h)
  const uint16_t* pbf;         // flat bf16 shadow of p32
  float* grad;                 // flat fp32 gradient buffer
  uint16_t* gbf_a;             // if set (DP with a bf16 wire format): the fc backward writes bucket A's
                               // gradients [OFF_WD1, TOTAL) as bf16 straight into this flat buffer (the
                               // all-reduce operand) instead of fp32 into `grad` -- no separate cast pass
  uint16_t* gbf_b;             // likewise for bucket B [0, OFF_WD1): the conv-slab reduce writes bf16 here
  // activations / workspace (bf16 stored as uint16)
  uint16_t* p1;  uint8_t* idx1;   // [B][14][14][32]
  uint16_t* p2;  uint8_t* idx2;   // [B][3136]
  float* fc1_slab;                // [fc1_splits][B][1024]
  uint16_t* hd;  uint16_t* dh;    // [B][1024]
  float* dlogits;                 // [B][10]
  float* loss_row; float* correct_row;  // [B]
  uint16_t* dz2;                  // [B][14][14][64]
  float* wg2_slab;                // [wg2_splits][801][64]
  float* wg1_slab;                // [2B][832] (one slab per half image)
  int fc1_splits, wg2_splits;
  float keep_prob;
  uint32_t seed, rank;
  // Next-batch prefetch (device dataset mode): the kernel that bumps the step also gathers the NEXT
  // step's batch -- rows[b] = perm[...], xpre[b] = data[rows[b]] ([B][784] fp32), ypre[b] = its label
  // -- and tags it with that step in rows[B]. Consumers load the prefetched value speculatively
  // beside the tag and the step and fall back to the step -> perm -> row chain on a mismatch, so the
  // forward starts with one memory round trip to an L2-resident buffer instead of three dependent
  // loads ending in a random 3 KB row of a 172 MB array.
  int* rows;
  float* xpre;
  int* ypre;
  int64_t* dbg;                // timing-stamp builds only (TFD_STAMP): per-block phase clocks
  // DP with sufficient-factor gradients (mnist_fc_grad_sfb): the fc-layer factors of ALL ranks,
  // all-gathered. sfb_p2 = [W*B][3136] pooled conv2 activations (rank r's rows at r*B; rank r's p2
  // IS its slot); sfb_dr = [W][sfb_rs] per-rank slots holding dh [B][1024] bf16, hd [B][1024] bf16
  // and dlogits [B][10] fp32, in that order (this rank's dh / hd / dlogits point into its slot).
  int sfb_world;
  const uint16_t* sfb_p2;
  const uint16_t* sfb_dr;
  int64_t sfb_rs;
  // ZeRO-sharded SFB: only the 64-row fc1 dW tile rows [sfb_by_lo, sfb_by_hi] (this rank's shard)
  // plus the bias tile row are computed; sfb_by_hi < sfb_by_lo (default 0, -1) means all rows
  int sfb_by_lo, sfb_by_hi;
};

int mnist_fc1_splits(int B);
int mnist_wg2_splits(int B);
void mnist_forward(const MnistStepArgs& a, bool train, hipStream_t s);        // conv1, conv2, fc1, head
void mnist_forward_conv(const MnistStepArgs& a, hipStream_t s);               // conv1, conv2 (read region B)
void mnist_forward_fc(const MnistStepArgs& a, bool train, hipStream_t s);     // fc1, head (read region A)
// fc1 dW/dX + out-layer grads. part 0: one launch; part 1: dW + out grads (bucket A complete);
// part 2: dX (DP launches 1 then 2 so bucket A's all-reduce starts before the dX GEMM)
void mnist_backward_a(const MnistStepArgs& a, hipStream_t s, int part = 0);
// conv2 wgrad slabs + conv2 dgrad + conv1 wgrad slabs (one launch) -> bucket B's slabs done
void mnist_backward_b(const MnistStepArgs& a, hipStream_t s);
// deterministic conv weight-gradient slab reduction (+ the global_step bump, MnistStepArgs::step_bump)
void mnist_conv_grad_reduce(const MnistStepArgs& a, hipStream_t s);

// One-GPU optimizer tail: TF ApplyAdam over the whole flat buffer with the conv weight-gradient
// slab reduction fused in (the conv region takes its gradient straight from the per-block slabs),
// t = *t (written by the head kernel, MnistStepArgs::t_out), *step bumped once by the kernel.
struct MnistAdamArgs {
  float* p; float* m; float* v;
  uint16_t* pbf;  // bf16 shadow written beside p; null: none (the fp32 engine reads p itself)
  float lr, beta1, beta2, eps;
  const int64_t* t;
  int64_t* step;
  const uint16_t* gbf;  // if non-null: the fc-region (bucket A) gradients are bf16 here (gbf_a)
};
// fc_region = false: the conv region only
void mnist_adam_fused(const MnistStepArgs& a, const MnistAdamArgs& o, hipStream_t s, bool fc_region = true);
// DP, sufficient-factor broadcasting: every fc-layer weight gradient is a sum of per-example outer
// products (dW_fc1 = [P2;1]^T dH, dW_out = [Hd;1]^T dlogits), so the all-reduced gradient is ONE
// GEMM over the all-gathered factors (K = W*B). Writes the summed fc-region gradients (bucket A)
// like mnist_backward_a part 1 (bf16 into gbf_a when set), identical on every rank.
// with_reduce: the same launch also runs mnist_conv_grad_reduce's blocks (next-batch gather + conv
// slab reduce + step bump; needs t_out like its one-launch form) -- the merged DP tail.
void mnist_fc_grad_sfb(const MnistStepArgs& a, hipStream_t s, bool with_reduce = false);
// fc1 dW tile-row range (64 rows per tile row) covering flat fc1 weight rows [row0, row1)
void mnist_sfb_tile_rows(int row0, int row1, int* by_lo, int* by_hi);
// bf16 elements of one rank's sfb_dr slot for batch B (dh + hd + dlogits, padded to 64)
int64_t mnist_sfb_slot_elems(int B);

// ---------------- reference-precision (fp32) MNIST step: csrc/kernels/mnist_f32.hip ----------------
// Same dataflow and flat parameter layout as the bf16 step, every operand and activation fp32,
// every GEMM on v_mfma_f32_16x16x4_f32 (csrc/gemm_f32.h). The conv-slab layouts match the bf16
// step's, so mnist_conv_grad_reduce (MnistStepArgs view) finishes the conv gradients.
struct MnistF32Args {
  int B;
  const float* data; const int* labels; const int* perm; int n_data;
  const int64_t* step;
  const float* p32;            // flat fp32 params
  float* grad;                 // flat fp32 gradients
  float* p1; uint8_t* idx1;    // [B][14][14][32]
  float* p2; uint8_t* idx2;    // [B][3136]
  float* fc1_slab;             // [splits][B][1024]
  float* hd; float* dh;        // [B][1024]
  float* dlogits;              // [B][10]
  float* loss_row; float* correct_row;
  float* dz2;                  // [B][14][14][64]
  float* wg2_slab;             // [wg2_splits][801][64]
  float* wg1_slab;             // [2B][832]
  int fc1_splits, wg2_splits;
  float keep_prob;
  uint32_t seed, rank;
  int64_t* t_out;              // if set: the head writes step + 1 here (the fused optimizer tail's t)
};
int mnist_f32_fc1_splits();
int mnist_f32_wg2_splits(int B);
void mnist_f32_forward(const MnistF32Args& a, bool train, hipStream_t s);
void mnist_f32_backward(const MnistF32Args& a, hipStream_t s);  // fc + conv grads (slabs for conv)

// ---------------- optimizers (flat, fp32 master + bf16 shadow) ----------------
struct AdamArgs {
  float* p; float* m; float* v; const float* g; uint16_t* pbf;
  const uint16_t* gbf;         // if non-null, gradients are read from this bf16 buffer instead of g
  int64_t n;
  float lr, beta1, beta2, eps;
  const int64_t* step;         // device step counter; Adam's t = *step + t_offset (read-only here)
  int t_offset;
  float grad_scale;            // multiply g (e.g. 1/N for sum-all-reduce)
};
void adam_apply(const AdamArgs& a, hipStream_t s);
// ONE launch over up to 3 disjoint ranges [beg, beg + n) of the flat buffers (a's pointers are the
// buffer bases, a.n is ignored): the ZeRO-1 optimizer (conv bucket + this rank's fc1 shard + tail)
// without a launch per range. Every beg and every n but the last must be a multiple of 4.
void adam_apply_ranges(const AdamArgs& a, int nr, const int64_t* beg, const int64_t* n, hipStream_t s);
struct SgdArgs {
  float* p; float* mom; const float* g; uint16_t* pbf; const uint16_t* gbf; int64_t n;
  float lr, momentum, weight_decay, grad_scale; int nesterov;
};
// roofline probes: the optimizer's byte floor (Adam's 28 B/param of traffic, optional extra fp32 read
// stream of nx4 float4) and an empty launch (tools/debug/roofline_probe.py)
void stream_floor(float* p, float* m, float* v, const uint16_t* g, uint16_t* pbf, const float* x, int64_t n4, int64_t nx4,
                  int blocks, int unroll, hipStream_t s);
void noop_launch(int blocks, hipStream_t s);
void sgd_apply(const SgdArgs& a, hipStream_t s);
void cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t s);
void cast_bf16_f32(const uint16_t* x, float* y, int64_t n, float scale, hipStream_t s);
void scale_f32(float* x, int64_t n, float scale, hipStream_t s);
void copy_f32(float* dst, const float* src, int64_t n, hipStream_t s);
void vec_accumulate(float* dst, const float* src, int64_t n, float alpha, hipStream_t s);

}  // namespace tfd
