// Flat parameter / gradient layout of the reference 2-conv MNIST CNN
// (/root/reference/mnist_python_m.py:185-196, mnist_single.py:34-51).
//
// One flat fp32 buffer holds every trainable tensor; each weight is immediately followed by its
// bias so that a weight-gradient GEMM can emit the bias gradient as one extra output row (the
// "ones row" trick: d bias = 1^T dY). Regions are padded to 64 elements (256 B alignment).
// Backward produces the tail region [OFF_WD1, TOTAL) first (bucket A, 98% of the bytes), then the
// head region [0, OFF_WD1) (bucket B) -- the DP reducer buckets follow this split.
#pragma once
#include <stdint.h>

namespace tfd {
namespace mnist {

constexpr int IMG = 28, C1 = 32, P1H = 14, C2 = 64, P2H = 7, FEAT = P2H * P2H * C2 /*3136*/, HID = 1024, NCLS = 10;
constexpr int KTAPS = 25;

constexpr int64_t OFF_WC1 = 0;                         // [5][5][1][32]
constexpr int64_t OFF_BC1 = OFF_WC1 + KTAPS * C1;      // [32]
constexpr int64_t OFF_WC2 = 832;                       // [5][5][32][64]
constexpr int64_t OFF_BC2 = OFF_WC2 + KTAPS * C1 * C2; // [64]   (row 800 of a [801][64] block)
constexpr int64_t OFF_WD1 = OFF_BC2 + C2;              // 52096: [3136][1024]
constexpr int64_t OFF_BD1 = OFF_WD1 + (int64_t)FEAT * HID; // [1024] (row 3136 of [3137][1024])
constexpr int64_t OFF_OUT = OFF_BD1 + HID;             // 3264384: [1024][10]
constexpr int64_t OFF_BOUT = OFF_OUT + HID * NCLS;     // [10]  (row 1024 of [1025][10])
constexpr int64_t TOTAL = 3274688;                      // padded to a multiple of 64
constexpr int64_t NUM_PARAMS = 3274634;                 // reference count
constexpr int64_t BUCKET_SPLIT = OFF_WD1;               // [0,split) = bucket B, [split,TOTAL) = bucket A

static_assert(OFF_BC1 == 800, "layout");
static_assert(OFF_WD1 == 52096, "layout");
static_assert(OFF_BOUT + NCLS <= TOTAL, "layout");

}  // namespace mnist
}  // namespace tfd
