"""Operand-layout probe of the 128-row GEMM core: dense 4096^3 with a k-contiguous A (linear_fwd:
A KC, B MN-contiguous) against both operands MN-contiguous (linear_wgrad: the weight-gradient
layout, fp32 store, no split-K), plus ResNet-50 1x1 weight-gradient shapes as one dense GEMM
(no split: few tiles) -- separates the operand layout from the split-K / atomics cost.

    python tools/debug/mnc_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from tensorflow_distributed_amd import _native  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    _native.require()
    dev = torch.device("cuda", 0)
    old = torch.ops.tfd.conv_gemm_core(0)
    for n in (4096, 8192):
        x = torch.randn(n, n, device=dev).bfloat16()
        w = torch.randn(n, n, device=dev).bfloat16()
        dw = torch.empty(n, n, device=dev)
        f = 2.0 * n ** 3
        t1 = timeit(lambda: torch.ops.tfd.linear_fwd(x, w, None))
        t2 = timeit(lambda: torch.ops.tfd.linear_wgrad(x, w, dw))
        print(f"dense {n}^3: A KC (linear_fwd) {t1:8.1f} us {f / t1 / 1e6:7.1f} TF/s | both MNC (linear_wgrad) "
              f"{t2:8.1f} us {f / t2 / 1e6:7.1f} TF/s", flush=True)
    torch.ops.tfd.conv_gemm_core(old)


if __name__ == "__main__":
    main()
