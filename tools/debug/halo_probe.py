"""Per-layer probe of the 3x3 stride-1 convs of ResNet-50 at batch 128: the LDS halo-tile kernel
(csrc/conv_halo.h, tfd::conv_halo_mode 2) against the im2col-gather implicit GEMM (mode 0), forward,
forward + BN statistics, dgrad (+ residual add), one JSON line per (layer, pass). Median over 5 timed
replays of a 20-launch CUDA graph; random-normal operands.

    python tools/debug/halo_probe.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflow_distributed_amd import _native  # noqa: E402

SHAPES = [("l1.3x3.64", 56, 64), ("l2.3x3.128", 28, 128), ("l3.3x3.256", 14, 256), ("l4.3x3.512", 7, 512)]


def timed(fn, reps=20, trials=5):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    out = []
    for _ in range(trials):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / reps)
    return statistics.median(out)


def main():
    _native.require()
    ops = torch.ops.tfd
    dev = torch.device("cuda", 0)
    N = int(os.environ.get("N", "128"))
    old = ops.conv_halo_mode(-1)
    try:
        for name, H, C in SHAPES:
            g = torch.Generator(device=dev).manual_seed(0)
            x = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
            w = (torch.randn(3, 3, C, C, device=dev, generator=g) * 0.05).to(torch.bfloat16)
            dy = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
            acc = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
            flop = 2.0 * N * H * H * C * C * 9
            res = {}
            for mode in (0, 2):
                ops.conv_halo_mode(mode)
                res[mode] = {
                    "fwd": timed(lambda: ops.conv2d_fwd(x, w, 1, 1)),
                    "fwd_stats": timed(lambda: ops.conv2d_fwd_stats(x, w, 1, 1)),
                    "dgrad": timed(lambda: ops.conv2d_dgrad(dy, w, [N, H, H, C], 1, 1)),
                    "dgrad_add": timed(lambda: ops.conv2d_dgrad(dy, w, [N, H, H, C], 1, 1, acc)),
                }
            for p in res[0]:
                g_us, h_us = res[0][p], res[2][p]
                print(json.dumps({"layer": name, "pass": p, "gather_us": round(g_us, 2), "halo_us": round(h_us, 2),
                                  "gather_TF": round(flop / g_us / 1e6, 1), "halo_TF": round(flop / h_us / 1e6, 1),
                                  "speedup": round(g_us / h_us, 3)}), flush=True)
    finally:
        ops.conv_halo_mode(old)


if __name__ == "__main__":
    main()
