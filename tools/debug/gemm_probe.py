"""Throughput probe of the NHWC conv / dense GEMM kernels (torch.ops.tfd.*) on ResNet-50 layer shapes
at batch 128, next to PyTorch-ROCm (MIOpen / hipBLASLt) on the same shapes and dtype. Prints one line
per (shape, pass): our us, torch us, our TFLOP/s. Random-normal operands (not zeros: DVFS reads high
on zero-filled operands).

    python tools/debug/gemm_probe.py [--iters 20] [--only fwd,dgrad,wgrad]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from tensorflow_distributed_amd import _native  # noqa: E402

# (name, H, C, K, R, stride) at N = 128; pad = R // 2
SHAPES = [
    ("l1.1x1.64-64", 56, 64, 64, 1, 1),
    ("l1.3x3.64", 56, 64, 64, 3, 1),
    ("l1.1x1.64-256", 56, 64, 256, 1, 1),
    ("l1.1x1.256-64", 56, 256, 64, 1, 1),
    ("l2.3x3.128", 28, 128, 128, 3, 1),
    ("l2.1x1.128-512", 28, 128, 512, 1, 1),
    ("l2.1x1.512-128", 28, 512, 128, 1, 1),
    ("l3.3x3.256", 14, 256, 256, 3, 1),
    ("l3.1x1.256-1024", 14, 256, 1024, 1, 1),
    ("l3.1x1.1024-256", 14, 1024, 256, 1, 1),
    ("l4.3x3.512", 7, 512, 512, 3, 1),
    ("l4.1x1.512-2048", 7, 512, 2048, 1, 1),
    ("l4.1x1.2048-512", 7, 2048, 512, 1, 1),
    # stride-2 entries of each stage (v1.5: the 3x3 and the 1x1 downsample carry the stride)
    ("l2.3x3.128.s2", 56, 128, 128, 3, 2),
    ("l2.ds.256-512.s2", 56, 256, 512, 1, 2),
    ("l3.3x3.256.s2", 28, 256, 256, 3, 2),
    ("l3.ds.512-1024.s2", 28, 512, 1024, 1, 2),
    ("l4.3x3.512.s2", 14, 512, 512, 3, 2),
    ("l4.ds.1024-2048.s2", 14, 1024, 2048, 1, 2),
    # the stem: 3 input channels padded to 8 (pad_channels)
    ("stem.7x7.8-64.s2", 224, 8, 64, 7, 2),
]


def timeit(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--N", type=int, default=128)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--torch", type=int, default=1)
    ap.add_argument("--match", default="", help="only shapes whose name contains this")
    a = ap.parse_args()
    _native.require()
    dev = torch.device("cuda", 0)
    passes = a.only.split(",")
    tot = {p: [0.0, 0.0, 0.0] for p in passes}
    # dense GEMM sanity point: 4096^3
    x = torch.randn(4096, 4096, device=dev).bfloat16()
    w = torch.randn(4096, 4096, device=dev).bfloat16()
    wt_ = w.t().contiguous()
    t = timeit(lambda: torch.ops.tfd.linear_fwd(x, w, None), a.iters)
    t2 = timeit(lambda: torch.ops.tfd.gemm_nt(x, wt_), a.iters)
    tt = timeit(lambda: x @ w, a.iters)
    print(f"dense4096^3 fwd: core128 {t:8.1f} us {2 * 4096**3 / t / 1e6:7.1f} TF/s | core256 {t2:8.1f} us "
          f"{2 * 4096**3 / t2 / 1e6:7.1f} TF/s | torch {tt:8.1f} us {2 * 4096**3 / tt / 1e6:7.1f} TF/s", flush=True)
    shapes = SHAPES if not a.match else [x for x in SHAPES if a.match in x[0]]
    for name, H, C, K, R, st in shapes:
        N, pad = a.N, R // 2
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(R, R, C, K, device=dev) * 0.05).bfloat16()
        Ho = (H + 2 * pad - R) // st + 1
        dy = torch.randn(N, Ho, Ho, K, device=dev).bfloat16()
        dw = torch.zeros(R, R, C, K, device=dev)
        flop = 2.0 * N * Ho * Ho * K * R * R * C
        xt = x.permute(0, 3, 1, 2)  # NCHW view of NHWC storage = channels_last
        wt = w.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last)
        dyt = dy.permute(0, 3, 1, 2)
        for p in passes:
            if p == "fwd":
                ours = lambda: torch.ops.tfd.conv2d_fwd(x, w, st, pad)  # noqa: E731
                ref = lambda: F.conv2d(xt, wt, stride=st, padding=pad)  # noqa: E731
            elif p == "dgrad":
                ours = lambda: torch.ops.tfd.conv2d_dgrad(dy, w, [N, H, H, C], st, pad)  # noqa: E731
                ref = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
                    dyt, xt, wt, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [True, False, False])
            else:
                ours = lambda: torch.ops.tfd.conv2d_wgrad(x, dy, dw, st, pad)  # noqa: E731
                ref = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
                    dyt, xt, wt, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False])
            # both GEMM cores of the conv ops: 128-row register-staged, 256-row DMA (forced on)
            old = torch.ops.tfd.conv_gemm_core(0)
            t = timeit(ours, a.iters)
            torch.ops.tfd.conv_gemm_core(2)
            t2 = timeit(ours, a.iters)
            torch.ops.tfd.conv_gemm_core(old)
            tt = timeit(ref, a.iters) if a.torch else float("nan")
            tot[p][0] += t
            tot[p][1] += tt
            tot[p][2] += min(t, t2)
            print(f"{name:18s} {p:5s}: core128 {t:8.1f} us {flop / t / 1e6:7.1f} TF/s | core256 {t2:8.1f} us "
                  f"{flop / t2 / 1e6:7.1f} TF/s | torch {tt:8.1f} us {flop / tt / 1e6:7.1f} TF/s", flush=True)
    for p, (o, r, b) in tot.items():
        print(f"TOTAL {p}: core128 {o:.1f} us, best of both {b:.1f} us, torch {r:.1f} us")


if __name__ == "__main__":
    main()
