"""Dense bf16 GEMM probe of the 256 x 256 core (torch.ops.tfd.gemm_nt: C = A . Bt^T) against the
128 x 128 core (linear_fwd) and hipBLASLt (torch.matmul) on the same GPU: correctness vs an fp32
reference, then TF/s on uniform [-1, 1) operands (not zeros: DVFS reads high on zero-filled data).

    python tools/debug/gemm256_probe.py [--iters 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from tensorflow_distributed_amd import _native  # noqa: E402


def timeit(fn, iters):
    for _ in range(5):
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
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    _native.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in [(256, 256, 64), (300, 264, 72), (1000, 520, 1032), (4096, 4096, 4096)]:
        A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        Bt = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).bfloat16()
        C = torch.ops.tfd.gemm_nt(A, Bt).float()
        ref = A.float() @ Bt.float().t()
        err = ((C - ref).abs().max() / ref.abs().max()).item()
        print(f"check M={M} N={N} K={K}: max rel err {err:.2e} {'OK' if err < 1e-2 else 'BAD'}", flush=True)
    for S in (4096, 8192):
        A = (torch.rand(S, S, device=dev, generator=g) * 2 - 1).bfloat16()
        Bt = (torch.rand(S, S, device=dev, generator=g) * 2 - 1).bfloat16()
        B = Bt.t().contiguous()
        fl = 2 * S ** 3
        t256 = timeit(lambda: torch.ops.tfd.gemm_nt(A, Bt), a.iters)
        t128 = timeit(lambda: torch.ops.tfd.linear_fwd(A, B, None), a.iters)
        tt = timeit(lambda: A @ B, a.iters)
        print(f"dense {S}^3: g256 {t256:8.1f} us {fl / t256 / 1e6:7.1f} TF/s | g128 {t128:8.1f} us "
              f"{fl / t128 / 1e6:7.1f} TF/s | torch {tt:8.1f} us {fl / tt / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
