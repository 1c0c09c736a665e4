"""Floors for the MNIST step's roofline, measured on the box:

* the optimizer's byte floor: tfd::roofline_stream moves exactly ApplyAdam's traffic over the flat
  parameter buffer (fp32 p/m/v read + written in place, bf16 gradient read, bf16 shadow written:
  28 B/param) with no math, swept over grid size and loads in flight; "+slabs" also reads the
  13.1 MB of conv weight-gradient slabs the one-GPU tail reduces;
* the same buffers through the real flat Adam kernel (tfd::adam_flat), for the gap at equal bytes;
* the dependent-launch boundary: a chain of empty kernels in one captured graph.

Every number is the median over 7 replays of a graph of R launches (the buffers stay resident in
the 256 MB Infinity Cache between replays, as in the training loop). One JSON line per config.

    python tools/debug/roofline_probe.py
"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tensorflow_distributed_amd import _native  # noqa: E402
from tensorflow_distributed_amd.models import mnist_cnn as M  # noqa: E402


def timed(fn, reps=50, trials=7):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
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
    return statistics.median(out), min(out)


def main():
    _native.require()
    dev = torch.device("cuda", 0)
    n = M.TOTAL // 4 * 4
    p = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.ones(n, device=dev)
    g = (torch.randn(n, device=dev) * 1e-3).to(torch.bfloat16)
    pbf = torch.empty(n, dtype=torch.bfloat16, device=dev)
    nslab = 64 * 801 * 64 + 2 * 128 * 832  # conv2 + conv1 weight-gradient slabs at B = 128
    x = torch.zeros(min(n, nslab) // 4 * 4, device=dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    base_bytes = 28 * n
    for extra in (None, x):
        nb = base_bytes + (0 if extra is None else 4 * extra.numel())
        for blocks in (1024, 2048, 4096, 8192, (n // 4 + 255) // 256):
            for unroll in (1, 2, 4):
                if blocks * 256 * unroll > n // 4 * 2:
                    continue
                med, best = timed(lambda: torch.ops.tfd.roofline_stream(p, m, v, g, pbf, extra, blocks, unroll))
                print(json.dumps({"probe": "stream_floor" + ("+slabs" if extra is not None else ""), "blocks": blocks,
                                  "unroll": unroll, "bytes": nb, "us_median": round(med, 3), "us_min": round(best, 3),
                                  "TB_per_s": round(nb / med / 1e6, 3)}), flush=True)
    med, best = timed(lambda: torch.ops.tfd.adam_flat(p, m, v, g, pbf, 1e-3, 0.9, 0.999, 1e-8, step, 1.0))
    print(json.dumps({"probe": "adam_flat (adam_kernel, 2048 blocks)", "bytes": base_bytes, "us_median": round(med, 3),
                      "us_min": round(best, 3), "TB_per_s": round(base_bytes / med / 1e6, 3)}), flush=True)
    for blocks in (1, 256, 1024):
        med, best = timed(lambda: torch.ops.tfd.noop(blocks), reps=300)
        print(json.dumps({"probe": "noop chain (dependent launch boundary)", "blocks": blocks,
                          "us_median": round(med, 3), "us_min": round(best, 3)}), flush=True)


if __name__ == "__main__":
    main()
