"""Microbenchmark of the IPC one-shot all-reduce: W processes (sharing one GPU on the test box, one
GPU each on a node), R in-place all-reduces of an n-element bf16 (or fp32) bucket, timed per call
with HIP events on rank 0 after a warm-up; rank 0 prints one JSON line.

    python tools/debug/ipc_bench.py --world 2 --n 52096 --reps 200 [--fp32]

On one shared GPU the numbers include the processes' time-slicing of the device; what they compare
is two kernel designs under the same conditions (run the kernel trace with rocprofv3 for the
per-kernel device time).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _worker(rank, world, n, reps, fp32, max_blocks):
    import torch

    from tensorflow_distributed_amd.parallel.ipc import make_ipc_comm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = make_ipc_comm(rank, world, 0, n, max_blocks=max_blocks)
    dt = torch.float32 if fp32 else torch.bfloat16
    x = (torch.arange(n, device=dev, dtype=torch.float32) % 13).to(dt)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(20):
            comm.all_reduce(x, 1.0 / world)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            comm.all_reduce(x, 1.0 / world)
        e1.record(s)
    torch.cuda.synchronize()
    ok = bool(torch.equal(x.float(), (torch.arange(n, device=dev, dtype=torch.float32) % 13).to(dt).float()))
    err = comm.error()
    comm.close()
    return e0.elapsed_time(e1) * 1e3 / reps, ok, err


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--n", type=int, default=52096)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--max_blocks", type=int, default=8)
    a = ap.parse_args()
    from dist_util import run_ranks

    res = run_ranks(_worker, a.world, a.n, a.reps, a.fp32, a.max_blocks, timeout=300)
    print(json.dumps({"world": a.world, "n": a.n, "max_blocks": a.max_blocks, "dtype": "fp32" if a.fp32 else "bf16",
                      "us_per_allreduce_rank0": round(res[0][0], 2),
                      "us_per_allreduce_max": round(max(r[0] for r in res), 2),
                      "values_ok": all(r[1] for r in res), "errors": [r[2] for r in res]}))


if __name__ == "__main__":
    main()
