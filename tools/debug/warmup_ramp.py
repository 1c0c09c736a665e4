"""Diagnose the short-run vs long-run gap of bench.py (VERDICT r1 'weak' item 1).

Builds the engine exactly like bench.py, captures the step graph, then times every replay of a
cold run individually with HIP events (plus host wall per chunk), so a clock ramp, a first-replay
cost or a steady drift shows up as a shape over the first few hundred steps.

    python tools/debug/warmup_ramp.py [--steps 400]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--batch_size", type=int, default=128)
    a = ap.parse_args()
    import torch

    from tensorflow_distributed_amd import _native
    from tensorflow_distributed_amd.models import mnist_cnn as M

    _native.require()
    dev = torch.device("cuda", 0)
    B = a.batch_size
    eng = torch.classes.tfd.MnistEngine(B, 0, 0.75, 1, 0)
    eng.set_adam(0.01, 0.9, 0.999, 1e-8)
    eng.set_local_bf16_grads(1)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        g = torch.Generator(device=dev).manual_seed(1000)
        data = torch.rand(55000, 784, device=dev, generator=g)
        labels = torch.randint(0, 10, (55000,), device=dev, generator=g, dtype=torch.int32)
        perm = torch.randperm(55000, device=dev, generator=g).to(torch.int32)
        eng.params().copy_(M.flat_from_dict(M.init_params(1)).to(dev))
        eng.sync_shadow()
        eng.set_dataset(data, labels, perm)
        eng.set_input_mode(1)
        eng.train_step()
        eng.capture_train_step("train")
    torch.cuda.synchronize()
    n = a.steps
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    with torch.cuda.stream(s):
        evs[0].record(s)
        for i in range(n):
            eng.replay("train", 1)
            evs[i + 1].record(s)
    torch.cuda.synchronize()
    per = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(n)]
    # host-timed chunks like bench.py after this warm run: 20 steps, then 1000 steps
    res = {"per_step_us_first40": [round(v, 1) for v in per[:40]]}
    for lo, hi in ((0, 5), (5, 25), (25, 100), (100, 200), (200, n)):
        if hi <= n:
            res[f"mean_us_{lo}_{hi}"] = round(sum(per[lo:hi]) / (hi - lo), 2)
    for k in (20, 1000, 20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            eng.replay("train", k)
        torch.cuda.synchronize()
        res[f"host_us_per_step_{k}_after_warm"] = round((time.perf_counter() - t0) * 1e6 / k, 2)
    # a cold-ish repeat: sleep 2 s (clocks drop), then 20 steps
    time.sleep(2.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        eng.replay("train", 20)
    torch.cuda.synchronize()
    res["host_us_per_step_20_after_2s_idle"] = round((time.perf_counter() - t0) * 1e6 / 20, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
