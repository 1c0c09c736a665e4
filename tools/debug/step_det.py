"""Debug: is the whole MNIST training step (dataset mode, prefetch, dropout, fused Adam tail)
bit-reproducible? Runs TRIALS trials of STEPS steps from one identical state (eager steps, or
replays of a one-step graph) and reports, per trial, the first step whose state differs from
trial 0 and where: the forward (loss rows / pool1 / hidden), the bf16 fc gradients, or the
parameters by region.

usage: python tools/debug/step_det.py [steps] [trials]"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from tensorflow_distributed_amd import _native
from tensorflow_distributed_amd.models import mnist_cnn as M

REGIONS = {"conv1": (0, 832), "conv2": (832, 52096), "fc1": (52096, 3264384), "out": (3264384, 3274688)}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    _native.require()
    dev = torch.device("cuda", 0)
    B, n = 128, 8192
    g = torch.Generator(device=dev).manual_seed(5)
    data = torch.rand(n, 784, device=dev, generator=g)
    labels = torch.randint(0, 10, (n,), device=dev, generator=g, dtype=torch.int32)
    perm = torch.randperm(n, device=dev, generator=g).to(torch.int32)
    init = M.flat_from_dict(M.init_params(3)).to(dev)
    s = torch.cuda.Stream()
    for mode in ("eager", "graph"):
        ref = None
        for tr in range(trials):
            eng = torch.classes.tfd.MnistEngine(B, 0, 0.75, 1234, 0)
            eng.set_adam(0.01, 0.9, 0.999, 1e-8)
            eng.set_fused_tail(1)
            eng.set_local_bf16_grads(1)
            rec = []
            with torch.cuda.stream(s):
                eng.params().copy_(init)
                eng.sync_shadow()
                eng.set_dataset(data, labels, perm)
                eng.set_input_mode(1)
                if mode == "graph":
                    eng.capture_train_step("g")
                for i in range(steps):
                    if mode == "graph":
                        eng.replay("g", 1)
                    else:
                        eng.train_step()
                    rec.append({"loss": eng.loss_rows().clone(), "pool1": eng.pool1().clone(),
                                "hidden": eng.hidden().clone(), "gbf": eng.grads_bf16().clone(),
                                "params": eng.params().clone()})
            torch.cuda.synchronize()
            if ref is None:
                ref = rec
                print(f"{mode} trial 0: final loss {rec[-1]['loss'].float().mean().item():.6f}", flush=True)
                continue
            first = None
            for i, (r, q) in enumerate(zip(ref, rec)):
                diff = [k for k in ("loss", "pool1", "hidden", "gbf") if not torch.equal(r[k], q[k])]
                diff += [f"params.{name}" for name, (lo, hi) in REGIONS.items()
                         if not torch.equal(r["params"][lo:hi], q["params"][lo:hi])]
                if diff:
                    first = (i, diff)
                    break
            fl = rec[-1]["loss"].float().mean().item()
            if first is None:
                print(f"{mode} trial {tr}: identical over {steps} steps (final loss {fl:.6f})", flush=True)
            else:
                i, diff = first
                extra = ""
                if "gbf" in diff:
                    d = (ref[i]["gbf"].float() - rec[i]["gbf"].float()).abs()
                    for name, (lo, hi) in REGIONS.items():
                        nz = int((d[lo:hi] > 0).sum())
                        if nz:
                            extra += f" gbf.{name}:{nz}"
                print(f"{mode} trial {tr}: first difference at step {i}: {diff}{extra} (final loss {fl:.6f})", flush=True)
            del rec


if __name__ == "__main__":
    main()
