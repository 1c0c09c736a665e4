"""Cost of the sufficient-factor fc-gradient kernel (mnist_fc_grad_sfb) at world W = 1..8 on one
GPU (MnistEngine.sfb_probe): the compute an 8-GPU SFB step adds in place of the 6.4 MB all-reduce.
    python tools/debug/sfb_probe.py [--batch 128]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from tensorflow_distributed_amd import _native  # noqa: E402
from tensorflow_distributed_amd.models import mnist_cnn as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    _native.require()
    dev = torch.device("cuda", 0)
    B = a.batch
    eng = torch.classes.tfd.MnistEngine(B, 0, 0.75, 1, 0)
    eng.set_adam(0.01, 0.9, 0.999, 1e-8)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.params().copy_(M.flat_from_dict(M.init_params(1)).to(dev))
        eng.sync_shadow()
        g = torch.Generator(device=dev).manual_seed(1)
        data = torch.rand(4096, 784, device=dev, generator=g)
        labels = torch.randint(0, 10, (4096,), device=dev, generator=g, dtype=torch.int32)
        perm = torch.randperm(4096, device=dev, generator=g).to(torch.int32)
        eng.set_dataset(data, labels, perm)
        eng.set_input_mode(1)
        eng.train_step()
        out = {}
        for W in (1, 2, 4, 8):
            eng.sfb_probe(W, 20)
            out[W] = round(eng.sfb_probe(W, a.iters) * 1e3, 2)
    torch.cuda.synchronize()
    print(json.dumps({"sfb_kernel_us_by_world": out, "batch": B}))


if __name__ == "__main__":
    main()
