"""Bit-reproducibility of the native MNIST step when several processes share the GPU.

The same forward/backward on fixed inputs must give identical activations and gradients on every
repeat and in every process (this caught kernels built with packed-fp32 VALU ops giving sporadic
differences under GPU sharing -- docs/DESIGN.md section 6)."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(__file__))
from dist_util import run_ranks  # noqa: E402

pytestmark = pytest.mark.gpu


def _worker(rank, world, B, R):
    from tensorflow_distributed_amd import _native
    from tensorflow_distributed_amd.models import mnist_cnn as M

    _native.require()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = torch.classes.tfd.MnistEngine(B, 0, 1.0, 5, 0)
    eng.set_adam(0.01, 0.9, 0.999, 1e-8)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(B, 784, generator=g)
    y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)
    s = torch.cuda.Stream()
    first, worst = None, 0.0
    with torch.cuda.stream(s):
        eng.params().copy_(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()}).to(dev))
        eng.sync_shadow()
        eng.feed_x().copy_(x.to(dev))
        eng.feed_y().copy_(y.to(dev))
        for _ in range(R):
            eng.grads().zero_()
            eng.forward(True)
            eng.backward_a()
            eng.backward_b()
            snap = torch.cat([eng.pool1().float().flatten(), eng.hidden().float().flatten(), eng.grads()]).cpu()
            if first is None:
                first = snap
            else:
                worst = max(worst, (snap - first).abs().max().item())
    torch.cuda.synchronize()
    return worst, first


@pytest.mark.parametrize("world", [1, 4])
def test_step_bit_reproducible_under_gpu_sharing(cuda, world):
    res = run_ranks(_worker, world, 16, 25, timeout=300)
    for r, (worst, first) in enumerate(res):
        assert worst == 0.0, f"rank {r}: repeats differ by up to {worst}"
        assert torch.equal(first, res[0][1]), f"rank {r} differs from rank 0"
