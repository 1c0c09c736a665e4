"""Replays a captured ResNet-18 step graph built in BN slot mode, switching the process to row mode
after two replays, with the width-paired stem on and off (tests/test_resnet_gpu.py
test_captured_graph_keeps_its_bn_mode, split by stem form)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from tensorflow_distributed_amd import _native  # noqa: E402
from tensorflow_distributed_amd.models.resnet import ResNet  # noqa: E402


def run(stem_w2, switch, x, lab, cuda):
    torch.ops.tfd.set_bn_part_slots(4)
    m = ResNet(18, num_classes=16, device=cuda, seed=3, width=16, stem_w2=stem_w2)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            m.train_step(x, lab, lr=0.01)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = m.train_step(x, lab, lr=0.01)
    losses = []
    for i in range(4):
        if switch and i == 2:
            torch.ops.tfd.set_bn_part_slots(0)
        g.replay()
        torch.cuda.synchronize()
        losses.append(round(float(out.item()), 5))
        gs = m.stem.g()
        print(f"   replay {i}: stem grad |g| {float(gs.norm()):.6f} ch0-2 {float(gs[:, :, :3].norm()):.6f} "
              f"flat |g| {float(m.fp.grad.norm()):.6f} master |w| {float(m.fp.master.norm()):.4f}"
              + (f" paired |g| {float(m.stem.paired_g.norm()):.6f}" if m.stem.paired_g is not None else ""), flush=True)
    return losses


def run_eager(stem_w2, x, lab, cuda, steps=6):
    torch.ops.tfd.set_bn_part_slots(4)
    m = ResNet(18, num_classes=16, device=cuda, seed=3, width=16, stem_w2=stem_w2)
    out = []
    for _ in range(steps):
        out.append(round(float(m.train_step(x, lab, lr=0.01).item()), 5))
    return out


def main():
    _native.require()
    cuda = torch.device("cuda", 0)
    torch.manual_seed(31)
    x = torch.randn(8, 32, 32, 3, device=cuda)
    lab = torch.randint(0, 16, (8,), dtype=torch.int32, device=cuda)
    old = torch.ops.tfd.bn_part_slots()
    for stem_w2 in (False, True):
        print(f"eager stem_w2={stem_w2}: {run_eager(stem_w2, x, lab, cuda)}", flush=True)
    for stem_w2 in (False, True):
        for switch in (False, True):
            print(f"stem_w2={stem_w2} switch={switch}: {run(stem_w2, switch, x, lab, cuda)}", flush=True)
    torch.ops.tfd.set_bn_part_slots(old)


if __name__ == "__main__":
    main()
