"""Same-hardware vendor-library baseline: the same training steps as bench.py / bench_resnet.py,
written as plain PyTorch-ROCm (MIOpen convolutions, hipBLASLt GEMMs, torch fused Adam/SGD,
bf16 autocast, channels_last), optionally captured in a torch CUDA graph.

This is what a user would get on an MI355X without this framework's kernels; it is the bar the
native path has to beat (docs/DESIGN.md section 7). Nothing here is used by the framework.

    python tools/bench_torch_ref.py --model mnist --batch_size 128 --steps 200
    python tools/bench_torch_ref.py --model resnet50 --batch_size 64 --steps 10
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class MnistCNN(nn.Module):
    """Reference conv_net (mnist_python_m.py:104-128) in NCHW torch layers."""

    def __init__(self, keep_prob=0.75):
        super().__init__()
        self.c1 = nn.Conv2d(1, 32, 5, padding=2)
        self.c2 = nn.Conv2d(32, 64, 5, padding=2)
        self.fc1 = nn.Linear(3136, 1024)
        self.out = nn.Linear(1024, 10)
        self.p = 1.0 - keep_prob
        for t in self.parameters():  # reference init: N(0,1) everywhere (Q6)
            nn.init.normal_(t)

    def forward(self, x):
        x = x.view(-1, 1, 28, 28)
        x = F.max_pool2d(F.relu(self.c1(x)), 2)
        x = F.max_pool2d(F.relu(self.c2(x)), 2)
        x = F.relu(self.fc1(x.flatten(1)))
        x = F.dropout(x, self.p, self.training)
        return self.out(x)


class Bottleneck(nn.Module):
    def __init__(self, cin, mid, stride):
        super().__init__()
        cout = mid * 4
        self.c1, self.b1 = nn.Conv2d(cin, mid, 1, bias=False), nn.BatchNorm2d(mid)
        self.c2, self.b2 = nn.Conv2d(mid, mid, 3, stride, 1, bias=False), nn.BatchNorm2d(mid)
        self.c3, self.b3 = nn.Conv2d(mid, cout, 1, bias=False), nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = F.relu(self.b2(self.c2(y)))
        y = self.b3(self.c3(y))
        return F.relu(y + (x if self.down is None else self.down(x)))


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1, self.b1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False), nn.BatchNorm2d(cout)
        self.c2, self.b2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False), nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = self.b2(self.c2(y))
        return F.relu(y + (x if self.down is None else self.down(x)))


class ResNet(nn.Module):
    """ResNet v1.5 (stride on the 3x3), same topology as models/resnet.py."""

    def __init__(self, depth=50, num_classes=1000):
        super().__init__()
        layers = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3]}[depth]
        bott = depth >= 50
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        blocks, cin = [], 64
        for i, n in enumerate(layers):
            mid = 64 * 2 ** i
            for j in range(n):
                s = 2 if (j == 0 and i > 0) else 1
                if bott:
                    blocks.append(Bottleneck(cin, mid, s))
                    cin = mid * 4
                else:
                    blocks.append(BasicBlock(cin, mid, s))
                    cin = mid
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = self.blocks(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mnist", choices=["mnist", "resnet18", "resnet50"])
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--graph", type=int, default=1, help="capture the step in a torch CUDA graph")
    ap.add_argument("--compile", action="store_true", help="torch.compile the model (inductor)")
    a = ap.parse_args(argv)
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    B = a.batch_size
    if a.model == "mnist":
        model = MnistCNN().to(dev)
        opt = torch.optim.Adam(model.parameters(), lr=0.01, fused=True, capturable=bool(a.graph))
        x = torch.rand(B, 784, device=dev)
        y = torch.randint(0, 10, (B,), device=dev)
    else:
        model = ResNet(int(a.model[6:])).to(dev).to(memory_format=torch.channels_last)
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, fused=True)
        x = torch.randn(B, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (B,), device=dev)
    model.train()
    fwd = torch.compile(model) if a.compile else model

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(fwd(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        return loss

    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    if a.graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = step()
        run = lambda: g.replay()  # noqa: E731
    else:
        run = step
    for _ in range(a.warmup):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": f"images/sec PyTorch-ROCm reference path ({a.model})", "value": round(B * a.steps / dt, 1),
                      "unit": "images/s", "ms_per_step": round(dt * 1e3 / a.steps, 4), "batch": B,
                      "graph": bool(a.graph), "compile": a.compile, "dtype": "bf16 autocast",
                      "torch": torch.__version__}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
