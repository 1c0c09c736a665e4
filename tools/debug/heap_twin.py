"""Torch-only twin of the ResNet DP capture cycle: is the host-heap
corruption seen after destroying a captured two-stream step graph the platform's or ours?

The cycle of tools/debug/rn_configure_loop.py with every tfd piece replaced by plain torch ops:
a chain of convs/matmuls on the compute stream stands in for the backward; each "bucket" records an
event on the compute stream, the comm stream waits on it and runs a torch copy + add (the stand-in
for the collective), and a join event brings the comm stream back. Per cycle: rebuild the "reducer"
(new comm stream, new buffers), two eager steps, capture the step, replay 3x, drop the graph.

    python -X faulthandler tools/debug/heap_twin.py [pooled|fresh] [iters] [keep|drop]

pooled: one event set for the process (as models/resnet.py now does); fresh: new torch.cuda.Event
objects per step (the round-3 code). Run under MALLOC_CHECK_=3 so glibc aborts at the first bad free.
"""
import sys

import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "pooled"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 60
keep = (sys.argv[3] if len(sys.argv) > 3 else "drop") == "keep"
dev = torch.device("cuda", 0)
NB = 6
pool_events = [torch.cuda.Event() for _ in range(NB + 1)]
w = [torch.randn(64, 64, 3, 3, device=dev) * 0.05 for _ in range(NB)]
x = torch.randn(8, 64, 32, 32, device=dev)
kept = []


class Reducer:
    def __init__(self):
        self.stream = torch.cuda.Stream(dev)
        self.grad = torch.zeros(NB, 1 << 16, device=dev)
        self.wire = torch.zeros(NB, 1 << 16, device=dev, dtype=torch.bfloat16)

    def step(self):
        cur = torch.cuda.current_stream(dev)
        h = x
        evs = pool_events if mode == "pooled" else [torch.cuda.Event() for _ in range(NB + 1)]
        for b in range(NB):
            h = torch.nn.functional.conv2d(h, w[b], padding=1).relu_()
            self.grad[b].copy_(h.flatten()[: 1 << 16])
            evs[b].record(cur)
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(evs[b])
                self.wire[b].copy_(self.grad[b])
                self.wire[b].add_(1.0)
        evs[NB].record(self.stream)
        cur.wait_event(evs[NB])
        return self.wire.float().sum()


s = torch.cuda.Stream(dev)
print(f"mode {mode} keep {keep}", flush=True)
for it in range(iters):
    r = Reducer()
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(2):
            r.step()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = r.step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize(dev)
    if keep:
        kept.append(g)
    del g, out, r
    if it % 10 == 0:
        print(f"iter {it} ok", flush=True)
print("done", flush=True)
