"""bench_resnet's probe flow in ONE process: reducer rebuilt (set_comm), two eager steps, the step
captured and replayed, the graph dropped -- repeated. comm: none | ipc1 (a world-1 IpcComm, forced DP)."""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_amd import _native  # noqa: E402

_native.require()
from tensorflow_distributed_amd.models.resnet import ResNet  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "none"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 30
slots = int(sys.argv[3]) if len(sys.argv) > 3 else -1
masked = int(sys.argv[4]) if len(sys.argv) > 4 else 1
if slots >= 0:
    torch.ops.tfd.set_bn_part_slots(slots)
dev = torch.device("cuda", 0)
m = ResNet(18, num_classes=1000, device=dev, seed=0)
m.masked_join = bool(masked)
print(f"mode {mode} slots {torch.ops.tfd.bn_part_slots()} masked {m.masked_join}", flush=True)
comm = None
if mode == "ipc1":
    from tensorflow_distributed_amd.parallel.ipc import IpcCollectives, make_ipc_comm

    comm = IpcCollectives(make_ipc_comm(0, 1, 0, m.fp.total))
elif mode == "rccl1":
    uid = torch.classes.tfd.RcclComm.unique_id()
    comm = torch.classes.tfd.RcclComm(uid, 1, 0, 0)
nograph = len(sys.argv) > 5 and sys.argv[5] == "nograph"
keep = len(sys.argv) > 5 and sys.argv[5] == "keep"  # never destroy a captured graph
kept = []
g = torch.Generator(device=dev).manual_seed(100)
x = torch.randn(8, 64, 64, 3, device=dev, generator=g)
y = torch.randint(0, 1000, (8,), device=dev, generator=g, dtype=torch.int32)
s = torch.cuda.Stream(dev)
for it in range(iters):
    if comm is not None:
        m.set_comm(comm, [0.5, 2.0][it % 2], force_dp=True)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(2):
            m.train_step(x, y, lr=0.1)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    if nograph:
        if it % 10 == 0:
            print(f"iter {it} ok", flush=True)
        continue
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = m.train_step(x, y, lr=0.1)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize(dev)
    if keep:
        kept.append(graph)
    del graph, out
    if it % 10 == 0:
        print(f"iter {it} ok", flush=True)
print("done", flush=True)
