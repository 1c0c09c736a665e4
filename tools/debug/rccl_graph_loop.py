"""Host-heap check of captured RCCL collectives: capture a graph whose only work is a side-stream
RCCL all-reduce (plus the copy feeding it), replay it, destroy it -- repeated -- under glibc's heap
checks (run with MALLOC_CHECK_=3 MALLOC_PERTURB_=165).
  mode ours : the framework's RcclComm (csrc/runtime/comm.cpp: a HIP user object per captured call)
  mode torch: torch.distributed's RCCL ("nccl") process group at world 1 (no tfd code involved)
Argument 2: cycles; argument 3: 'sync' = synchronize + sleep 10 ms after each graph's destruction."""
import os
import sys
import time

import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "ours"
cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 100
settle = len(sys.argv) > 3 and sys.argv[3] == "sync"
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
if mode == "ours":
    sys.path.insert(0, ".")
    from tensorflow_distributed_amd import _native

    _native.require()
    comm = torch.classes.tfd.RcclComm(torch.classes.tfd.RcclComm.unique_id(), 1, 0, 0)
    ar = lambda t: comm.all_reduce(t, "sum")  # noqa: E731
else:
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    ar = lambda t: dist.all_reduce(t)  # noqa: E731
src = torch.randn(1 << 20, device=dev)
buf = torch.empty(1 << 20, device=dev, dtype=torch.bfloat16)
side = torch.cuda.Stream(dev)
cap = torch.cuda.Stream(dev)
for it in range(cycles):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        side.wait_stream(cap)
        with torch.cuda.stream(side):
            buf.copy_(src)
            ar(buf)
        cap.wait_stream(side)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    del g
    if settle:
        torch.cuda.synchronize()
        time.sleep(0.01)
    if it % 20 == 0:
        print(f"iter {it} ok", flush=True)
print("done", flush=True)
