"""bench_resnet's probe flow in ONE process: reducer rebuilt (set_comm), two eager steps, the step
captured and replayed, the graph dropped -- repeated. comm: none | ipc1 (a world-1 IpcComm, forced DP)
| rccl1 (a world-1 RcclComm) | stub1 (a torch-op stand-in for the collective: copy / in-place scale).
TFD_LOOP_FP32=1: fp32 wire (in-place all_reduce instead of the bf16 all_reduce_into).
Bisection of the host-heap corruption (round 5): TFD_LOOP_NOSTREAM=1 drops the reducer's comm stream
(no event hand-offs, no side-stream work); TFD_LOOP_DEFER=1 keeps the side stream but issues every
bucket's hand-off (event record, stream wait, collective) from the main thread after backward()
instead of from inside the autograd engine's backward thread; TFD_LOOP_SPLIT=1 records each bucket's
ready event inside backward (the overlap point on the compute stream) but issues the side-stream wait and
the collective from the main thread after backward()."""
import os
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
if os.environ.get("TFD_LOOP_SPLIT") == "1":
    from tensorflow_distributed_amd.models import resnet as _R

    _orig_finish2 = _R.BucketReducer.finish

    def _mark_ready2(self, name):
        b = self.bucket_of[name]
        self.count[b] += 1
        if self.count[b] == self.need[b] and self.stream is not None:
            self.bucket_events[b].record(torch.cuda.current_stream(self.fp.device))
            self.__dict__.setdefault("_pending", []).append(b)

    def _finish2(self):
        for b in self.__dict__.pop("_pending", []):
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(self.bucket_events[b])
                lo, hi = self.buckets[b]
                c = self.bucket_comm[b]
                if self.bf16 and hasattr(c, "all_reduce_into"):
                    c.all_reduce_into(self.fp.grad[lo:hi], self.gbf[lo:hi], "sum")
                elif self.bf16:
                    self.gbf[lo:hi].copy_(self.fp.grad[lo:hi])
                    c.all_reduce(self.gbf[lo:hi], "sum")
                else:
                    c.all_reduce(self.fp.grad[lo:hi], "sum")
            self.launched += 1
        _orig_finish2(self)

    _R.BucketReducer.mark_ready = _mark_ready2
    _R.BucketReducer.finish = _finish2
if os.environ.get("TFD_LOOP_DEFER") == "1":
    from tensorflow_distributed_amd.models import resnet as _R

    _orig_finish = _R.BucketReducer.finish

    def _mark_ready(self, name):
        b = self.bucket_of[name]
        self.count[b] += 1
        if self.count[b] == self.need[b] and self.stream is not None:
            self.__dict__.setdefault("_pending", []).append(b)

    def _finish(self):
        for b in self.__dict__.pop("_pending", []):
            ev = self.bucket_events[b]
            ev.record(torch.cuda.current_stream(self.fp.device))
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                lo, hi = self.buckets[b]
                c = self.bucket_comm[b]
                if self.bf16 and hasattr(c, "all_reduce_into"):
                    c.all_reduce_into(self.fp.grad[lo:hi], self.gbf[lo:hi], "sum")
                elif self.bf16:
                    self.gbf[lo:hi].copy_(self.fp.grad[lo:hi])
                    c.all_reduce(self.gbf[lo:hi], "sum")
                else:
                    c.all_reduce(self.fp.grad[lo:hi], "sum")
            self.launched += 1
        _orig_finish(self)

    _R.BucketReducer.mark_ready = _mark_ready
    _R.BucketReducer.finish = _finish
dev = torch.device("cuda", 0)
m = ResNet(18, num_classes=1000, device=dev, seed=0)
m.masked_join = bool(masked)
print(f"mode {mode} slots {torch.ops.tfd.bn_part_slots()} masked {m.masked_join}", flush=True)
comm = None
if mode == "ipc1":
    from tensorflow_distributed_amd.parallel.ipc import IpcCollectives, make_ipc_comm

    comm = IpcCollectives(make_ipc_comm(0, 1, 0, m.fp.total))
elif mode == "stub1":
    class _Stub:  # the collective as plain torch ops on the caller's (comm) stream
        def world(self):
            return 1

        def all_reduce(self, t, op="sum"):
            t.mul_(1.0)

        def all_reduce_into(self, src, dst, op="sum"):
            dst.copy_(src)

    comm = _Stub()
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
        m.set_comm(comm, [0.5, 2.0][it % 2], force_dp=True, bf16_grads=os.environ.get("TFD_LOOP_FP32") != "1")
        if os.environ.get("TFD_LOOP_NOSTREAM") == "1":
            m.reducer.stream = None
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
    graph = torch.cuda.CUDAGraph(keep_graph=it == 0)
    with torch.cuda.graph(graph):
        out = m.train_step(x, y, lr=0.1)
    if it == 0:  # what the captured step is made of (kernel / memcpy / memset / event nodes ...)
        c = torch.ops.tfd.graph_node_types(int(graph.raw_cuda_graph())).tolist()
        names = ["kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event", "event_record"]
        print("graph nodes: " + ", ".join(f"{names[i] if i < len(names) else i}={v}" for i, v in enumerate(c) if v),
              flush=True)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize(dev)
    if keep:
        kept.append(graph)
    del graph, out
    if it % 10 == 0:
        print(f"iter {it} ok", flush=True)
print("done", flush=True)
