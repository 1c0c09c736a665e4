"""GPU-resident parameter server: the async (``--sync_replicas=False``) and backup-worker
(``replicas_to_aggregate < num_workers``) modes with the variables, optimizer slots and the
sync-mode accumulator on the PS task's GPU (VERDICT r2 "next round" item 6; reference roles
``/root/reference/mnist_python_m.py:72-75, 164-177, 210-222, 247-253``).

Same protocol and semantics as the host PS of :mod:`.async_ps` (round-robin variable sharding over
PS tasks, Hogwild updates, TF's accumulator that averages the first R fresh gradients of a step and
drops stale ones) -- only the data plane moved:

* **push**: the worker copies the ranges of its fp32 gradient that PS p owns into its mailbox slot
  on PS p's GPU (``GpuPsPort.push_grad``: device-to-device copies into IPC-mapped memory), then sends
  a 32-byte Gloo header ``[PUSH, worker, local_step, 0]``;
* **update**: the PS runs the flat optimizer kernel on the mailbox slot (async) or accumulates it
  (sync, ``csrc/kernels/optim.hip``) -- no host-side arithmetic;
* **pull**: the PS writes its updated ranges straight into the worker's engine parameters
  (``GpuPsShard.push``) and replies with ``[global_step, t, dropped, dropped_total]``; the worker
  refreshes its bf16 shadow.

Only checkpointing (``pull_state``) and restoring slots move tensors through the host, as TF's
Saver would. Setup: each worker sends HELLO + the IPC export of its parameter buffer to every PS
that owns variables; the PS answers with the export of its mailbox and the slot size.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .async_ps import OP_INIT, OP_PULL, OP_PULL_STATE, OP_PUSH, OP_STOP, ShardLayout

OP_HELLO = 6
EXPORT_BYTES = 80  # hipIpcMemHandle_t (64) + offset + size (csrc/runtime/gpu_ps.cpp)
OPT_KIND = {"adam": 0, "sgd": 1, "momentum": 2}


def _ranges_tensor(layout: ShardLayout, ps: int) -> torch.Tensor:
    r = [[off, n] for _, off, n in layout.ranges[ps]]
    return torch.tensor(r if r else [[0, 0]], dtype=torch.int64)


def _opt_args(opt):
    kind = OPT_KIND[opt.kind]
    if opt.kind == "momentum" and getattr(opt, "use_nesterov", False):
        kind = 3
    return (kind, float(opt.learning_rate), float(getattr(opt, "beta1", 0.9)), float(getattr(opt, "beta2", 0.999)),
            float(getattr(opt, "epsilon", 1e-8)), float(getattr(opt, "momentum", 0.0)))


class GpuParameterServerService:
    """The body of ``server.join()`` on a PS task whose shard lives on ``device``."""

    def __init__(self, ps_index: int, num_ps: int, num_workers: int, layout: ShardLayout, optimizer,
                 device: torch.device, sync: bool = False, replicas_to_aggregate: Optional[int] = None):
        from .. import _native
        from ..training.optimizers import base_optimizer

        _native.require()
        self.ps = ps_index
        self.num_workers = num_workers
        self.layout = layout
        self.opt = base_optimizer(optimizer)
        self.device = device
        self.sync = sync
        self.r2a = replicas_to_aggregate or num_workers
        from ..models import mnist_cnn as M

        self.shard = torch.classes.tfd.GpuPsShard(device.index, _ranges_tensor(layout, ps_index), M.TOTAL,
                                                  num_workers, *_opt_args(self.opt), bool(sync))
        self.n = layout.sizes[ps_index]
        self.slot_elems = (max(self.n, 4) + 3) // 4 * 4
        self.global_step = 0
        self.initialized = False
        self.updates = 0
        self.count = 0
        self.waiting: List[int] = []
        self.dropped = 0
        self.workers: Dict[int, int] = {}  # rank -> worker index

    @property
    def t(self) -> int:
        return int(self.shard.updates())

    def serve(self) -> None:
        stopped = 0
        hdr = torch.zeros(4, dtype=torch.int64)
        ex = torch.zeros(EXPORT_BYTES, dtype=torch.uint8)
        pending_pulls = []
        while stopped < self.num_workers:
            src = dist.recv(hdr)
            op, wk = int(hdr[0]), int(hdr[1])
            if op == OP_HELLO:
                dist.recv(ex, src=src)
                self.shard.open_worker(wk, ex)
                self.workers[src] = wk
                dist.send(torch.tensor([self.slot_elems, self.n, 0, 0], dtype=torch.int64), src)
                dist.send(self.shard.mailbox(), src)
                continue
            if op == OP_STOP:
                stopped += 1
                continue
            w = self.workers[src]
            if op == OP_INIT:
                self.shard.pull_init(w, int(hdr[3]))  # the chief's engine parameters, peer memory
                if wk < 0 and self.n:  # restored optimizer slots follow (host tensors, restore only)
                    slots = []
                    for _ in self._slot_names():
                        s = torch.zeros(self.n, dtype=torch.float32)
                        dist.recv(s, src=src)
                        slots.append(s.to(self.device))
                    m = slots[0] if slots else None
                    v = slots[1] if len(slots) > 1 else None
                    self.shard.load_state(self.shard.params().clone(), m, v, int(hdr[3]))
                self.global_step = int(hdr[2])
                self.initialized = True
                for p in pending_pulls:
                    self._reply(p)
                pending_pulls = []
                continue
            if op == OP_PULL_STATE:
                self._reply(src, state=True)
                continue
            if op == OP_PUSH:
                if self.sync:
                    local_step = int(hdr[2])
                    if local_step == self.global_step and self.count < self.r2a:
                        self.shard.accumulate(w)
                        self.count += 1
                        self.waiting.append(src)
                        if self.count == self.r2a:
                            self.shard.apply_accumulated(1.0 / self.r2a)
                            self.updates += 1
                            self.global_step += 1
                            self.count = 0
                            for dst in self.waiting:
                                self._reply(dst)
                            self.waiting = []
                    else:
                        self.dropped += 1
                        self._reply(src, dropped=True)
                    continue
                self.shard.apply(w, 1.0)
                self.updates += 1
                if self.ps == 0:
                    self.global_step += 1
            if not self.initialized:
                pending_pulls.append(src)  # a non-chief waiting for the chief's init
                continue
            self._reply(src)

    def _slot_names(self):
        return {"adam": ["m", "v"], "momentum": ["m"]}.get(self.opt.kind, [])

    def _reply(self, dst: int, dropped: bool = False, state: bool = False) -> None:
        if self.n and not state:
            self.shard.push(self.workers[dst])  # fresh values into the worker's engine, before the token
        dist.send(torch.tensor([self.global_step, self.t, int(dropped), self.dropped], dtype=torch.int64), dst)
        if state and self.n:
            dist.send(self.shard.params().cpu(), dst)
            for name in self._slot_names():
                dist.send((self.shard.slot_m() if name == "m" else self.shard.slot_v()).cpu(), dst)


class GpuPSClient:
    """Worker side; PS task p has global rank p. ``params`` is the worker engine's flat fp32
    parameter buffer (the PS tasks write into it); ``refresh`` re-derives whatever the engine keeps
    from it (the bf16 shadow) after every pull."""

    def __init__(self, worker_index: int, layout: ShardLayout, params: torch.Tensor, refresh, slot_names=()):
        self.worker = worker_index
        self.layout = layout
        self.params = params
        self.refresh = refresh
        self.slot_names = list(slot_names)
        self.global_step = 0
        self.t = 0
        self.last_dropped = False
        self.dropped_total = 0
        self.port = torch.classes.tfd.GpuPsPort(params.device.index, layout.num_ps)
        ex = self.port.export_buffer(params)
        for p in self._targets():
            dist.send(torch.tensor([OP_HELLO, worker_index, 0, 0], dtype=torch.int64), p)
            dist.send(ex, p)
            rep = torch.zeros(4, dtype=torch.int64)
            dist.recv(rep, src=p)
            mb = torch.zeros(EXPORT_BYTES, dtype=torch.uint8)
            dist.recv(mb, src=p)
            self.port.open_ps(p, mb, _ranges_tensor(layout, p), int(rep[0]))

    def _targets(self) -> List[int]:
        return [p for p in range(self.layout.num_ps) if p == 0 or self.layout.sizes[p] > 0]

    def _replies(self, state: bool = False, flat_cpu: Optional[torch.Tensor] = None):
        dropped = False
        got: Dict[str, torch.Tensor] = {}
        if state:
            got = {name: torch.zeros_like(flat_cpu) for name in self.slot_names}
        for p in self._targets():
            hdr = torch.zeros(4, dtype=torch.int64)
            dist.recv(hdr, src=p)
            dropped = dropped or bool(hdr[2])
            if state and self.layout.sizes[p]:
                shard = torch.zeros(self.layout.sizes[p], dtype=torch.float32)
                dist.recv(shard, src=p)
                self.layout.scatter(flat_cpu, p, shard)
                for name in self.slot_names:
                    dist.recv(shard, src=p)
                    self.layout.scatter(got[name], p, shard)
            if p == 0:
                self.global_step, self.t, self.dropped_total = int(hdr[0]), int(hdr[1]), int(hdr[3])
        self.last_dropped = dropped
        if not state:
            self.refresh()
        return got

    def init(self, step: int = 0, t: int = 0, slots: Optional[Dict[str, torch.Tensor]] = None) -> None:
        """Chief: the PS tasks read the initial (or restored) values from this worker's engine; with
        ``slots`` (restore) the optimizer moments follow as host tensors."""
        torch.cuda.synchronize(self.params.device)
        who = -1 - self.worker if slots else self.worker
        for p in self._targets():
            dist.send(torch.tensor([OP_INIT, who, step, t], dtype=torch.int64), p)
            if slots and self.layout.sizes[p]:
                for name in self.slot_names:
                    dist.send(self.layout.gather(slots[name], p).contiguous(), p)

    def pull(self) -> int:
        for p in self._targets():
            dist.send(torch.tensor([OP_PULL, self.worker, 0, 0], dtype=torch.int64), p)
        self._replies()
        return self.global_step

    def push_pull(self, grad: torch.Tensor, local_step: int = 0) -> int:
        """``grad``: the worker's flat fp32 gradient on its GPU (computed at ``local_step``). Returns
        the fresh global step; the engine parameters hold the fresh values."""
        for p in self._targets():
            if self.layout.sizes[p]:
                self.port.push_grad(p, self.worker, grad)
            dist.send(torch.tensor([OP_PUSH, self.worker, local_step, 0], dtype=torch.int64), p)
        self._replies()
        return self.global_step

    def pull_state(self, flat_params_cpu: torch.Tensor) -> Tuple[Dict[str, torch.Tensor], int, int]:
        """Checkpoint read: parameters (into ``flat_params_cpu``), slots, ps:0's update count, step."""
        for p in self._targets():
            dist.send(torch.tensor([OP_PULL_STATE, self.worker, 0, 0], dtype=torch.int64), p)
        got = self._replies(state=True, flat_cpu=flat_params_cpu)
        return got, self.t, self.global_step

    def stop(self) -> None:
        for p in self._targets():
            dist.send(torch.tensor([OP_STOP, self.worker, 0, 0], dtype=torch.int64), p)
