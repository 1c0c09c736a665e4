"""Asynchronous parameter-server data parallelism (``--sync_replicas=False``,
``/root/reference/mnist_python_m.py:72-75, 247-253``).

Each PS task owns the variables ``replica_device_setter`` places on it (round-robin over PS tasks
in creation order, ``global_step`` first, so it lives on ps:0) and their optimizer slots. A worker
step is Hogwild-style, exactly like TF1's unsynchronised ApplyAdam on the PS:

    worker: fwd+bwd on its device -> for each PS shard: send PUSH(grad shard) -> recv fresh params
    PS    : recv from any worker -> apply the optimizer to its shard (no aggregation, stale reads
            allowed) -> global_step += 1 (ps:0) -> send the updated shard back

Transport: the Gloo control group (point-to-point ``send``/``recv`` with a 4-int header). The PS
keeps its shards on CPU (the reference's ``ps_device="/job:ps/cpu:0"``). Protocol ops: INIT (chief
uploads the initial values), PULL (fetch only), PUSH (apply then fetch), STOP (worker finished).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch
import torch.distributed as dist

from ..training.optimizers import FlatApplier

OP_INIT, OP_PULL, OP_PUSH, OP_STOP = 1, 2, 3, 4


class ShardLayout:
    """Which flat-buffer ranges (one per variable) each PS task owns."""

    def __init__(self, var_ranges: Sequence[Tuple[str, int, int]], num_ps: int, var_order: Sequence[str]):
        # round-robin in creation order; index 0 is global_step (a scalar kept by ps:0)
        self.num_ps = num_ps
        owner = {name: (i + 1) % num_ps for i, name in enumerate(var_order)}
        self.ranges: Dict[int, List[Tuple[str, int, int]]] = {p: [] for p in range(num_ps)}
        for name, off, n in var_ranges:
            self.ranges[owner[name]].append((name, off, n))
        self.sizes = {p: sum(n for _, _, n in r) for p, r in self.ranges.items()}

    def gather(self, flat: torch.Tensor, ps: int) -> torch.Tensor:
        parts = [flat[off:off + n] for _, off, n in self.ranges[ps]]
        return torch.cat(parts) if parts else flat.new_zeros(0)

    def scatter(self, flat: torch.Tensor, ps: int, shard: torch.Tensor) -> None:
        o = 0
        for _, off, n in self.ranges[ps]:
            flat[off:off + n].copy_(shard[o:o + n])
            o += n


def mnist_layout(num_ps: int) -> ShardLayout:
    from ..models import mnist_cnn as M

    ranges = []
    for key, tf_name, shape in M.PARAM_SPECS:
        n = 1
        for s in shape:
            n *= s
        ranges.append((tf_name, M.OFFSETS[key], n))
    order = [tf for _, tf, _ in M.PARAM_SPECS]
    return ShardLayout(ranges, num_ps, order)


class ParameterServerService:
    """The body of ``server.join()`` on a PS task in async mode."""

    def __init__(self, ps_index: int, num_ps: int, num_workers: int, layout: ShardLayout, optimizer):
        self.ps = ps_index
        self.num_workers = num_workers
        self.layout = layout
        self.num_ps = num_ps
        n = layout.sizes[ps_index]
        self.params = torch.zeros(n, dtype=torch.float32)
        self.applier = FlatApplier(optimizer, n)
        self.global_step = 0
        self.initialized = False
        self.updates = 0

    def serve(self) -> None:
        stopped = 0
        hdr = torch.zeros(4, dtype=torch.int64)
        n = self.params.numel()
        buf = torch.zeros(n, dtype=torch.float32)
        pending_pulls = []
        while stopped < self.num_workers:
            src = dist.recv(hdr)
            op, wk = int(hdr[0]), int(hdr[1])
            if op == OP_STOP:
                stopped += 1
                continue
            if op == OP_INIT:
                if n:
                    dist.recv(buf, src=src)
                self.params.copy_(buf)
                self.global_step = int(hdr[2])
                self.applier.t = int(hdr[3])
                self.initialized = True
                for p in pending_pulls:
                    self._reply(p)
                pending_pulls = []
                continue
            if op == OP_PUSH:
                if n:
                    dist.recv(buf, src=src)
                self.applier.apply(self.params, buf)
                self.updates += 1
                if self.ps == 0:
                    self.global_step += 1
            if not self.initialized:
                pending_pulls.append(src)  # non-chief waiting for the chief's init (Supervisor wait)
                continue
            self._reply(src)

    def _reply(self, dst: int) -> None:
        out = torch.tensor([self.global_step, self.applier.t, 0, 0], dtype=torch.int64)
        dist.send(out, dst)
        if self.params.numel():
            dist.send(self.params, dst)


class AsyncPSClient:
    """Worker side of the protocol; PS task p has global rank p."""

    def __init__(self, worker_index: int, layout: ShardLayout):
        self.worker = worker_index
        self.layout = layout
        self.global_step = 0

    def _targets(self) -> List[int]:
        # ps:0 always takes part (it keeps global_step); others only if they own variables
        return [p for p in range(self.layout.num_ps) if p == 0 or self.layout.sizes[p] > 0]

    def _exchange(self, op: int, flat_params: torch.Tensor, flat_grad: torch.Tensor = None, step: int = 0,
                  t: int = 0) -> None:
        targets = self._targets()
        for p in targets:
            dist.send(torch.tensor([op, self.worker, step, t], dtype=torch.int64), p)
            if self.layout.sizes[p] == 0:
                continue
            if op == OP_INIT:
                dist.send(self.layout.gather(flat_params, p).contiguous(), p)
            elif op == OP_PUSH:
                dist.send(self.layout.gather(flat_grad, p).contiguous(), p)
        if op == OP_INIT:
            return
        for p in targets:
            hdr = torch.zeros(4, dtype=torch.int64)
            dist.recv(hdr, src=p)
            if self.layout.sizes[p]:
                shard = torch.zeros(self.layout.sizes[p], dtype=torch.float32)
                dist.recv(shard, src=p)
                self.layout.scatter(flat_params, p, shard)
            if p == 0:
                self.global_step = int(hdr[0])

    def init(self, flat_params_cpu: torch.Tensor, step: int = 0, t: int = 0) -> None:
        self._exchange(OP_INIT, flat_params_cpu, step=step, t=t)

    def pull(self, flat_params_cpu: torch.Tensor) -> int:
        self._exchange(OP_PULL, flat_params_cpu)
        return self.global_step

    def push_pull(self, flat_params_cpu: torch.Tensor, flat_grad_cpu: torch.Tensor) -> int:
        self._exchange(OP_PUSH, flat_params_cpu, flat_grad_cpu)
        return self.global_step

    def stop(self) -> None:
        for p in self._targets():
            dist.send(torch.tensor([OP_STOP, self.worker, 0, 0], dtype=torch.int64), p)
