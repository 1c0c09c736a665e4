"""Parameter-server data parallelism: the asynchronous mode (``--sync_replicas=False``,
``/root/reference/mnist_python_m.py:72-75, 247-253``) and the
synchronous mode WITH BACKUP WORKERS (``replicas_to_aggregate < num_workers``,
``/root/reference/mnist_python_m.py:62-65, 210-233``).

Each PS task owns the variables ``replica_device_setter`` places on it (round-robin over PS tasks
in creation order, ``global_step`` first, so it lives on ps:0) and their optimizer slots, on CPU
(the reference's ``ps_device="/job:ps/cpu:0"``).

* **async** -- Hogwild, exactly TF1's unsynchronised ApplyAdam on the PS:
  ``worker: fwd+bwd -> PUSH(grad shard) -> recv fresh params``;
  ``PS: apply the optimizer to its shard at once (stale reads allowed), global_step += 1 (ps:0)``.
* **sync** (backup workers) -- TF1's ``SyncReplicasOptimizer`` accumulator semantics, per shard:
  a PUSH carries the worker's ``local_step`` (the global step its parameters came from). A fresh
  gradient (``local_step == step``) is accumulated while fewer than ``R`` have arrived; the R-th
  triggers ONE averaged update (``sum / R``), ``step += 1`` and the reply to every contributor
  (their "token"). A stale gradient (``local_step < step``: a straggler that lost the race) is
  DROPPED and answered at once with the fresh parameters, so the straggler rejoins the next step
  without the fast workers ever waiting for it -- only for the first ``R`` arrivals.

Transport: the Gloo control group (point-to-point ``send``/``recv`` with a 4-int header). Ops:
INIT (chief uploads values, optionally optimizer slots), PULL (fetch), PUSH (gradient), STOP
(worker finished), PULL_STATE (parameters + optimizer slots + update count: the chief's
Supervisor checkpoints what the PS actually holds, so a restart resumes Adam with its moments).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..training.optimizers import FlatApplier

OP_INIT, OP_PULL, OP_PUSH, OP_STOP, OP_PULL_STATE = 1, 2, 3, 4, 5


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
    """The body of ``server.join()`` on a PS task (async, or sync with ``replicas_to_aggregate``)."""

    def __init__(self, ps_index: int, num_ps: int, num_workers: int, layout: ShardLayout, optimizer,
                 sync: bool = False, replicas_to_aggregate: Optional[int] = None):
        self.ps = ps_index
        self.num_workers = num_workers
        self.layout = layout
        self.num_ps = num_ps
        n = layout.sizes[ps_index]
        self.params = torch.zeros(n, dtype=torch.float32)
        self.applier = FlatApplier(optimizer, n)
        self.global_step = 0   # ps:0: the global step; other shards: their update count (equal in sync mode)
        self.initialized = False
        self.updates = 0
        self.sync = sync
        self.r2a = replicas_to_aggregate or num_workers
        self.accum = torch.zeros(n, dtype=torch.float32) if sync else None
        self.count = 0
        self.waiting: List[int] = []
        self.dropped = 0       # stale (straggler) gradients discarded

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
                for slot in self.applier.slots().values():  # hdr[3] = t; slots follow when hdr[1] < 0
                    if wk < 0 and n:
                        dist.recv(slot, src=src)
                    elif wk >= 0:
                        slot.zero_()
                self.global_step = int(hdr[2])
                self.applier.t = int(hdr[3])
                self.initialized = True
                for p in pending_pulls:
                    self._reply(p)
                pending_pulls = []
                continue
            if op == OP_PULL_STATE:
                self._reply(src, state=True)
                continue
            if op == OP_PUSH:
                if n:
                    dist.recv(buf, src=src)
                if self.sync:
                    local_step = int(hdr[2])
                    if local_step == self.global_step and self.count < self.r2a:
                        self.accum.add_(buf)
                        self.count += 1
                        self.waiting.append(src)
                        if self.count == self.r2a:
                            self.applier.apply(self.params, self.accum, 1.0 / self.r2a)
                            self.updates += 1
                            self.global_step += 1
                            self.accum.zero_()
                            self.count = 0
                            for w in self.waiting:
                                self._reply(w)
                            self.waiting = []
                    else:
                        self.dropped += 1
                        self._reply(src, dropped=True)
                    continue
                self.applier.apply(self.params, buf)
                self.updates += 1
                if self.ps == 0:
                    self.global_step += 1
            if not self.initialized:
                pending_pulls.append(src)  # non-chief waiting for the chief's init (Supervisor wait)
                continue
            self._reply(src)

    def _reply(self, dst: int, dropped: bool = False, state: bool = False) -> None:
        out = torch.tensor([self.global_step, self.applier.t, int(dropped), self.dropped], dtype=torch.int64)
        dist.send(out, dst)
        if self.params.numel():
            dist.send(self.params, dst)
            if state:
                for slot in self.applier.slots().values():
                    dist.send(slot, dst)


class AsyncPSClient:
    """Worker side of the protocol; PS task p has global rank p."""

    def __init__(self, worker_index: int, layout: ShardLayout, slot_names: Sequence[str] = ()):
        self.worker = worker_index
        self.layout = layout
        self.global_step = 0
        self.t = 0
        self.last_dropped = False   # sync mode: was this worker's last gradient stale (dropped)?
        self.dropped_total = 0      # ps:0's count of dropped stale gradients
        self.slot_names = list(slot_names)

    def _targets(self) -> List[int]:
        # ps:0 always takes part (it keeps global_step); others only if they own variables
        return [p for p in range(self.layout.num_ps) if p == 0 or self.layout.sizes[p] > 0]

    def _exchange(self, op: int, flat_params: torch.Tensor, flat_grad: torch.Tensor = None, step: int = 0,
                  t: int = 0, slots: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
        targets = self._targets()
        who = -1 - self.worker if (op == OP_INIT and slots) else self.worker
        for p in targets:
            dist.send(torch.tensor([op, who, step, t], dtype=torch.int64), p)
            if self.layout.sizes[p] == 0:
                continue
            if op == OP_INIT:
                dist.send(self.layout.gather(flat_params, p).contiguous(), p)
                for name in self.slot_names if slots else ():
                    dist.send(self.layout.gather(slots[name], p).contiguous(), p)
            elif op == OP_PUSH:
                dist.send(self.layout.gather(flat_grad, p).contiguous(), p)
        got_slots: Dict[str, torch.Tensor] = {}
        if op == OP_INIT:
            return got_slots
        if op == OP_PULL_STATE:
            got_slots = {name: torch.zeros_like(flat_params) for name in self.slot_names}
        dropped = False
        for p in targets:
            hdr = torch.zeros(4, dtype=torch.int64)
            dist.recv(hdr, src=p)
            dropped = dropped or bool(hdr[2])
            if self.layout.sizes[p]:
                shard = torch.zeros(self.layout.sizes[p], dtype=torch.float32)
                dist.recv(shard, src=p)
                self.layout.scatter(flat_params, p, shard)
                if op == OP_PULL_STATE:
                    for name in self.slot_names:
                        dist.recv(shard, src=p)
                        self.layout.scatter(got_slots[name], p, shard)
            if p == 0:
                self.global_step = int(hdr[0])
                self.t = int(hdr[1])
                self.dropped_total = int(hdr[3])
        self.last_dropped = dropped
        return got_slots

    def init(self, flat_params_cpu: torch.Tensor, step: int = 0, t: int = 0,
             slots: Optional[Dict[str, torch.Tensor]] = None) -> None:
        """Chief: upload the initial (or restored) values; with ``slots`` also the optimizer moments."""
        self._exchange(OP_INIT, flat_params_cpu, step=step, t=t, slots=slots)

    def pull(self, flat_params_cpu: torch.Tensor) -> int:
        self._exchange(OP_PULL, flat_params_cpu)
        return self.global_step

    def push_pull(self, flat_params_cpu: torch.Tensor, flat_grad_cpu: torch.Tensor, local_step: int = 0) -> int:
        """Send a gradient computed at ``local_step``; returns the fresh global step (params updated)."""
        self._exchange(OP_PUSH, flat_params_cpu, flat_grad_cpu, step=local_step)
        return self.global_step

    def pull_state(self, flat_params_cpu: torch.Tensor) -> Tuple[Dict[str, torch.Tensor], int, int]:
        """Parameters (into ``flat_params_cpu``), optimizer slots, ps:0's update count t and step."""
        slots = self._exchange(OP_PULL_STATE, flat_params_cpu)
        return slots, self.t, self.global_step

    def stop(self) -> None:
        for p in self._targets():
            dist.send(torch.tensor([OP_STOP, self.worker, 0, 0], dtype=torch.int64), p)
