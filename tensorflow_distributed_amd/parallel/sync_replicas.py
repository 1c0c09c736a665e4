"""Synchronous data parallelism with ``SyncReplicasOptimizer`` semantics
(``/root/reference/mnist_python_m.py:210-233``).

TF1 aggregates ``replicas_to_aggregate`` fresh gradients per global step in PS-side
``ConditionalAccumulator``s and releases one token per worker after ApplyAdam. In the all-reduce
world that becomes:

* ``replicas_to_aggregate == total_num_replicas`` (the reference default, 2 of 2): one averaged
  all-reduce per step. On GPUs it is the native engine's bucketed RCCL all-reduce overlapped with
  the conv backward (``MnistEngine.train_step``); on CPUs a Gloo all-reduce of the flat gradient.
  The blocking collective is the token barrier (M4), and every rank applies the identical update,
  so ``global_step`` stays equal everywhere (M5).
* ``replicas_to_aggregate < total_num_replicas`` (backup workers): every worker computes its
  gradient and timestamps completion; a tiny all-gather of the timestamps picks the R earliest
  (rank breaks ties); contributors all-reduce ``1 * grad``, the others ``0 * grad``; everybody
  applies the sum scaled by ``1/R``. The dropped (slowest) gradients are exactly TF's stale ones.
"""
from __future__ import annotations

import time
from typing import Optional

import torch
import torch.distributed as dist


class GlooGradAverager:
    """CPU gradient averaging over a (worker) process group; in-place on the flat buffer."""

    def __init__(self, group=None, world: int = 1, splits=None):
        self.group = group
        self.world = world
        self.splits = sorted(splits or [])  # bucket boundaries (flat offsets); none = one bucket
        self.last_ms = 0.0  # host time of the last all-reduce (metrics JSONL: allreduce_ms)

    def __call__(self, flat_grad: torch.Tensor) -> None:
        if self.world > 1:
            t0 = time.perf_counter()
            edges = [0] + [e for e in self.splits if 0 < e < flat_grad.numel()] + [flat_grad.numel()]
            for lo, hi in zip(edges[:-1], edges[1:]):
                dist.all_reduce(flat_grad[lo:hi], group=self.group)
            flat_grad.div_(self.world)
            self.last_ms = (time.perf_counter() - t0) * 1e3


def select_contributors(finish_time: float, rank: int, world: int, replicas_to_aggregate: int, group=None):
    """All-gather finish times; return the sorted list of the R earliest worker ranks (0-based)."""
    t = torch.tensor([finish_time, float(rank)], dtype=torch.float64)
    if world == 1:
        return [0]
    allt = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(allt, t, group=group)
    order = sorted(range(world), key=lambda r: (allt[r][0].item(), allt[r][1].item()))
    return sorted(order[:replicas_to_aggregate])


class SyncReplicasStepper:
    """One global step of sync DP for a model runner (CPU or native GPU)."""

    def __init__(self, runner, worker_rank: int, num_workers: int, replicas_to_aggregate: int,
                 group=None, straggler_delay_s: Optional[dict] = None, splits=None):
        self.runner = runner
        self.rank = worker_rank
        self.world = num_workers
        self.r2a = replicas_to_aggregate
        self.group = group
        self.delay = straggler_delay_s or {}  # test hook: {worker_rank: seconds} artificial slowness
        self.last_contributors = list(range(num_workers))
        native = hasattr(runner, "eng")
        if not native and self.r2a == self.world:
            runner.comm = GlooGradAverager(group, num_workers, splits)  # splits: the "buckets" schedule

    def step(self, x, y) -> None:
        r = self.runner
        if self.r2a == self.world:
            r.train_step(x, y)  # averaged all-reduce inside (RCCL buckets on GPU, Gloo on CPU)
            return
        g, _ = r.compute_grads(x, y)
        if self.rank in self.delay:
            time.sleep(self.delay[self.rank])
        contrib = select_contributors(time.time(), self.rank, self.world, self.r2a, self.group)
        self.last_contributors = contrib
        w = 1.0 if self.rank in contrib else 0.0
        if hasattr(r, "eng"):
            r.reduce_grads(w)
            r.apply_grads(None, 1.0 / self.r2a)
        else:
            if w != 1.0:
                g.mul_(w)
            if self.world > 1:
                dist.all_reduce(g, group=self.group)
            r.apply_grads(g, 1.0 / self.r2a)


def broadcast_state(runner, src_worker: int = 0, group=None, group_src_rank: Optional[int] = None) -> None:
    """Chief -> all workers: params, optimizer slots, global step (CPU/Gloo path; the native GPU
    runner uses ``broadcast_from`` over RCCL)."""
    if hasattr(runner, "broadcast_from") and getattr(runner, "comm", None) is not None:
        runner.broadcast_from(src_worker)
        return
    src = group_src_rank if group_src_rank is not None else src_worker
    tensors = [runner.params()] + list(runner.slot_tensors().values())
    for t in tensors:
        buf = t.detach().cpu().contiguous()
        dist.broadcast(buf, src, group=group)
        t.copy_(buf.to(t.device))
    step = torch.tensor([runner.global_step()], dtype=torch.int64)
    dist.broadcast(step, src, group=group)
    if hasattr(runner, "applier"):
        runner.applier.t = int(step.item())
    runner.set_global_step(int(step.item()))
    if hasattr(runner, "eng"):
        runner.set_params(runner.params())
