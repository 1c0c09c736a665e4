"""Optimizers with TF1 ``tf.train`` semantics (reference: ``AdamOptimizer(lr)`` at
``/root/reference/mnist_single.py:95`` and ``mnist_python_m.py:208``; ``SyncReplicasOptimizer`` at
``mnist_python_m.py:210-233``).

Two layers:

* Plain config objects (``AdamOptimizer``, ``GradientDescentOptimizer``, ``MomentumOptimizer``)
  that model runners hand to their device implementation: the native GPU engine applies them with
  one fused flat HIP kernel (``csrc/kernels/optim.hip``); :class:`FlatApplier` below is the torch
  implementation used on CPU workers and by the parameter-server role (same update equations).
* :class:`SyncReplicasOptimizer` -- the distributed aggregation policy: average exactly
  ``replicas_to_aggregate`` gradients per global step out of ``total_num_replicas`` workers
  (``replicas_to_aggregate < total`` = backup workers). Executed by
  :mod:`tensorflow_distributed_amd.parallel.sync_replicas`.

TF ApplyAdam: ``lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)``; ``m = m + (g - m)(1 - b1)``;
``v = v + (g^2 - v)(1 - b2)``; ``p -= lr_t * m / (sqrt(v) + eps)``, ``t`` = update count (the
``beta1_power``/``beta2_power`` accumulators are ``b^t``).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Optional

import torch


@dataclass
class AdamOptimizer:
    learning_rate: float = 0.001
    beta1: float = 0.9
    beta2: float = 0.999
    epsilon: float = 1e-8
    name: str = "Adam"
    kind: str = field(default="adam", init=False)


@dataclass
class GradientDescentOptimizer:
    learning_rate: float = 0.01
    name: str = "GradientDescent"
    kind: str = field(default="sgd", init=False)


@dataclass
class MomentumOptimizer:
    learning_rate: float = 0.01
    momentum: float = 0.9
    use_nesterov: bool = False
    name: str = "Momentum"
    kind: str = field(default="momentum", init=False)


@dataclass
class SyncReplicasOptimizer:
    """``tf.train.SyncReplicasOptimizer(opt, replicas_to_aggregate, total_num_replicas)``."""
    opt: object
    replicas_to_aggregate: Optional[int] = None
    total_num_replicas: Optional[int] = None
    name: str = "sync_replicas"

    def resolve(self, num_workers: int) -> "SyncReplicasOptimizer":
        r = self.replicas_to_aggregate if self.replicas_to_aggregate is not None else num_workers
        t = self.total_num_replicas if self.total_num_replicas is not None else num_workers
        if not 1 <= r <= t:
            raise ValueError(f"replicas_to_aggregate={r} must be in [1, total_num_replicas={t}]")
        return SyncReplicasOptimizer(self.opt, r, t, self.name)

    @property
    def has_backup_workers(self) -> bool:
        return self.replicas_to_aggregate is not None and self.total_num_replicas is not None and \
            self.replicas_to_aggregate < self.total_num_replicas


def base_optimizer(opt):
    return opt.opt if isinstance(opt, SyncReplicasOptimizer) else opt


class FlatApplier:
    """Applies an optimizer config to a flat fp32 parameter tensor (any device) with TF semantics.

    Slot tensors (``m``/``v`` for Adam, ``accum`` for momentum) are flat buffers of the same size;
    ``t`` counts applied updates (for the parameter server it is the number of updates applied to
    this shard, exactly like TF's per-PS ``beta1_power``).
    """

    def __init__(self, opt, numel: int, device=None):
        self.opt = base_optimizer(opt)
        self.device = device
        self.t = 0
        k = self.opt.kind
        z = lambda: torch.zeros(numel, dtype=torch.float32, device=device)  # noqa: E731
        self.m = z() if k in ("adam", "momentum") else None
        self.v = z() if k == "adam" else None

    @torch.no_grad()
    def apply(self, p: torch.Tensor, g: torch.Tensor, scale: float = 1.0) -> None:
        o = self.opt
        g = g if scale == 1.0 else g * scale
        self.t += 1
        if o.kind == "adam":
            b1, b2 = o.beta1, o.beta2
            lr_t = o.learning_rate * (1 - b2 ** self.t) ** 0.5 / (1 - b1 ** self.t)
            self.m.add_(g - self.m, alpha=1 - b1)
            self.v.add_(g * g - self.v, alpha=1 - b2)
            p.sub_(lr_t * self.m / (self.v.sqrt() + o.epsilon))
        elif o.kind == "momentum":
            self.m.mul_(o.momentum).add_(g)
            if o.use_nesterov:
                p.sub_(o.learning_rate * (g + o.momentum * self.m))
            else:
                p.sub_(o.learning_rate * self.m)
        else:
            p.sub_(o.learning_rate * g)

    def slots(self) -> "OrderedDict[str, torch.Tensor]":
        out = OrderedDict()
        if self.m is not None:
            out["m"] = self.m
        if self.v is not None:
            out["v"] = self.v
        return out

    def powers(self):
        o = self.opt
        if o.kind != "adam":
            return {}
        return {"beta1_power": o.beta1 ** self.t, "beta2_power": o.beta2 ** self.t}
