"""Process-group bootstrap: one process per GPU, RCCL (xGMI) for tensors, Gloo/TCP for control.

Replaces the reference's ``tf.train.ClusterSpec`` + in-process gRPC ``Server`` rendezvous
(``/root/reference/mnist_python_m.py:145-161``): ranks meet at a TCP store (``MASTER_ADDR`` /
``MASTER_PORT``, or the coordinator address derived from ``--ps_hosts``), exchange the RCCL
unique id over the Gloo control group, and build a native :class:`torch.classes.tfd.RcclComm`
bound to ``local_rank`` (the ``task_index % num_gpus`` device rule of ``:164-172``).

The control plane (barriers, small host scalars, metric reduction, checkpoint coordination) runs
on Gloo so it never perturbs the GPU streams; gradient traffic goes through the native comm on its
own HIP stream inside the captured step graph.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: Optional[torch.device] = None
    comm: object = None  # torch.classes.tfd.RcclComm when world > 1, on GPU, one rank per device
    initialized_pg: bool = False
    shared_device: bool = False  # >= 2 ranks on one GPU: RCCL refuses that, the IPC transport carries DP

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    def barrier(self) -> None:
        if self.world > 1:
            dist.barrier()

    def max_scalar(self, x: float) -> float:
        if self.world == 1:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_scalars(self, xs):
        if self.world == 1:
            return [float(v) for v in xs]
        t = torch.tensor([float(v) for v in xs], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.tolist()

    def broadcast_tensor_cpu(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world > 1:
            dist.broadcast(t, src)
        return t

    def shutdown(self) -> None:
        if self.comm is not None:
            self.comm = None
        if self.initialized_pg and dist.is_initialized():
            dist.destroy_process_group()
            self.initialized_pg = False


def env_rank_world():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_process_group(rank: int, world: int, master_addr: str = None, master_port: int = None,
                       timeout_s: float = 300.0) -> bool:
    """Gloo control group over a TCP store (127.0.0.1 default; never relies on hostname lookup)."""
    if world <= 1 or dist.is_initialized():
        return False
    addr = master_addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(master_port or os.environ.get("MASTER_PORT", "29500"))
    dist.init_process_group("gloo", init_method=f"tcp://{addr}:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s))
    return True


def make_rccl_comm(rank: int, world: int, device_index: int):
    """Native RCCL communicator; the 128-byte unique id travels over the Gloo group."""
    from .. import _native

    _native.require()
    if rank == 0:
        uid = torch.classes.tfd.RcclComm.unique_id()
    else:
        uid = torch.zeros(128, dtype=torch.uint8)
    if world > 1:
        dist.broadcast(uid, 0)
    return torch.classes.tfd.RcclComm(uid, world, rank, device_index)


def init_from_env(use_gpu: Optional[bool] = None, num_gpus: Optional[int] = None, rccl: bool = True) -> DistContext:
    """Bootstrap from torchrun-style env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
    rank, world, local = env_rank_world()
    ctx = DistContext(rank=rank, world=world, local_rank=local)
    ctx.initialized_pg = init_process_group(rank, world)
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    if use_gpu:
        n = num_gpus or torch.cuda.device_count()
        idx = local % max(n, 1)
        torch.cuda.set_device(idx)
        ctx.device = torch.device("cuda", idx)
        if rccl and world > 1:
            from .transport import devices_shared

            ctx.shared_device = devices_shared(ctx.device, world)
            if not ctx.shared_device:
                ctx.comm = make_rccl_comm(rank, world, idx)
    else:
        ctx.device = torch.device("cpu")
    return ctx
