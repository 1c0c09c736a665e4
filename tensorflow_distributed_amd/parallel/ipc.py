"""Peer-to-peer IPC communicator bootstrap (native ``IpcComm``, csrc/runtime/ipc_comm.cpp).

Every rank exports its staging + signal buffers (``hipIpcGetMemHandle``), the 128-byte handles
are all-gathered over the Gloo control group, and every rank opens its peers' exports. Used for
latency-bound buckets (the conv-gradient bucket B, ~200 KB) next to RCCL,
or alone (every bucket) when RCCL is unavailable -- e.g. several ranks sharing one GPU in tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def make_ipc_comm(rank: int, world: int, device_index: int, capacity_elems: int, group=None,
                  spin_limit_ms: float = None, max_blocks: int = None):
    """max_blocks: grid cap of the spinning collectives -- 64 with one rank per GPU, 8 (the default,
    safe everywhere) when ranks share a GPU: both kernels' blocks must be co-resident, see
    IpcComm::blocks."""
    from .. import _native

    _native.require()
    import os

    if spin_limit_ms is None:
        # generous: a peer may still be loading code objects on its first call (observed > 2 s when
        # ranks share a GPU); any finite limit keeps a missing peer from hanging the device
        spin_limit_ms = float(os.environ.get("TFD_IPC_SPIN_MS", "30000"))
    # local step (allocation + export) first, then agree on its success before the collective
    # handle exchange: a rank that failed locally must not leave its peers blocked in all_gather
    comm, h, err = None, None, None
    try:
        comm = torch.classes.tfd.IpcComm(world, rank, device_index, capacity_elems)
        comm.set_spin_limit_ms(spin_limit_ms)
        comm.set_max_blocks(int(max_blocks or 8))
        h = comm.handle()
    except Exception as e:  # noqa: BLE001 - reported on every rank below
        err = e
    if world > 1:
        bad = torch.tensor([1 if err is not None else 0], dtype=torch.int64)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=group)
        if int(bad.item()):
            if comm is not None:
                comm.close()
            raise IpcSetupError(f"IPC setup failed on at least one rank (here: {err!r})")
    elif err is not None:
        raise IpcSetupError(f"IPC setup failed: {err!r}") from err
    if world > 1:
        allh = [torch.zeros_like(h) for _ in range(world)]
        dist.all_gather(allh, h, group=group)
        comm.open(torch.stack(allh))
    else:
        comm.open(h.reshape(1, -1))
    return comm


class IpcSetupError(RuntimeError):
    """Raised on EVERY rank when any rank's local IPC setup failed (collective decision)."""


class IpcCollectives:
    """RcclComm-shaped facade over IpcComm (``all_reduce(t, op)``, ``world()``, ``broadcast``) so
    bucket reducers can run on the IPC transport, e.g. several ranks sharing one GPU in tests."""

    def __init__(self, ipc):
        self.ipc = ipc

    def world(self) -> int:
        return self.ipc.world()

    def rank(self) -> int:
        return self.ipc.rank()

    def all_reduce(self, t, op: str = "sum") -> None:
        if op not in ("sum", "avg", "mean"):
            raise ValueError(f"IpcCollectives: unsupported op {op}")
        self.ipc.all_reduce(t, 1.0 if op == "sum" else 1.0 / self.ipc.world())

    def all_reduce_into(self, src, dst, op: str = "sum") -> None:
        """dst = the ranks' sum of src (dtypes may differ: fp32 gradients in, the bf16 wire sums out --
        the cast a bucket otherwise pays as a separate pass before its collective)."""
        if op not in ("sum", "avg", "mean"):
            raise ValueError(f"IpcCollectives: unsupported op {op}")
        self.ipc.all_reduce_into(src, dst, 1.0 if op == "sum" else 1.0 / self.ipc.world())
