"""Choice of the gradient transport for synchronous data parallelism on GPUs.

The reference lets several workers share one device: ``--num_gpus=1`` with two workers puts both on
``gpu:0`` (``task_index % num_gpus``, ``/root/reference/mnist_python_m.py:164-168``). RCCL refuses
two ranks of one communicator on the same device, so the framework picks the transport from where
the ranks actually are:

* every rank on its own GPU -> RCCL over xGMI for the bandwidth bucket (fc1, 98% of the bytes),
  plus the peer-to-peer IPC one-shot kernel for the latency-bound conv bucket (self-checked
  against RCCL on the node before use);
* two or more ranks on one GPU -> the IPC transport carries every bucket (it only needs
  ``hipIpcOpenMemHandle`` between processes, which works on a shared device).

Both paths run the engine's identical DP schedule (comm stream, captured collectives, 1/N folded
into the optimizer), so a one-GPU box exercises the code an 8-GPU node runs.
"""
from __future__ import annotations

import os
import socket
import sys
from typing import Optional

import torch
import torch.distributed as dist


def device_key(device: torch.device) -> str:
    """Host-unique identity of a GPU (two ranks with equal keys share the device)."""
    idx = device.index or 0
    uid = ""
    try:
        uid = str(getattr(torch.cuda.get_device_properties(idx), "uuid", "") or "")
    except Exception:  # pragma: no cover - property availability depends on the torch build
        uid = ""
    vis = os.environ.get("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES", ""))
    return f"{socket.gethostname()}|{uid}" if uid else f"{socket.gethostname()}|{vis}|{idx}"


def device_label(device: torch.device) -> str:
    """Human-readable identity of a rank's GPU for benchmark records: index, PCI bus, uuid."""
    idx = device.index or 0
    p = torch.cuda.get_device_properties(idx)
    bus = getattr(p, "pci_bus_id", None)
    uid = str(getattr(p, "uuid", "") or "")
    return f"cuda:{idx}" + (f" pci:{bus}" if bus is not None else "") + (f" uuid:{uid}" if uid else "")


def devices_shared(device: torch.device, world: int, group=None) -> bool:
    """True when at least two ranks of ``group`` run on the same GPU (all-gather of device keys)."""
    if world <= 1:
        return False
    keys = [None] * world
    dist.all_gather_object(keys, device_key(device), group=group)
    return len(set(keys)) < len(keys)


def make_rccl(rank: int, world: int, device_index: int, group=None, src: int = 0):
    """Native RCCL communicator; the 128-byte unique id is broadcast over the Gloo ``group`` from
    global rank ``src`` (the group's first member)."""
    from .. import _native

    _native.require()
    uid = torch.classes.tfd.RcclComm.unique_id() if rank == 0 else torch.zeros(128, dtype=torch.uint8)
    if world > 1:
        dist.broadcast(uid, src, group=group)
    return torch.classes.tfd.RcclComm(uid, world, rank, device_index)


def _ref_all_reduce(comm, y, group):
    """Reference sum: RCCL when there is a communicator, else Gloo on a host copy."""
    if comm is not None:
        comm.all_reduce(y, "sum")
        return y
    h = y.cpu()
    dist.all_reduce(h, group=group)
    return h.to(y.device)


def _ref_all_gather(comm, mine, world, group):
    if comm is not None:
        out = torch.empty(world * mine.numel(), dtype=mine.dtype, device=mine.device)
        comm.all_gather(mine, out)
        return out
    parts = [torch.empty(mine.numel(), dtype=torch.float32) for _ in range(world)]
    dist.all_gather(parts, mine.float().cpu(), group=group)
    return torch.cat(parts).to(mine.device, mine.dtype)


def ipc_self_check(ipc, comm, n: int, device: torch.device, group=None) -> bool:
    """One all-reduce through IPC and through the reference (RCCL, or Gloo when ranks share a GPU)
    on random data; the results must agree."""
    g = torch.Generator(device=device).manual_seed(77 + ipc.rank())
    x = torch.randn(n, device=device, generator=g)
    y = _ref_all_reduce(comm, x.clone(), group)
    ipc.all_reduce(x, 1.0)
    torch.cuda.synchronize(device)
    return bool(ipc.error() == 0 and torch.allclose(x, y, rtol=1e-4, atol=1e-4))


def ipc_gather_self_check(ipc, comm, shards, device: torch.device, group=None) -> bool:
    """The in-place bf16 all-gather (SFB factors, ZeRO weight shards) at every shard size the step
    will run through IPC, against the reference gather: a gather is a copy, so bit-exact."""
    W, r = int(ipc.world()), int(ipc.rank())
    ok = True
    for S in shards:
        g = torch.Generator(device=device).manual_seed(91 + r + 1000 * S)
        mine = torch.randn(S, device=device, generator=g).to(torch.bfloat16)
        buf = torch.zeros(W * S, dtype=torch.bfloat16, device=device)
        buf[r * S:(r + 1) * S] = mine
        ipc.all_gather(buf)
        ref = _ref_all_gather(comm, mine, W, group)
        torch.cuda.synchronize(device)
        ok = ok and bool(ipc.error() == 0 and torch.equal(buf, ref))
    return ok


def small_bucket_ipc(rank: int, world: int, device: torch.device, comm, max_bytes: int, group=None, log=None,
                     force: bool = False):
    """IPC one-shot all-reduce for a bucket reducer's small buckets (bf16 wire, <= ``max_bytes``),
    beside an RCCL communicator: created, self-checked against ``comm`` (RCCL) on every rank, and
    kept only when every rank agrees (``IpcCollectives``), else None -- the small buckets then stay on
    RCCL. ``force``: also at world 1 (the one-GPU rehearsal of this path)."""
    from .ipc import IpcCollectives, make_ipc_comm

    log = log or (lambda m: print(m, file=sys.stderr))
    if max_bytes <= 0 or (world <= 1 and not force):
        return None
    cap = max(1024, (max_bytes + 1) // 2)  # elements: a bucket of max_bytes in bf16 (an fp32 one needs half)
    ipc, ok = None, 0
    try:
        ipc = make_ipc_comm(rank, world, device.index or 0, cap, group=group, max_blocks=64)
    except Exception as e:  # pragma: no cover - depends on the node's IPC support
        log(f"# small-bucket ipc setup failed: {e!r}")
    if ipc is not None:
        ok = int(ipc_self_check(ipc, comm, min(cap, 65536), device, group))
    flags = torch.tensor([1 - ok], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)
    if int(flags.item()) == 0:
        return IpcCollectives(ipc)
    log("# small-bucket ipc self-check failed; every bucket stays on RCCL")
    if ipc is not None:
        ipc.close()
    return None


def _gather_shards(eng, world: int, cap: int, sfb: bool, zero: bool):
    """Shard sizes (bf16 elements) of the all-gathers that will run through an IPC staging of
    ``cap`` fp32 elements (MnistEngine::ipc_gathers)."""
    from ..models import mnist_cnn as M

    shards = []
    if sfb:
        shards += [int(eng.batch()) * M.FEAT, int(eng.sfb_shard_elems())]
    if zero and world > 1:
        shards.append(M.FEAT * M.HID // world)
    return sorted({S for S in shards if 2 * cap >= S and S % 8 == 0})


class DPTransport:
    """What :func:`attach_engine` wired into an engine (for logs / bench JSON)."""

    def __init__(self, kind: str, comm=None, ipc=None):
        self.kind = kind  # "none" | "rccl" | "rccl+ipc" | "ipc"
        self.comm = comm
        self.ipc = ipc

    def error(self) -> int:
        """Sticky IPC barrier-timeout word (0 = healthy). A timeout leaves that collective's output
        unreduced, so callers must check this and fail instead of training on desynced replicas."""
        return int(self.ipc.error()) if self.ipc is not None else 0

    def check(self, what: str = "") -> None:
        e = self.error()
        if e:
            raise RuntimeError(f"IPC collective barrier timed out{(' (' + what + ')') if what else ''}: "
                               "replicas may have diverged")

    def close(self) -> None:
        if self.ipc is not None:
            self.ipc.close()
            self.ipc = None
        self.comm = None


def attach_engine(eng, rank: int, world: int, device: torch.device, group=None, src: int = 0,
                  mode: str = "auto", comm=None, bf16: bool = True, small_ipc: bool = True,
                  force_dp: bool = False, capacity: Optional[int] = None, log=None,
                  sfb: bool = False, zero: bool = False) -> DPTransport:
    """Give ``eng`` (``MnistEngine``) its gradient transport.

    mode: ``auto`` (IPC everywhere when ranks share a GPU, else RCCL + IPC small bucket),
    ``rccl``, ``ipc``. ``comm``: an existing RCCL communicator to reuse. ``force_dp`` with world 1
    runs the full DP schedule over a world-1 communicator (one-GPU coverage of the RCCL path).
    ``sfb``: fc-region gradients by sufficient-factor broadcasting (``MnistEngine.set_fc_sfb``: the
    fc factors are all-gathered -- over IPC when its staging holds them -- instead of all-reducing
    the 6.4 MB fc gradient). ``zero``: the engine will shard fc1 (``set_zero``); the IPC staging is
    sized to hold one bf16 fc1 shard too, so the per-step weight all-gather takes the IPC one-shot
    path (every peer read at once) instead of RCCL's ring.
    """
    from ..models import mnist_cnn as M
    from .ipc import make_ipc_comm

    log = log or (lambda m: print(m, file=sys.stderr))
    if world <= 1 and not force_dp:
        return DPTransport("none")
    shared = devices_shared(device, world, group)
    if mode == "auto":
        mode = "ipc" if shared else "rccl"
    cap = capacity or M.TOTAL
    # IPC staging (fp32 units) that also holds one SFB gather shard (bf16 elements)
    small_cap = max(M.BUCKET_SPLIT, (int(eng.sfb_shard_elems()) + 1) // 2) if sfb else M.BUCKET_SPLIT
    if zero and world > 1:  # one bf16 fc1 shard (MnistEngine.set_zero: zshard = |wd1| / world)
        small_cap = max(small_cap, (M.FEAT * M.HID // world + 1) // 2)

    def _sfb(tr: DPTransport) -> DPTransport:
        if sfb and bf16:
            eng.set_fc_sfb(True)
            tr.kind += "+sfb"
        return tr

    if mode == "ipc":
        ipc = make_ipc_comm(rank, world, device.index or 0, max(cap, small_cap), group=group,
                            max_blocks=8 if shared else 64)
        if world > 1:  # every IPC collective of this configuration against Gloo; no fallback exists here
            ok = int(ipc_self_check(ipc, None, M.BUCKET_SPLIT, device, group)
                     and ipc_gather_self_check(ipc, None, _gather_shards(eng, world, max(cap, small_cap), sfb, zero),
                                               device, group))
            flags = torch.tensor([1 - ok], dtype=torch.int64)
            dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)
            if int(flags.item()):
                ipc.close()
                raise RuntimeError("IPC transport self-check failed (all-reduce or all-gather disagrees with Gloo)")
        eng.set_ipc(ipc, cap, bf16)
        if force_dp:
            eng.set_force_dp(True)
        return _sfb(DPTransport("ipc", ipc=ipc))
    if mode != "rccl":
        raise ValueError(f"unknown DP transport {mode!r}")
    if comm is None:
        comm = make_rccl(rank, world, device.index or 0, group=group, src=src)
    eng.set_comm(comm, bf16)
    if force_dp:
        eng.set_force_dp(True)
    kind = "rccl"
    if small_ipc and world > 1:
        ok_ar, ok_ag, ipc = 0, 0, None
        try:
            ipc = make_ipc_comm(rank, world, device.index or 0, small_cap, group=group, max_blocks=64)
        except Exception as e:  # pragma: no cover - depends on the node's IPC support (all ranks raise)
            log(f"# ipc setup failed: {e!r}")
        if ipc is not None:  # every rank has one (make_ipc_comm agrees collectively) -> matched checks
            ok_ar = int(ipc_self_check(ipc, comm, M.BUCKET_SPLIT, device, group))
            ok_ag = int(ipc_gather_self_check(ipc, comm, _gather_shards(eng, world, small_cap, sfb, zero), device,
                                              group))
        flags = torch.tensor([1 - ok_ar, 1 - ok_ag], dtype=torch.int64)
        dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)  # every rank must agree
        if int(flags[0].item()) == 0:
            eng.set_ipc(ipc, M.BUCKET_SPLIT, bf16)
            if int(flags[1].item()):  # per-path fallback: the gathers go through RCCL
                log("# ipc all-gather self-check failed; SFB / ZeRO gathers stay on RCCL")
                eng.set_ipc_gather(False)
                return _sfb(DPTransport("rccl+ipc(ar)", comm=comm, ipc=ipc))
            return _sfb(DPTransport("rccl+ipc", comm=comm, ipc=ipc))
        log("# ipc self-check failed; the conv bucket stays on RCCL")
        if ipc is not None:
            ipc.close()
    return _sfb(DPTransport(kind, comm=comm))
