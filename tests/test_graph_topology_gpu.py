"""Dependency edges of the REAL captured DP step graphs (graph-edge test).

``MnistEngine.capture_topology(n)`` captures n training steps exactly as the benchmark's replayed
graph and returns nodes / edges / per-operation tags (hipGraphGetNodes / hipGraphGetEdges plus
hipStreamGetCaptureInfo_v2 at every schedule operation); utils/graph_check.py then requires, for
every collective, a dependency path from the kernel that produced its operand and to every kernel
that consumes its result, plus the write-after-read edges into the next step. On one GPU whose
ranks time-slice a missing edge can hide (the collective happens to finish first); with 8 real
peers it would be a race, so the structure is checked instead of the numbers. A schedule with one
cross-stream wait removed (``set_debug_drop_wait``) must fail the same check."""
import pytest
import torch

from dist_util import run_ranks

pytestmark = pytest.mark.gpu

SCHEDULES = {"sfb": (True, False, False), "sfb+zero": (True, True, False), "sfb+mr": (True, False, True),
             "sfb+zero+mr": (True, True, True), "allreduce": (False, False, False)}


def _engine(cuda, world_rank=0, B=64):
    from tensorflow_distributed_amd.models import mnist_cnn as M

    e = torch.classes.tfd.MnistEngine(B, 0, 0.75, 7, world_rank)
    e.set_adam(0.01, 0.9, 0.999, 1e-8)
    n = 1024
    g = torch.Generator(device=cuda).manual_seed(3)
    e.params().copy_(M.flat_from_dict(M.init_params(5)).to(cuda) * 0.05)
    e.sync_shadow()
    e.set_dataset(torch.rand(n, 784, device=cuda, generator=g),
                  torch.randint(0, 10, (n,), dtype=torch.int32, device=cuda, generator=g),
                  torch.randperm(n, device=cuda, generator=g).to(torch.int32))
    e.set_input_mode(1)
    return e


def _check(eng, n, drop="", require_nodes=True):
    from tensorflow_distributed_amd.utils.graph_check import Topology, violations

    eng.set_debug_drop_wait(drop)
    try:
        lines = list(eng.capture_topology(n))
    finally:
        eng.set_debug_drop_wait("")
    t = Topology(lines)
    assert len(t.types) > 10 and sum(len(v) for v in t.succ.values()) > 10, lines[:20]
    return t, (violations(t) if require_nodes else violations(t, collectives=()))


def test_one_gpu_step_topology(cuda):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        e = _engine(cuda)
        e.train_step()
        t, v = _check(e, 2)
    assert v == [], v
    labels = [lb for lb, _, _ in t.tags]
    assert labels[:5] == ["conv_fwd", "fc_fwd", "fc_bwd", "conv_bwd", "opt"], labels


@pytest.mark.parametrize("mode", ["rccl", "ipc"])
@pytest.mark.parametrize("sched", list(SCHEDULES))
def test_forced_dp_world1_topology(cuda, sched, mode):
    """The multi-GPU schedules over a real world-1 communicator: every collective ordered after its
    producer and before its consumers, 3 steps. A world-1 in-place RCCL collective captures no node
    of its own; the topology capture puts a marker kernel at its place in the comm stream
    (MnistEngine::tag), so the RCCL schedule's edges are checked like the IPC one's, and dropping one
    of its cross-stream waits must be caught over both transports."""
    from tensorflow_distributed_amd.parallel.transport import attach_engine

    sfb, zero, mr = SCHEDULES[sched]
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        e = _engine(cuda)
        tr = attach_engine(e, 0, 1, cuda, mode=mode, force_dp=True, sfb=sfb, zero=zero)
        if zero:
            e.set_zero(True)
        e.set_sfb_merge_reduce(mr)
        e.train_step()
        t, v = _check(e, 3)
        assert v == [], (sched, v)
        labels = {lb for lb, _, _ in t.tags}
        want = {"gather_p2", "gather_dr", "ar_conv", "sfb_gemm"} if sfb else {"ar_fc", "ar_conv", "opt_fc"}
        assert want <= labels, labels
        if zero:
            assert "wag" in labels
        # fault injection: the schedule without one of its cross-stream waits is caught
        drop = "sfb_gemm<-gather_dr" if sfb else "fc_fwd<-opt_fc"
        _, v2 = _check(e, 2, drop)
        assert v2, f"dropping {drop} went unnoticed"
        e.train_step()  # the engine still runs normally afterwards
    torch.cuda.synchronize()
    tr.check()
    tr.close()


def _ipc_topology_worker(rank, world, sched):
    from tensorflow_distributed_amd import _native
    from tensorflow_distributed_amd.parallel.transport import attach_engine
    from tensorflow_distributed_amd.utils.graph_check import Topology, violations

    _native.require()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    sfb, zero, mr = SCHEDULES[sched]
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        e = _engine(dev, rank)
        tr = attach_engine(e, rank, world, dev, mode="ipc", sfb=sfb, zero=zero)
        if zero:
            e.set_zero(True)
        e.set_sfb_merge_reduce(mr)
        e.train_step()
        lines = list(e.capture_topology(2))
    torch.cuda.synchronize()
    err = tr.error()
    tr.close()
    return violations(Topology(lines)), sorted({ln.split()[1].split("@")[0] for ln in lines if ln.startswith("tag")}), err


@pytest.mark.parametrize("sched", list(SCHEDULES))
def test_two_rank_ipc_topology(cuda, sched):
    """World 2 over the IPC transport (both ranks on this GPU): the world > 1 schedule variants --
    fc-region optimizer before the conv bucket's wait, the ZeRO shard gather issued inside the step."""
    res = run_ranks(_ipc_topology_worker, 2, sched, timeout=300)
    for rank, (v, labels, err) in enumerate(res):
        assert err == 0, rank
        assert v == [], (rank, v)
        assert "ar_conv" in labels, labels
        if SCHEDULES[sched][0]:
            assert {"opt_fc", "opt_conv"} <= set(labels), labels
