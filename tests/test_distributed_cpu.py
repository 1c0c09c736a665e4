"""Multi-process data parallelism on Gloo/CPU: sync DP equivalence,
bit-identical replicas, backup workers (replicas_to_aggregate < N), async parameter server."""
import numpy as np
import pytest
import torch

from dist_util import run_ranks

pytestmark = pytest.mark.slow


def _data(n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, 784, generator=g), torch.randint(0, 10, (n,), generator=g)


def _dp_worker(rank, world, steps, B):
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.models.mnist_runner import TorchMnistRunner
    from tensorflow_distributed_amd.parallel.sync_replicas import SyncReplicasStepper, broadcast_state
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer

    r = TorchMnistRunner(B, AdamOptimizer(0.01), keep_prob=1.0, rank=rank)
    if rank == 0:
        r.load_flat(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(4).items()}), {}, 0)
    broadcast_state(r, 0)
    st = SyncReplicasStepper(r, rank, world, world)
    x, y = _data(B * world * steps, 11)
    for s in range(steps):
        lo = (s * world + rank) * B
        st.step(x[lo:lo + B], y[lo:lo + B])
    return r.params().clone(), r.global_step()


@pytest.mark.parametrize("world", [2, 8])
def test_sync_dp_equals_big_batch_single_process(world):
    """Gloo sync DP at 2 ranks and at the 8 of the driver's 8-GPU job == one process with N x B."""
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.models.mnist_runner import TorchMnistRunner
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer

    steps, B = 3, 8
    outs = run_ranks(_dp_worker, world, steps, B, timeout=400)
    for p, st in outs:
        assert torch.equal(p, outs[0][0]), "replicas diverged"
        assert st == steps
    ref = TorchMnistRunner(B * world, AdamOptimizer(0.01), keep_prob=1.0)
    ref.load_flat(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(4).items()}), {}, 0)
    x, y = _data(B * world * steps, 11)
    for s in range(steps):
        lo = s * world * B
        ref.train_step(x[lo:lo + world * B], y[lo:lo + world * B])
    # Adam amplifies summation-order differences where v ~ 0 (a handful of elements): bound them --
    # the update's relative L2 error, at most a few elements past the elementwise bound, none far off
    init = M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(4).items()})
    got, want = outs[0][0], ref.params()
    d = (got - want).abs()
    assert ((got - init) - (want - init)).norm() / (want - init).norm() < 1e-3
    assert int((d > 1e-4 + 1e-3 * want.abs()).sum()) <= 3 and d.max() < 1e-3, d.max()


def _backup_worker(rank, world, r2a, slow_rank):
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.models.mnist_runner import TorchMnistRunner
    from tensorflow_distributed_amd.parallel.sync_replicas import SyncReplicasStepper, broadcast_state
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer

    B = 8
    r = TorchMnistRunner(B, AdamOptimizer(0.01), keep_prob=1.0, rank=rank)
    if rank == 0:
        r.load_flat(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(9).items()}), {}, 0)
    broadcast_state(r, 0)
    st = SyncReplicasStepper(r, rank, world, r2a, straggler_delay_s={slow_rank: 3.0})
    x, y = _data(B * world, 3)
    st.step(x[rank * B:(rank + 1) * B], y[rank * B:(rank + 1) * B])
    return r.params().clone(), st.last_contributors


def test_backup_workers_drop_the_straggler():
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.models.mnist_runner import TorchMnistRunner
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer

    world, r2a, slow = 3, 2, 1
    outs = run_ranks(_backup_worker, world, r2a, slow)
    for p, contrib in outs:
        assert contrib == [0, 2]
        assert torch.equal(p, outs[0][0])
    # reference: average of the two fast workers' gradients, one Adam step
    B = 8
    x, y = _data(B * world, 3)
    grads = []
    for rk in (0, 2):
        r = TorchMnistRunner(B, AdamOptimizer(0.01), keep_prob=1.0)
        r.load_flat(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(9).items()}), {}, 0)
        g, _ = r.compute_grads(x[rk * B:(rk + 1) * B], y[rk * B:(rk + 1) * B])
        grads.append(g.clone())
    r.apply_grads((grads[0] + grads[1]), 0.5)
    torch.testing.assert_close(outs[0][0], r.params(), rtol=1e-4, atol=1e-6)


def _async_role(rank, world, steps, num_ps):
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.models.mnist_runner import TorchMnistRunner
    from tensorflow_distributed_amd.parallel import async_ps
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer

    layout = async_ps.mnist_layout(num_ps)
    nw = world - num_ps
    if rank < num_ps:
        svc = async_ps.ParameterServerService(rank, num_ps, nw, layout, AdamOptimizer(0.01))
        svc.serve()
        return ("ps", svc.updates, svc.global_step)
    wk = rank - num_ps
    r = TorchMnistRunner(8, AdamOptimizer(0.01), keep_prob=1.0, rank=wk)
    client = async_ps.AsyncPSClient(wk, layout)
    flat = torch.zeros(M.TOTAL)
    if wk == 0:
        client.init(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(5).items()}))
    client.pull(flat)
    r.set_params(flat)
    x, y = _data(8 * steps, 20 + wk)
    gsteps = []
    for s in range(steps):
        g, _ = r.compute_grads(x[s * 8:(s + 1) * 8], y[s * 8:(s + 1) * 8])
        gs = client.push_pull(flat, g.clone())
        r.set_params(flat)
        gsteps.append(gs)
    client.stop()
    return ("worker", gsteps, flat.clone())


@pytest.mark.parametrize("num_ps", [1, 2])
def test_async_parameter_server(num_ps):
    steps, nw = 3, 2
    outs = run_ranks(_async_role, num_ps + nw, steps, num_ps)
    ps = [o for o in outs if o[0] == "ps"]
    wk = [o for o in outs if o[0] == "worker"]
    assert all(o[1] == steps * nw for o in ps), "every PS shard applies every worker's update"
    assert ps[0][2] == steps * nw, "global_step counts every worker step (async)"
    allsteps = sorted(s for o in wk for s in o[1])
    assert allsteps == list(range(1, steps * nw + 1))


def test_round_robin_placement():
    from tensorflow_distributed_amd.parallel import async_ps
    from tensorflow_distributed_amd.parallel.cluster import ClusterSpec, replica_device_setter

    c = ClusterSpec({"ps": ["h:1", "h:2"], "worker": ["h:3"]})
    names = ["global_step", "Variable", "Variable_1", "Variable_2"]
    pl = replica_device_setter(c, names)
    assert pl == {"global_step": "/job:ps/task:0/cpu:0", "Variable": "/job:ps/task:1/cpu:0",
                  "Variable_1": "/job:ps/task:0/cpu:0", "Variable_2": "/job:ps/task:1/cpu:0"}
    lay = async_ps.mnist_layout(2)
    assert [n for n, _, _ in lay.ranges[1]] == ["Variable", "Variable_2", "Variable_4", "Variable_6"]
    assert c.rank("ps", 1) == 1 and c.rank("worker", 0) == 2 and c.world_size == 3


def _shared_worker(rank, world):
    import torch

    from tensorflow_distributed_amd.parallel.transport import device_key, devices_shared

    same = devices_shared(torch.device("cuda", 0), world)
    own = devices_shared(torch.device("cuda", rank), world)
    return same, own, device_key(torch.device("cuda", rank))


def test_transport_detects_shared_devices():
    """Two ranks on 'gpu:0' share a device (IPC transport); gpu:0 + gpu:1 do not (RCCL)."""
    from dist_util import run_ranks

    res = run_ranks(_shared_worker, 2)
    assert all(r[0] for r in res) and not any(r[1] for r in res)
    assert res[0][2] != res[1][2]


def _ps_state_role(rank, world, sync):
    """1 PS + 2 workers: PUSH/PULL_STATE/INIT-with-slots protocol (sync: R = 2 accumulator)."""
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.parallel import async_ps
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer, FlatApplier

    layout = async_ps.mnist_layout(1)
    if rank == 0:
        svc = async_ps.ParameterServerService(0, 1, 2, layout, AdamOptimizer(0.01), sync=sync, replicas_to_aggregate=2)
        svc.serve()
        return ("ps", svc.updates, svc.global_step, svc.dropped)
    wk = rank - 1
    client = async_ps.AsyncPSClient(wk, layout, slot_names=["m", "v"])
    flat = torch.zeros(M.TOTAL)
    p0 = M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(5).items()})
    if wk == 0:
        client.init(p0.clone())
    client.pull(flat)
    g = torch.randn(M.TOTAL, generator=torch.Generator().manual_seed(100 + wk)) * 1e-2
    step = client.push_pull(flat, g, local_step=0)
    out = {"step": step, "flat": flat.clone(), "dropped": client.last_dropped}
    if sync and wk == 1:
        # a straggler's gradient for step 0 arriving after the step-0 update is stale: dropped
        step2 = client.push_pull(flat, g, local_step=0)
        out["stale_step"], out["stale_dropped"] = step2, client.last_dropped
    slots, t, gs = client.pull_state(flat.clone())
    out.update(slots=slots, t=t)
    client.stop()
    return ("worker", out)


def test_sync_ps_accumulator_averages_r_fresh_gradients_and_drops_stale():
    import torch.nn.functional as F  # noqa: F401

    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer, FlatApplier

    outs = run_ranks(_ps_state_role, 3, True)
    ps = outs[0]
    w0, w1 = outs[1][1], outs[2][1]
    assert ps[1] == 1 and ps[2] == 1 and ps[3] == 1, ps  # one averaged update, one stale push dropped
    assert w0["step"] == w1["step"] == 1 and not w0["dropped"] and not w1["dropped"]
    assert w1["stale_dropped"] and w1["stale_step"] == 1
    p = M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(5).items()})
    gs = [torch.randn(M.TOTAL, generator=torch.Generator().manual_seed(100 + w)) * 1e-2 for w in (0, 1)]
    ap = FlatApplier(AdamOptimizer(0.01), M.TOTAL)
    ap.apply(p, gs[0] + gs[1], 0.5)
    real = lambda t: torch.cat([v.reshape(-1) for v in M.dict_from_flat(t).values()])  # noqa: E731 (no padding)
    torch.testing.assert_close(real(w0["flat"]), real(p), rtol=1e-6, atol=1e-7)
    assert torch.equal(w0["flat"], w1["flat"])
    torch.testing.assert_close(real(w0["slots"]["m"]), real(ap.m), rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(real(w0["slots"]["v"]), real(ap.v), rtol=1e-6, atol=1e-12)
    assert w0["t"] == 1


def test_async_ps_state_pull_has_the_optimizer_slots():
    outs = run_ranks(_ps_state_role, 3, False)
    ps = outs[0]
    assert ps[1] == 2 and ps[2] == 2  # async: every push applied
    for _, w in outs[1:]:
        assert w["t"] == 2 and w["slots"]["m"].abs().sum() > 0 and w["slots"]["v"].abs().sum() > 0


def _sfb_worker(rank, world, B):
    import torch.distributed as dist

    from tensorflow_distributed_amd.models import mnist_cnn as M

    torch.manual_seed(100 + rank)
    p = {k: v * 0.05 for k, v in M.init_params(3).items()}
    x = torch.rand(B, 784)
    y = torch.randint(0, 10, (B,))
    mask = (torch.rand(B, 1024) < 0.75).float()
    # all-reduce path: this rank's autograd gradients, summed over ranks
    q = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    loss = M.softmax_xent_mean(M.conv_net(x, q, keep_prob=0.75, dropout_mask=mask), y)
    loss.backward()
    ar = {k: q[k].grad.clone() for k in ("wd1", "bd1", "out", "out_b")}
    for v in ar.values():
        dist.all_reduce(v)
    # sufficient-factor path: gather every rank's factors, one GEMM over all rows
    facs = M.fc_sufficient_factors(x, y, p, keep_prob=0.75, dropout_mask=mask)
    gathered = []
    for f in facs:
        parts = [torch.zeros_like(f) for _ in range(world)]
        dist.all_gather(parts, f.contiguous())
        gathered.append(torch.cat(parts))
    sfb = M.fc_grads_from_factors(*gathered)
    return {k: (ar[k], sfb[k]) for k in ar}


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sufficient_factor_fc_gradients_equal_the_all_reduce(world):
    """The DP fc-gradient algorithm of the native engine (mnist_fc_grad_sfb), on the fp32 oracle
    over gloo: the GEMM over all ranks' gathered factors equals the all-reduced sum of the ranks'
    own fc gradients (dropout included), for every fc tensor."""
    res = run_ranks(_sfb_worker, world, 16, timeout=300)
    for out in res:
        for k, (ar, sfb) in out.items():
            torch.testing.assert_close(sfb, ar, rtol=1e-4, atol=1e-5, msg=k)


def _gpu_ps_vote(rank, world, hosts, capable):
    from tensorflow_distributed_amd.training.dist_main import agree_gpu_ps

    return agree_gpu_ps(capable[rank], hosts[rank])


def test_gpu_ps_use_is_decided_collectively():
    """the GPU-resident PS (IPC peer memory) is used only when every ps and worker task
    is on one host and has a GPU; every task gets the same answer (no PS serving one protocol while
    a worker speaks the other)."""
    same, split = ["h|1"] * 3, ["h|1", "h|1", "other|2"]
    for hosts, capable, want in ((same, [True] * 3, True), (split, [True] * 3, False),
                                 (same, [True, False, True], False)):
        res = run_ranks(_gpu_ps_vote, 3, hosts, capable)
        assert [ok for ok, _ in res] == [want] * 3, (hosts, capable, res)
        if not want:
            assert len({why for _, why in res}) == 1 and res[0][1]
