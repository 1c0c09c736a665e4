"""Peer-to-peer IPC all-reduce and the engine's data-parallel step with several ranks on ONE GPU
(RCCL refuses duplicate devices; the IPC transport does not), so the multi-rank orchestration --
buckets on the comm stream, events, hipGraph capture of collectives, 1/N in Adam -- is exercised
on the single-GPU box."""
import pytest
import torch

from dist_util import run_ranks

pytestmark = pytest.mark.gpu


def _ar_worker(rank, world, n, max_blocks=8):
    from tensorflow_distributed_amd.parallel.ipc import make_ipc_comm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = make_ipc_comm(rank, world, 0, n, max_blocks=max_blocks)
    outs = []
    base = torch.arange(n, dtype=torch.float32, device=dev) % 97
    t = base * (rank + 1)
    comm.all_reduce(t, 1.0)
    torch.cuda.synchronize()
    outs.append(t.cpu())
    # bf16 + scale, and hipGraph capture/replay of the collective
    tb = (base * (rank + 1)).to(torch.bfloat16)
    comm.all_reduce(tb, 0.5)
    torch.cuda.synchronize()
    outs.append(tb.float().cpu())
    # fp32 in, bf16 out (the ResNet reducer's fused wire cast): the fp32 sum, rounded once
    src = base * (rank + 1) + 0.25
    dst = torch.empty(n, dtype=torch.bfloat16, device=dev)
    comm.all_reduce_into(src, dst, 1.0)
    torch.cuda.synchronize()
    outs.append(dst.float().cpu())
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    x = torch.ones(n, device=dev) * (rank + 1)
    with torch.cuda.stream(s):
        comm.all_reduce(x, 1.0)  # warm
        x.fill_(rank + 1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            comm.all_reduce(x, 1.0)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    outs.append(x.cpu())
    err = comm.error()
    comm.close()
    return outs, err


# every compile-time world size of the kernels (W = 2..8, csrc/comm/ipc_allreduce.hip); world 8 also
# at the distinct-GPU grid cap (64 blocks, parallel/transport.py) besides the shared-device one (8)
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,n,max_blocks", [(2, 52096, 8), (3, 1000, 8), (4, 200000, 8), (5, 1000, 8),
                                                (6, 77777, 8), (7, 4096, 8), (8, 200000, 8), (8, 52096, 64)])
def test_ipc_allreduce_multiprocess_one_gpu(cuda, world, n, max_blocks):
    res = run_ranks(_ar_worker, world, n, max_blocks, timeout=300)
    base = torch.arange(n, dtype=torch.float32) % 97
    tot = sum(range(1, world + 1))
    for outs, err in res:
        assert err == 0
        assert torch.equal(outs[0], base * tot)
        ref_bf = sum((base * (r + 1)).to(torch.bfloat16).float() for r in range(world)) * 0.5
        torch.testing.assert_close(outs[1], ref_bf.to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)
        ref_into = sum(base * (r + 1) + 0.25 for r in range(world))
        assert torch.equal(outs[2], ref_into.to(torch.bfloat16).float())
        # three replays of an in-place all-reduce: x -> x * tot each time, starting from rank+1 per rank
        # (first replay sums (1..world), later replays multiply the identical value by world)
        assert torch.allclose(outs[3], torch.full((n,), float(tot * world ** 2)))


LR_SGD = 0.05


def _set_opt(eng, sgd):
    if sgd:
        eng.set_momentum(LR_SGD, 0.0, False)
    else:
        eng.set_adam(0.01, 0.9, 0.999, 1e-8)


def _close_elementwise(got, ref, what, rel=1.5e-2, absmax=4e-3):
    """Per tensor of the flat layout: |got - ref| <= rel |ref| + absmax max|ref| for EVERY element
    (bf16 wire rounding of the per-rank gradients, fp32 sums in a different order)."""
    from tensorflow_distributed_amd.models import mnist_cnn as M

    gd, rd = M.dict_from_flat(got), M.dict_from_flat(ref)
    for k in rd:
        r, d = rd[k].float(), gd[k].float()
        tol = rel * r.abs() + absmax * r.abs().max()
        bad = (d - r).abs() > tol
        assert not bad.any(), (f"{what} {k}: {int(bad.sum())}/{r.numel()} elements off; worst |d-r| "
                               f"{(d - r).abs().max().item():.3e} vs max|r| {r.abs().max().item():.3e}")


def _close_multistep(got, ref, what, rel_l2=8e-2, cap=0.15):
    """Several steps apart from the reference (each step sees weights the last one moved slightly
    differently; max-pool argmax / relu flips near ties move single elements): per tensor, the
    relative L2 error of the update <= rel_l2 and EVERY element within cap x the tensor's largest
    update. (The one-step tests hold each element to bf16-wire tolerance.)"""
    from tensorflow_distributed_amd.models import mnist_cnn as M

    gd, rd = M.dict_from_flat(got), M.dict_from_flat(ref)
    for k in rd:
        r, d = rd[k].float(), gd[k].float()
        err, big = (d - r).abs(), r.abs().max()
        rel = ((d - r).norm() / r.norm().clamp_min(1e-30)).item()
        msg = f"{what} {k}: rel L2 {rel:.3e}; worst |d-r| {err.max().item():.3e} vs max|r| {big.item():.3e}"
        assert rel <= rel_l2 and bool((err <= cap * big).all()), msg


def _engine_dp_worker(rank, world, B, steps, sfb=False, zero=False, sgd=False):
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.parallel.ipc import make_ipc_comm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = make_ipc_comm(rank, world, 0, M.TOTAL)
    eng = torch.classes.tfd.MnistEngine(B, 0, 1.0, 5, rank)
    _set_opt(eng, sgd)
    eng.set_ipc(comm, 1 << 30, True)
    if sfb:
        eng.set_fc_sfb(True)
        assert eng.fc_sfb()
    if zero:
        eng.set_zero(True)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(steps, world * B, 784, generator=g)
    y = torch.randint(0, 10, (steps, world * B), generator=g, dtype=torch.int32)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.params().copy_(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()}).to(dev))
        eng.sync_shadow()
        for i in range(steps):
            eng.feed_x().copy_(x[i, rank * B:(rank + 1) * B].to(dev))
            eng.feed_y().copy_(y[i, rank * B:(rank + 1) * B].to(dev))
            if i == 0:
                eng.train_step()
                eng.capture_train_step("t")
            else:
                eng.replay("t", 1)
            torch.cuda.current_stream().synchronize()
        eng.sync_params()  # ZeRO: gather every rank's fc1 shard (master, slots, bf16 shadow)
    torch.cuda.synchronize()
    out = eng.params().cpu(), int(eng.step_tensor().item()), comm.error(), eng.world()
    comm.close()
    return out


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,sfb,zero", [(2, False, False), (2, True, False), (4, True, True), (8, True, True)])
def test_engine_dp_over_ipc_matches_single_rank_big_batch(cuda, world, sfb, zero):
    """DP=N (N processes sharing the GPU, IPC transport, captured graph; sfb: fc gradients from the
    all-gathered factors; zero: ZeRO-1 fc1 shards, the N >= 4 default) == DP=1 with N*B over three SGD
    steps: per tensor L2 and every element bounded (SGD: the update is the gradient, no m/sqrt(v)
    amplification of the bf16 wire rounding where |g| ~ 0)."""
    from tensorflow_distributed_amd.models import mnist_cnn as M

    B, steps = 32, 3
    res = run_ranks(_engine_dp_worker, world, B, steps, sfb, zero, True, timeout=300)
    for p, st, e, w in res:
        assert e == 0 and w == world and st == steps
        assert torch.equal(p, res[0][0]), "replicas diverged"
    p0 = res[0][0]
    eng = torch.classes.tfd.MnistEngine(world * B, 0, 1.0, 5, 0)
    _set_opt(eng, True)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(steps, world * B, 784, generator=g)
    y = torch.randint(0, 10, (steps, world * B), generator=g, dtype=torch.int32)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        eng.params().copy_(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()}).to(cuda))
        eng.sync_shadow()
        for i in range(steps):
            eng.feed_x().copy_(x[i].to(cuda))
            eng.feed_y().copy_(y[i].to(cuda))
            eng.train_step()
    torch.cuda.synchronize()
    ref = eng.params().cpu()
    init = M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()})
    _close_multistep(p0 - init, ref - init, "3-step update")


def _engine_dp_grads_worker(rank, world, B, sfb, zero=False):
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.parallel.ipc import make_ipc_comm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = make_ipc_comm(rank, world, 0, M.TOTAL)
    eng = torch.classes.tfd.MnistEngine(B, 0, 1.0, 5, rank)
    _set_opt(eng, True)
    eng.set_ipc(comm, 1 << 30, True)
    if sfb:
        eng.set_fc_sfb(True)
    if zero:
        eng.set_zero(True)
    g = torch.Generator().manual_seed(11)
    x = torch.rand(world * B, 784, generator=g)
    y = torch.randint(0, 10, (world * B,), generator=g, dtype=torch.int32)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.params().copy_(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()}).to(dev))
        eng.sync_shadow()
        eng.feed_x().copy_(x[rank * B:(rank + 1) * B].to(dev))
        eng.feed_y().copy_(y[rank * B:(rank + 1) * B].to(dev))
        eng.train_step()
        grads = eng.grads_bf16().float().cpu()  # the summed gradients the optimizer read
        eng.sync_params()  # ZeRO: every rank's updated fc1 shard
    torch.cuda.synchronize()
    out = grads, eng.params().cpu(), comm.error()
    comm.close()
    return out


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,sfb,zero,B", [(2, False, False, 32), (2, True, False, 32), (4, True, False, 32),
                                              (4, True, True, 32), (8, True, True, 128), (8, False, False, 32)])
def test_engine_dp_reduced_grads_elementwise(cuda, world, sfb, zero, B):
    """The gradient every rank's optimizer consumes after one DP=N step (bf16 wire: per-rank mean
    gradients cast to bf16, summed in fp32 in rank order, stored bf16; with sfb the fc gradients
    are one GEMM over all ranks' gathered factors; with zero -- the N >= 4 default -- each rank's
    optimizer reads only its fc1 shard, compared shard by shard) equals N x the DP=1 gradient of the
    N*B batch element by element within bf16 rounding, and the post-step parameters (one SGD step,
    shards gathered) equal the DP=1 step's. World 8 at B = 128 is the 8-GPU headline's shape: SFB
    over K = 8 x 128 gathered rows and a |wd1| / 8 ZeRO shard per rank."""
    from tensorflow_distributed_amd.models import mnist_cnn as M

    res = run_ranks(_engine_dp_grads_worker, world, B, sfb, zero, timeout=300)
    assert all(e == 0 for _, _, e in res)
    assert all(torch.equal(p, res[0][1]) for _, p, _ in res), "replicas diverged"
    w1, b1 = M.OFFSETS["wd1"], M.OFFSETS["bd1"]
    shard = (b1 - w1) // world
    if not zero:
        assert all(torch.equal(g, res[0][0]) for g, _, _ in res), "ranks consumed different gradients"
    eng = torch.classes.tfd.MnistEngine(world * B, 0, 1.0, 5, 0)
    g = torch.Generator().manual_seed(11)
    x = torch.rand(world * B, 784, generator=g)
    y = torch.randint(0, 10, (world * B,), generator=g, dtype=torch.int32)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        eng.params().copy_(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()}).to(cuda))
        eng.sync_shadow()
        eng.feed_x().copy_(x.to(cuda))
        eng.feed_y().copy_(y.to(cuda))
        eng.forward(True)
        eng.backward_a()
        eng.backward_b()
    torch.cuda.synchronize()
    gref = eng.grads().cpu()
    ref = gref * world  # per-rank means summed = world x the N*B mean
    for rk, (g, p, _) in enumerate(res):
        if zero:  # the optimizer of rank rk reads the conv region, its fc1 shard and the tail only
            lo, hi = w1 + rk * shard, w1 + (rk + 1) * shard
            g = torch.cat([g[:w1], torch.zeros(lo - w1), g[lo:hi], torch.zeros(b1 - hi), g[b1:]])
            r = torch.cat([ref[:w1], torch.zeros(lo - w1), ref[lo:hi], torch.zeros(b1 - hi), ref[b1:]])
        else:
            r = ref
        _close_elementwise(g, r, f"rank {rk} reduced gradient")
    init = M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()})
    # one SGD step with the 1/N scale: (init - p) / lr is the N*B mean gradient
    _close_elementwise((init - res[0][1]) / LR_SGD, gref, "post-step parameters")


def _resnet_dp_worker(rank, world, steps):
    from tensorflow_distributed_amd.models.resnet import ResNet
    from tensorflow_distributed_amd.parallel.ipc import IpcCollectives, make_ipc_comm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    m = ResNet(18, num_classes=16, device=dev, seed=5, width=16)
    comm = make_ipc_comm(rank, world, 0, m.fp.total)
    m.set_comm(IpcCollectives(comm), bucket_mb=0.25, bf16_grads=False)
    nb = len(m.reducer.buckets)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(steps, world * 4, 32, 32, 3, generator=g)
    y = torch.randint(0, 16, (steps, world * 4), generator=g, dtype=torch.int32)
    losses = []
    for i in range(steps):
        losses.append(m.train_step(x[i, rank * 4:(rank + 1) * 4].to(dev), y[i, rank * 4:(rank + 1) * 4].to(dev),
                                   lr=0.05).item())
    torch.cuda.synchronize()
    out = m.fp.master.cpu(), losses, comm.error(), nb, m.reducer.launched
    comm.close()
    return out


def test_resnet_bucketed_dp_over_ipc(cuda):
    """Two ranks on one GPU: bucketed all-reduce overlapped with the backward keeps replicas
    identical and equals manual averaging of the two half-batch gradients."""
    from tensorflow_distributed_amd.models.resnet import ResNet

    steps, world = 3, 2
    res = run_ranks(_resnet_dp_worker, world, steps, timeout=300)
    (p0, l0, e0, nb, launched), (p1, l1, e1, _, _) = res
    assert e0 == e1 == 0 and nb > 2 and launched == nb
    assert torch.equal(p0, p1)
    m = ResNet(18, num_classes=16, device=cuda, seed=5, width=16)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(steps, world * 4, 32, 32, 3, generator=g)
    y = torch.randint(0, 16, (steps, world * 4), generator=g, dtype=torch.int32)
    for i in range(steps):
        acc = torch.zeros_like(m.fp.grad)
        for r in range(world):
            m.reducer.reset()
            loss, _ = m.loss(x[i, r * 4:(r + 1) * 4].to(cuda), y[i, r * 4:(r + 1) * 4].to(cuda))
            loss.backward()
            acc += m.fp.grad
        torch.ops.tfd.momentum_flat(m.fp.master, m.fp.momentum, acc, m.fp.shadow, 0.05, 0.9, 1e-4, False, 0.5)
    torch.cuda.synchronize()
    torch.testing.assert_close(p0, m.fp.master.cpu(), rtol=1e-4, atol=1e-5)


def _rs_ag_worker(rank, world, S, max_blocks=8):
    from tensorflow_distributed_amd.parallel.ipc import make_ipc_comm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = make_ipc_comm(rank, world, 0, world * S, max_blocks=max_blocks)
    x = (torch.arange(world * S, dtype=torch.float32, device=dev) % 31) * (rank + 1)
    out = torch.empty(S, dtype=torch.bfloat16, device=dev)
    comm.reduce_scatter(x, out, 0.5)
    buf = torch.full((world * S,), -1.0, device=dev)
    buf[rank * S:(rank + 1) * S] = rank + 10.0
    comm.all_gather(buf)
    bb = torch.zeros(world * S, dtype=torch.bfloat16, device=dev)
    bb[rank * S:(rank + 1) * S] = rank + 1
    comm.all_gather(bb)
    torch.cuda.synchronize()
    r = out.float().cpu(), buf.cpu(), bb.float().cpu(), comm.error()
    comm.close()
    return r


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,S,max_blocks", [(2, 4096, 8), (4, 50000, 8), (8, 50000, 8), (8, 401408, 64)])
def test_ipc_reduce_scatter_all_gather(cuda, world, S, max_blocks):
    res = run_ranks(_rs_ag_worker, world, S, max_blocks, timeout=300)
    base = torch.arange(world * S, dtype=torch.float32) % 31
    tot = sum(range(1, world + 1))
    for r, (rs, ag, agb, err) in enumerate(res):
        assert err == 0
        torch.testing.assert_close(rs, (base[r * S:(r + 1) * S] * tot * 0.5).to(torch.bfloat16).float())
        assert torch.equal(ag, torch.cat([torch.full((S,), p + 10.0) for p in range(world)]))
        assert torch.equal(agb, torch.cat([torch.full((S,), float(p + 1)) for p in range(world)]))


def _engine_zero_worker(rank, world, B, steps, zero):
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.parallel.ipc import make_ipc_comm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = make_ipc_comm(rank, world, 0, M.TOTAL)
    eng = torch.classes.tfd.MnistEngine(B, 0, 1.0, 5, rank)
    eng.set_adam(0.01, 0.9, 0.999, 1e-8)
    eng.set_ipc(comm, M.BUCKET_SPLIT, True)
    if zero:
        eng.set_zero(True)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(steps, world * B, 784, generator=g)
    y = torch.randint(0, 10, (steps, world * B), generator=g, dtype=torch.int32)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.params().copy_(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()}).to(dev))
        eng.sync_shadow()
        for i in range(steps):
            eng.feed_x().copy_(x[i, rank * B:(rank + 1) * B].to(dev))
            eng.feed_y().copy_(y[i, rank * B:(rank + 1) * B].to(dev))
            if i == 0:
                eng.train_step()
                eng.capture_train_step("t")
            else:
                eng.replay("t", 1)
            torch.cuda.current_stream().synchronize()
        eng.sync_params()
    torch.cuda.synchronize()
    out = eng.params_bf16().float().cpu(), comm.error(), eng.params().cpu(), eng.adam_v().cpu()
    comm.close()
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_engine_zero1_matches_replicated_dp(cuda, world):
    """ZeRO-1 fc1 sharding (reduce-scatter -> 1/N optimizer -> all-gather at the next step) gives
    the same bf16 weights on every rank as replicated all-reduce DP."""
    B, steps = 16, 3
    zr = run_ranks(_engine_zero_worker, world, B, steps, True, timeout=300)
    rp = run_ranks(_engine_zero_worker, world, B, steps, False, timeout=300)
    assert all(r[1] == 0 for r in zr + rp)
    for r in zr[1:]:
        assert torch.equal(r[0], zr[0][0]), "ZeRO replicas diverged"
        # sync_params also gathered the fp32 master and the Adam moments of every shard
        assert torch.equal(r[2], zr[0][2]) and torch.equal(r[3], zr[0][3])
    assert torch.equal(zr[0][2].to(torch.bfloat16).float(), zr[0][0])
    # identical math: both buckets leave the kernels as bf16, every rank sums in rank order in fp32
    # (reduce-scatter and all-reduce alike), and Adam is elementwise -> bit-identical weights
    d = (zr[0][0] - rp[0][0]).abs()
    assert torch.equal(zr[0][0], rp[0][0]), (d.max().item(), (d > 0).float().mean().item())
    assert torch.equal(zr[0][2], rp[0][2])


@pytest.mark.parametrize("world", [2, 4])
def test_engine_sfb_zero_shards_equal_sfb(cuda, world):
    """SFB with ZeRO-1 (each rank forms and applies only its fc1 shard's gradient, bf16 shards
    all-gathered beside the next conv forward) gives bit-identical parameters to plain SFB."""
    B, steps = 32, 4
    zr = run_ranks(_engine_dp_worker, world, B, steps, True, True, timeout=300)
    rp = run_ranks(_engine_dp_worker, world, B, steps, True, False, timeout=300)
    for p, st, e, w in zr + rp:
        assert e == 0 and st == steps
    for p, *_ in zr:
        assert torch.equal(p, zr[0][0])
    d = (zr[0][0] - rp[0][0]).abs()
    assert torch.equal(zr[0][0], rp[0][0]), (d.max().item(), (d > 0).float().mean().item())
