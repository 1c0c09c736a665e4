"""Headline benchmark: images/sec (whole node) of the reference MNIST CNN training step, DP over
N MI355X (BASELINE.json metric; reference config: per-worker batch 128, Adam lr 0.01,
keep_prob 0.75 -- /root/reference/mnist_python_m.py:62-71,205-222).

One process per GPU: under torchrun the env says which rank this is; without a launcher
environment, ``--gpus N`` (N > 1) makes this process spawn the N ranks itself (parallel/spawn.py:
the parent never touches the GPU, relays rank 0's JSON line and fails if any rank fails), and a
job whose WORLD_SIZE differs from --gpus exits non-zero. Each step = fused HIP forward + backward + bucketed RCCL
gradient all-reduce (sum, 1/N folded into Adam) + fused flat Adam, with every kernel and
collective captured into ONE hipGraph that is replayed per step. Data is a device-resident
synthetic MNIST-shaped split (55000 x 784 fp32 in [0,1], random labels) indexed by a per-rank
permutation and the device global_step, so there is no host work inside the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch_size 128]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) MNIST CNN DP at 1/2/4/8 MI355X; step-time scaling"  # BASELINE.json
BASELINE_IMG_PER_S = 52.1  # 120 global steps x 256 images / 590 s (performance:6)
DATA_DESC = {
    "strokes": "synthetic (device-resident learnable MNIST-shaped set: 55000 class-conditional stroke images "
               "28x28 with their labels, utils/input_data.synthetic_mnist; random N(0,1) init; the timed steps "
               "are a learning state, not a collapsed one)",
    "random": "synthetic (device-resident MNIST-shaped 55000x784 uniform noise, random labels; random N(0,1) "
              "init; the model collapses to the label prior)",
}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch_size", type=int, default=128, help="per-GPU batch (reference --batch_size)")
    ap.add_argument("--eager", action="store_true", help="launch kernels per step instead of hipGraph replay")
    ap.add_argument("--fp32_grads", action="store_true", help="all-reduce fp32 grads (default bf16)")
    ap.add_argument("--ipc_small", type=int, default=1, help="1: peer-to-peer IPC one-shot all-reduce for the "
                    "small conv-gradient bucket (self-checked against RCCL at startup; falls back if it disagrees)")
    ap.add_argument("--transport", default="auto", choices=["auto", "rccl", "ipc"],
                    help="DP gradient transport: auto = IPC for every bucket when ranks share a GPU, else RCCL "
                    "(+ IPC for the small bucket)")
    ap.add_argument("--force_dp", type=int, default=0, help="1: run the full DP schedule (comm stream, captured "
                    "collectives) even at world 1 -- one-GPU rehearsal of the multi-GPU path")
    ap.add_argument("--min_warmup_ms", type=float, default=300.0, help="after --warmup steps, keep replaying "
                    "untimed steps until this much warm-up time has passed (GPU clock ramp; reported in the JSON)")
    ap.add_argument("--graph_steps", type=int, default=20, help="training steps captured per hipGraph "
                    "(device-side step counter/data cursor/dropout key make step i+1 of a graph the next step)")
    ap.add_argument("--lead_steps", type=int, default=0, help="timed region: launch this many one-step graphs "
                    "first, then ONE graph of the remaining steps (the GPU starts on the small launch while the "
                    "host enqueues the big one)")
    ap.add_argument("--spin_sync", type=int, default=0, help="1: after launching the timed steps, poll the end "
                    "event (hipEventQuery) before the closing torch.cuda.synchronize(), so the host notices "
                    "completion without the blocking wait's wake-up latency")
    ap.add_argument("--lean_gap", type=int, default=1, help="1: nothing but the barrier and synchronize between "
                    "the last warm-up step and the timed region (events made and the warm-up loss read beforehand)")
    ap.add_argument("--idle_us", type=float, default=0.0, help="diagnostic: host busy-wait before the timed region "
                    "(GPU idle), to measure what an idle gap costs the first timed steps")
    ap.add_argument("--phases", type=int, default=1, help="after the timed steps, replay a few steps of a graph "
                    "with HIP timing events at the phase boundaries and report the GPU phase breakdown (untimed)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"], help="compute dtype: bf16 MFMA operands "
                    "(fp32 accumulate/master/optimizer), or fp32 everything (the reference's precision)")
    ap.add_argument("--zero", type=int, default=-1, help="1: ZeRO-1 sharding of the fc1 weight (N > 1): with "
                    "--fc_sfb each rank forms only its shard's fc1 gradient and updates only that shard, the bf16 "
                    "shards are all-gathered (IPC one-shot) beside the next conv forward; -1 (default): on from 4 "
                    "ranks up, where the K = N*B fc GEMM and the full fc Adam (~28 us at N = 4) would otherwise "
                    "cost more than the 1.6 MB/peer weight gather that hides behind the conv forward")
    ap.add_argument("--fc_sfb", type=int, default=1, help="1 (N > 1 or --force_dp): fc-region gradients by "
                    "sufficient-factor broadcasting -- all-gather the fc factors (1.33 MB/rank) and form the summed "
                    "fc gradient locally instead of all-reducing it (6.4 MB); 0: bucketed all-reduce")
    ap.add_argument("--fused_tail", type=int, default=1, help="1: on one GPU the Adam kernel also reduces the "
                    "conv weight-gradient slabs and bumps the step (one kernel less)")
    ap.add_argument("--local_bf16_grads", type=int, default=1, help="1: on one GPU keep the fc-region gradients "
                    "in bf16 (the DP all-reduce wire format): fc backward writes and Adam reads 2 B per gradient")
    ap.add_argument("--fc_adam", type=int, default=0, help="1: on one GPU the fc1 Adam update runs in the fc1 "
                    "weight-gradient epilogue (fp32 gradient straight from the GEMM, fc1 bf16 shadow double-buffered; A/B neutral: "
                    "profiles/ab_fc1_adam_dw_epi_r3.log)")
    ap.add_argument("--conv_unfused", type=int, default=0, help="1: conv1 and conv2 forward as two kernels "
                    "(A/B of the fused conv1->conv2 kernel)")
    ap.add_argument("--state_steps", type=int, default=100, help="time the steps that follow this many training "
                    "steps from init (snapshot before the clock-ramp warm-up, restored before the timed region); "
                    "0: time whatever state the warm-up steps left")
    ap.add_argument("--data", default="strokes", choices=["strokes", "random"], help="device-resident training "
                    "set: learnable class-conditional strokes (default) or uniform noise with random labels")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu", action="store_true", help="plumbing dry-run: fp32 PyTorch CPU runner + Gloo "
                    "(exercises the launcher/barrier/JSON contract without a GPU; not a performance number)")
    argv = list(sys.argv[1:] if argv is None else argv)
    a = ap.parse_args(argv)
    from tensorflow_distributed_amd.parallel import spawn

    if spawn.needs_self_launch(a.gpus):
        # no launcher environment: this process only spawns the N ranks (it never touches the GPU)
        return spawn.self_launch(os.path.abspath(__file__), argv, a.gpus)
    if a.cpu:
        return _cpu_dry_run(a)

    import torch

    from tensorflow_distributed_amd import _native
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.parallel import dist as D

    _native.require()
    ctx = D.init_from_env(use_gpu=True)
    world, rank = ctx.world, ctx.rank
    spawn.check_world(a.gpus, world)
    dev = ctx.device
    B = a.batch_size
    eng = torch.classes.tfd.MnistEngine(B, dev.index, 0.75, a.seed, rank)
    eng.set_adam(a.lr, 0.9, 0.999, 1e-8)
    eng.set_dtype(a.dtype)
    eng.set_fused_tail(a.fused_tail)
    eng.set_local_bf16_grads(a.local_bf16_grads)
    eng.set_fc_adam(bool(a.fc_adam))
    eng.set_conv_unfused(a.conv_unfused)
    from tensorflow_distributed_amd.parallel.transport import attach_engine

    mode = a.transport
    if mode == "auto":
        mode = "ipc" if ctx.shared_device else "rccl"
    if a.zero < 0:
        a.zero = 1 if (world >= 4 and a.dtype == "bf16") else 0
    tr = attach_engine(eng, rank, world, dev, mode=mode, comm=ctx.comm, bf16=not a.fp32_grads,
                       small_ipc=bool(a.ipc_small), force_dp=bool(a.force_dp),
                       sfb=bool(a.fc_sfb) and a.dtype == "bf16", zero=bool(a.zero))
    if a.zero:
        eng.set_zero(True)
    s = torch.cuda.Stream(dev)
    n_data = 55000
    if a.data == "strokes":  # the learnable synthetic MNIST set (same images on every rank, like the
        # reference's workers that all read the full training split, mnist_python_m.py:291)
        from tensorflow_distributed_amd.utils.input_data import synthetic_mnist

        xi, yi = synthetic_mnist(n_data, 0)
        host_x = torch.from_numpy(xi.reshape(n_data, 784))
        host_y = torch.from_numpy(yi.astype("int32"))
    with torch.cuda.stream(s):
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        if a.data == "strokes":
            data = host_x.to(dev).float().div_(255.0)
            labels = host_y.to(dev)
        else:
            data = torch.rand(n_data, 784, device=dev, generator=g)
            labels = torch.randint(0, 10, (n_data,), device=dev, generator=g, dtype=torch.int32)
        perm = torch.randperm(n_data, device=dev, generator=g).to(torch.int32)
        if rank == 0:
            eng.params().copy_(M.flat_from_dict(M.init_params(a.seed)).to(dev))
        if world > 1:  # chief init -> everyone (reference M6): RCCL, or Gloo when ranks share a GPU
            if ctx.comm is not None:
                ctx.comm.broadcast(eng.params(), 0)
            else:
                torch.cuda.synchronize(dev)
                host = eng.params().cpu()
                ctx.broadcast_tensor_cpu(host, 0)
                eng.params().copy_(host.to(dev))
        eng.sync_shadow()
        eng.set_dataset(data, labels, perm)
        eng.set_input_mode(1)
        graph_mode = not a.eager
        eng.train_step()  # one eager step first: sets kernel attributes outside capture
        gsteps = max(1, a.graph_steps)
        lead = max(0, min(a.lead_steps, a.steps - 1)) if graph_mode else 0
        if graph_mode:
            try:
                eng.capture_train_step("train")
                if gsteps > 1:
                    eng.capture_train_steps("trainN", gsteps)
                if lead:
                    eng.capture_train_steps("timed", a.steps - lead)
            except Exception as e:  # pragma: no cover - capture support depends on the RCCL build
                print(f"# hipGraph capture failed ({e!r}); timing eager launches", file=sys.stderr)
                graph_mode = False
        if graph_mode:
            def run(k):
                if gsteps > 1 and k >= gsteps:
                    eng.replay("trainN", k // gsteps)
                if k % gsteps or gsteps == 1:
                    eng.replay("train", k % gsteps if gsteps > 1 else k)
        else:
            run = lambda k: [eng.train_step() for _ in range(k)]  # noqa: E731
        # The timed steps start from the training state after --state_steps steps (a model that is
        # still learning), not from wherever the clock-ramp warm-up below leaves it: snapshot it now,
        # warm up, restore it right before the timed region.
        snap = None
        if a.state_steps > 0:
            run(a.state_steps - 1)
            snap = [t.clone() for t in _state_tensors(eng)]
            _diag_digest("snapshot", eng, rank)
            snap_loss = eng.loss_rows().mean()  # the loss of step state_steps (read after timing)
        run(a.warmup)
    torch.cuda.synchronize(dev)
    if os.environ.get("TFD_DEBUG_IPC"):
        print(f"# rank {rank}: transport error after warmup = {tr.error()}", file=sys.stderr)
    # GPU clocks ramp over the first few hundred steps (profiles/warmup_ramp.log: 99 -> 92 us per
    # replay over 400 steps, back to 99.6 us after 2 s idle), so a 20-step timed region right after a
    # 5-step warm-up measures the ramp. Keep replaying untimed steps until --min_warmup_ms elapsed;
    # every rank runs the same count (decided by rank 0), so collectives stay matched.
    extra = 0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if a.lean_gap:  # torch creates the HIP events at their first record: do that outside the timed region
        with torch.cuda.stream(s):
            ev0.record(s)
            ev1.record(s)
    if a.min_warmup_ms > 0:
        t_w = time.perf_counter()
        chunk = 50
        while True:
            el = (time.perf_counter() - t_w) * 1e3
            go = torch.tensor([1 if el < a.min_warmup_ms else 0], dtype=torch.int64)
            ctx.broadcast_tensor_cpu(go, 0)
            if not int(go.item()):
                break
            with torch.cuda.stream(s):
                run(chunk)
                if a.lean_gap:
                    loss0_t = eng.loss_rows().mean()  # read after the timed region
            torch.cuda.synchronize(dev)
            extra += chunk
    if snap is not None:  # back to the snapshotted learning state (every rank: same step)
        with torch.cuda.stream(s):
            for dst, src in zip(_state_tensors(eng), snap):
                dst.copy_(src)
            eng.invalidate_prefetch()
            loss0_t = snap_loss
        del snap
        torch.cuda.synchronize(dev)
        _diag_digest("restored", eng, rank)
    if a.lean_gap and (extra or a.state_steps > 0):
        loss0 = None
    else:
        loss0 = float(eng.loss_rows().mean().item())

    ctx.barrier()
    torch.cuda.synchronize(dev)
    if a.idle_us > 0:
        t_i = time.perf_counter()
        while (time.perf_counter() - t_i) * 1e6 < a.idle_us:
            pass
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        ev0.record(s)
        if lead:
            eng.replay("train", lead)
            eng.replay("timed", 1)
        else:
            run(a.steps)
        ev1.record(s)
    t_launched = time.perf_counter()
    if a.spin_sync:
        while not ev1.query():
            pass
    torch.cuda.synchronize(dev)
    t_synced = time.perf_counter()
    ctx.barrier()
    dt = time.perf_counter() - t0
    if os.environ.get("TFD_BENCH_DIAG") and rank == 0:
        print(f"# timed region: host launch {1e6 * (t_launched - t0):.1f} us, sync wait "
              f"{1e6 * (t_synced - t_launched):.1f} us, barrier {1e6 * (t0 + dt - t_synced):.1f} us", file=sys.stderr)
    _diag_digest("timed", eng, rank)
    gpu_ms = ev0.elapsed_time(ev1)  # device time of the same K steps (diagnostic: host/sync overhead = dt - this)
    if a.zero:
        with torch.cuda.stream(s):
            eng.sync_params()
    dt = ctx.max_scalar(dt)
    tr.check("after the timed steps")
    topo = _job_topology(ctx, dev, tr, eng)
    phases = _phase_breakdown(eng, s, graph_mode, world, ctx) if a.phases else None
    # the phase steps ran on stream s: wait for them before reading the state on the default stream
    # (without this the last step's loss rows could be read mid-write: two runs of the same binary
    # printed the loss of step N or N - 1)
    torch.cuda.synchronize(dev)
    if loss0 is None:
        loss0 = float(loss0_t.item())
    loss1 = float(eng.loss_rows().mean().item())
    acc1 = float(eng.correct_rows().mean().item())  # last timed step's minibatch accuracy (train mode)
    # the conv1 weight gradient skips zero pooled gradients (TFD_C1W_SKIP0); those are the pixels the
    # pooled ReLU output is 0 at, so this is the share of that work the last timed step skipped
    p1_zero = float((eng.pool1() == 0).float().mean().item())
    gstep = int(eng.step_tensor().item())
    ms = dt * 1e3 / a.steps
    img_s = world * B * a.steps / dt
    if rank == 0:
        print(f"# world={world} B/gpu={B} steps={a.steps} global_step={gstep} loss {loss0:.3f}->{loss1:.3f} acc {acc1:.3f} "
              f"{ms:.4f} ms/step", file=sys.stderr)
        print(json.dumps({
            "metric": METRIC,
            "value": round(img_s, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_extra_steps": extra,
            "train_state": {"global_step": gstep, "loss_before_timed": round(loss0, 4),
                            "loss_after_timed": round(loss1, 4), "minibatch_accuracy": round(acc1, 4),
                            "state_steps": a.state_steps, "pool1_zero_fraction": round(p1_zero, 4)},
            "ms_per_step": round(ms, 5),
            "gpu_event_ms_per_step": round(gpu_ms / a.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / BASELINE_IMG_PER_S, 1),
            "dtype": a.dtype,
            "data": DATA_DESC[a.data],
            "phases_ms": phases,
            **topo,
            "config": {
                "model": "MNIST 2-conv CNN (reference conv_net: conv5x5x32-pool-conv5x5x64-pool-fc1024-dropout0.75-fc10), "
                         "Adam lr 0.01",
                "global_batch": world * B,
                "per_gpu_batch": B,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "grad_allreduce": "fp32" if (a.fp32_grads or a.dtype == "fp32") else "bf16",
                "hipgraph": graph_mode,
                "steps_per_graph": gsteps if graph_mode else 0,
                "dp_transport": tr.kind,
                "force_dp": bool(a.force_dp),
                "zero1_fc1": bool(a.zero),
                "fc_grads": ("fp32" if a.dtype == "fp32" else
                             "summed from all-gathered factors (sfb), bf16" if "sfb" in tr.kind else
                             "fc1: fp32 into Adam in the dW epilogue; out: bf16" if eng.fc_adam_active() else
                             "bf16" if (a.local_bf16_grads or world > 1) and not a.fp32_grads else "fp32"),
            },
        }), flush=True)
    tr.close()
    ctx.shutdown()
    return 0


def _diag_digest(where, eng, rank):
    """TFD_BENCH_DIAG: sha1 of the training state at a point of the run (reproducibility checks)."""
    if not os.environ.get("TFD_BENCH_DIAG") or rank != 0:
        return
    import hashlib

    import torch

    torch.cuda.synchronize()
    h = [hashlib.sha1(t.detach().contiguous().cpu().view(torch.uint8).numpy().tobytes()).hexdigest()[:10] for t in _state_tensors(eng)]
    print(f"# digest {where}: params {h[0]} bf16 {h[1]} m {h[2]} v {h[3]} step {int(eng.step_tensor().item())} "
          f"loss {float(eng.loss_rows().float().mean().item()):.4f}", file=sys.stderr)


def _state_tensors(eng):
    """Everything a training step reads and updates across steps: fp32 master, bf16 shadow, Adam
    slots, the device step counter (data cursor, dropout key, Adam's t)."""
    return [eng.params(), eng.params_bf16(), eng.adam_m(), eng.adam_v(), eng.step_tensor()]


def _job_topology(ctx, dev, tr, eng):
    """What the job really ran on, for the JSON: the communicator's own world size, every rank's
    device (index + PCI bus / uuid), and whether the replicas' parameters are bit-identical after
    the timed steps (sha1 of each rank's flat fp32 master, compared on rank 0)."""
    import hashlib

    import torch

    from tensorflow_distributed_amd.parallel.transport import device_label

    comm_world = 1
    if tr.comm is not None:
        comm_world = int(tr.comm.world())
    elif tr.ipc is not None:
        comm_world = int(tr.ipc.world())
    torch.cuda.synchronize(dev)
    digest = hashlib.sha1(eng.params().detach().cpu().numpy().tobytes()).hexdigest()[:16]
    mine = {"rank": ctx.rank, "device": device_label(dev), "params_sha1": digest}
    if ctx.world > 1:
        import torch.distributed as dist

        rows = [None] * ctx.world
        dist.all_gather_object(rows, mine)
    else:
        rows = [mine]
    return {"comm_world": comm_world, "devices": [r["device"] for r in rows],
            "replicas_identical": len({r["params_sha1"] for r in rows}) == 1,
            "params_sha1": rows[0]["params_sha1"]}


def _phase_breakdown(eng, stream, graph_mode, world, ctx):
    """GPU ms of fwd / fc bwd / conv bwd / optimizer / all-reduce of one step, from HIP timing
    events inside a separately captured graph (outside the timed region; median of 5 steps)."""
    import torch

    names = ("fwd", "bwd_fc", "bwd_conv", "optim", "allreduce", "comm_wait", "step")
    try:
        eng.set_phase_timing(True)
        rows = []
        with torch.cuda.stream(stream):
            eng.train_step()  # HIP needs an eager record of the timing events before graph replays time them
            if graph_mode:
                eng.capture_train_step("phases")
            for _ in range(5):
                if graph_mode:
                    eng.replay("phases", 1)
                else:
                    eng.train_step()
                rows.append(eng.phase_times().tolist())
        eng.set_phase_timing(False)
        if graph_mode:
            eng.drop_graph("phases")
        ctx.barrier()
        med = [sorted(r[i] for r in rows)[len(rows) // 2] for i in range(len(names))]
        return {k: round(v, 4) for k, v in zip(names, med)}
    except Exception as e:  # pragma: no cover - event capture support depends on the HIP build
        print(f"# phase timing unavailable: {e!r}", file=sys.stderr)
        return None


def _cpu_dry_run(a):
    import torch

    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.models.mnist_runner import TorchMnistRunner
    from tensorflow_distributed_amd.parallel import dist as D
    from tensorflow_distributed_amd.parallel.sync_replicas import SyncReplicasStepper, broadcast_state
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer

    from tensorflow_distributed_amd.parallel import spawn

    ctx = D.init_from_env(use_gpu=False)
    world, rank = ctx.world, ctx.rank
    spawn.check_world(a.gpus, world)
    r = TorchMnistRunner(a.batch_size, AdamOptimizer(a.lr), keep_prob=0.75, seed=a.seed, rank=rank)
    if rank == 0:
        r.load_flat(M.flat_from_dict(M.init_params(a.seed)), {}, 0)
    if world > 1:
        broadcast_state(r, 0)
    st = SyncReplicasStepper(r, rank, world, world)
    g = torch.Generator().manual_seed(1000 + rank)
    x = torch.rand(a.batch_size, 784, generator=g)
    y = torch.randint(0, 10, (a.batch_size,), generator=g)
    for _ in range(a.warmup):
        st.step(x, y)
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st.step(x, y)
    ctx.barrier()
    dt = ctx.max_scalar(time.perf_counter() - t0)
    if rank == 0:
        print(json.dumps({"metric": "images/sec (whole node) MNIST CNN DP [CPU dry-run]", "value": world * a.batch_size * a.steps / dt,
                          "unit": "images/s", "n_gpus": 0, "n_ranks": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": dt * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
                          "config": {"model": "mnist_cnn", "global_batch": world * a.batch_size, "seq_len": None,
                                     "parallelism": f"dp{world}", "device": "cpu"}}), flush=True)
    ctx.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
