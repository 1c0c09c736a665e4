"""Headline benchmark: images/sec (whole node) of the reference MNIST CNN training step, DP over
N MI355X (BASELINE.json metric; reference config: per-worker batch 128, Adam lr 0.01,
keep_prob 0.75 -- /root/reference/mnist_python_m.py:62-71,205-222).

One process per GPU: under torchrun the env says which rank this is; without a launcher
environment, ``--gpus N`` (N > 1) makes this process spawn the N ranks itself (parallel/spawn.py:
the parent never touches the GPU, relays rank 0's JSON line and fails if any rank fails), and a
job whose WORLD_SIZE differs from --gpus exits non-zero. Each step = fused HIP forward + backward
+ the DP gradient exchange (RCCL / peer-to-peer IPC collectives on a comm stream) + fused flat
Adam, with every kernel and collective captured into ONE hipGraph that is replayed per step.

Data: a device-resident synthetic MNIST-shaped split (55000 x 784 fp32 in [0,1]): by default the
learnable class-conditional stroke images of utils/input_data.synthetic_mnist with their labels
(``--data random``: uniform noise, random labels), indexed by a per-rank permutation and the
device global_step, so there is no host work inside the timed region.

Schedule: with N > 1 the ranks first probe every candidate DP schedule at this N (sufficient
factors + ZeRO-1, sufficient factors, bucketed all-reduce; parallel/schedule.py), untimed, and
time the fastest; the JSON reports every candidate's ms/step and the choice. ``--schedule NAME``
skips the probes. The job exits non-zero if the replicas' parameters differ after the timed steps.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch_size 128] [--schedule auto]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tensorflow_distributed_amd.parallel.schedule import MNIST_SCHEDULES as SCH_MNIST_SCHEDULES  # noqa: E402

METRIC = "images/sec (whole node) MNIST CNN DP at 1/2/4/8 MI355X; step-time scaling"  # BASELINE.json
BASELINE_IMG_PER_S = 52.1  # 120 global steps x 256 images / 590 s (performance:6)
DATA_DESC = {
    "strokes": "synthetic (device-resident learnable MNIST-shaped set: 55000 class-conditional stroke images "
               "28x28 with their labels, utils/input_data.synthetic_mnist; random N(0,1) init; the timed steps "
               "are a learning state, not a collapsed one)",
    "random": "synthetic (device-resident MNIST-shaped 55000x784 uniform noise, random labels; random N(0,1) "
              "init; the model collapses to the label prior)",
}
# DP schedules of the bf16 step (N > 1 or --force_dp): parallel/schedule.MNIST_SCHEDULES
SCHEDULES = SCH_MNIST_SCHEDULES


def _args(argv):
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
    ap.add_argument("--schedule", default="auto", choices=["auto"] + list(SCHEDULES),
                    help="DP schedule (N > 1 or --force_dp): auto = probe every candidate at this N and time the "
                    "fastest; a name = that schedule, no probes")
    ap.add_argument("--candidates", default=",".join(SCHEDULES), help="comma list of the schedules --schedule auto "
                    "probes")
    ap.add_argument("--probe_steps", type=int, default=200, help="timed steps per schedule probe (untimed for the "
                    "record)")
    ap.add_argument("--probe_warmup", type=int, default=60, help="untimed steps before each probe's timing")
    ap.add_argument("--zero", type=int, default=-1, help="override: 1/0 = ZeRO-1 fc1 sharding on/off (fixes the "
                    "schedule together with --fc_sfb; -1 = from --schedule)")
    ap.add_argument("--fc_sfb", type=int, default=-1, help="override: 1/0 = sufficient-factor fc gradients on/off "
                    "(-1 = from --schedule)")
    ap.add_argument("--merge_reduce", type=int, default=-1, help="override with --fc_sfb 1: 1/0 = conv slab reduce "
                    "inside the SFB GEMM launch on/off (-1 = from --schedule; with --fc_sfb/--zero alone: 1)")
    ap.add_argument("--min_warmup_ms", type=float, default=300.0, help="after --warmup steps, keep replaying "
                    "untimed steps until this much warm-up time has passed (GPU clock ramp; reported in the JSON)")
    ap.add_argument("--graph_steps", type=int, default=20, help="training steps captured per hipGraph "
                    "(device-side step counter/data cursor/dropout key make step i+1 of a graph the next step)")
    ap.add_argument("--lead_steps", type=int, default=0, help="timed region: launch this many one-step graphs "
                    "first, then ONE graph of the remaining steps (the GPU starts on the small launch while the "
                    "host enqueues the big one)")
    ap.add_argument("--lead_eager", type=int, default=0, help="timed region: launch this many steps as plain "
                    "kernel launches first, then ONE graph of the remaining steps (the GPU starts on the first "
                    "kernel while the host writes the graph's packets)")
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
    ap.add_argument("--fused_tail", type=int, default=1, help="1: on one GPU the Adam kernel also reduces the "
                    "conv weight-gradient slabs and bumps the step (one kernel less)")
    ap.add_argument("--local_bf16_grads", type=int, default=1, help="1: on one GPU keep the fc-region gradients "
                    "in bf16 (the DP all-reduce wire format): fc backward writes and Adam reads 2 B per gradient")
    ap.add_argument("--state_steps", type=int, default=100, help="time the steps that follow this many training "
                    "steps from init (snapshot before the clock-ramp warm-up, restored before the timed region); "
                    "0: time whatever state the warm-up steps left")
    ap.add_argument("--data", default="strokes", choices=["strokes", "random"], help="device-resident training "
                    "set: learnable class-conditional strokes (default) or uniform noise with random labels")
    ap.add_argument("--fp32_also", type=int, default=-1, help="after the bf16 headline, time the fp32 step (the "
                    "reference's precision) with the same protocol and report it under \"fp32\": 1 always, 0 never, "
                    "-1 at world 1 only")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu", action="store_true", help="plumbing dry-run: fp32 PyTorch CPU runner + Gloo "
                    "(exercises the launcher/barrier/JSON contract without a GPU; not a performance number)")
    return ap.parse_args(argv)


def _candidates(a, dp: bool):
    """(names to run, how the schedule was chosen). No DP: the one-GPU step, no schedule."""
    if not dp:
        return [None], "single"
    if a.dtype == "fp32":  # fp32 DP all-reduces the whole fp32 buffer (no SFB / ZeRO variants)
        return ["allreduce"], "fp32"
    if a.fc_sfb >= 0 or a.zero >= 0 or a.merge_reduce >= 0:  # explicit switches fix the schedule
        sfb = a.fc_sfb != 0
        zero = a.zero == 1
        name = ("sfb+zero" if zero else "sfb") if sfb else ("allreduce" if not zero else None)
        if name is None:
            raise SystemExit("error: --zero 1 needs --fc_sfb 1 (the ZeRO-1 path of this bench rides the SFB step)")
        if sfb and a.merge_reduce != 0:
            name += "+mr"
        return [name], "flag"
    if a.schedule != "auto":
        return [a.schedule], "flag"
    names = [c.strip() for c in a.candidates.split(",") if c.strip()]
    bad = [c for c in names if c not in SCHEDULES]
    if bad or not names:
        raise SystemExit(f"error: unknown schedule candidates {bad} (known: {list(SCHEDULES)})")
    return names, "probe"


class _Job:
    """One configured engine: params initialised on rank 0 and broadcast (reference M6), the
    device-resident dataset attached, the DP transport wired for ``sched``, graphs captured."""

    def __init__(self, a, ctx, data, labels, sched, graph_steps, extra_graph=0):
        import torch

        from tensorflow_distributed_amd.models import mnist_cnn as M
        from tensorflow_distributed_amd.parallel.transport import attach_engine

        self.a, self.ctx = a, ctx
        dev, rank, world = ctx.device, ctx.rank, ctx.world
        self.sched = sched
        cfg = SCHEDULES[sched] if sched else {"fc_sfb": 0, "zero": 0, "merge_reduce": 0}
        self.zero = bool(cfg["zero"]) and a.dtype == "bf16"
        eng = torch.classes.tfd.MnistEngine(a.batch_size, dev.index, 0.75, a.seed, rank)
        eng.set_adam(a.lr, 0.9, 0.999, 1e-8)
        eng.set_dtype(a.dtype)
        eng.set_fused_tail(a.fused_tail)
        eng.set_local_bf16_grads(a.local_bf16_grads)
        mode = a.transport
        if mode == "auto":
            mode = "ipc" if ctx.shared_device else "rccl"
        self.tr = attach_engine(eng, rank, world, dev, mode=mode, comm=ctx.comm, bf16=not a.fp32_grads,
                                small_ipc=bool(a.ipc_small), force_dp=bool(a.force_dp),
                                sfb=bool(cfg["fc_sfb"]) and a.dtype == "bf16", zero=self.zero)
        if self.zero:
            eng.set_zero(True)
        eng.set_sfb_merge_reduce(bool(cfg["merge_reduce"]))
        self.eng = eng
        self.stream = s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            g = torch.Generator(device=dev).manual_seed(1000 + rank)
            perm = torch.randperm(data.shape[0], device=dev, generator=g).to(torch.int32)
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
            self.graph_mode = not a.eager
            eng.train_step()  # one eager step first: sets kernel attributes outside capture
            self.gsteps = max(1, graph_steps)
            if self.graph_mode:
                try:
                    eng.capture_train_step("train")
                    if self.gsteps > 1:
                        eng.capture_train_steps("trainN", self.gsteps)
                    if extra_graph:
                        eng.capture_train_steps("timed", extra_graph)
                except Exception as e:  # pragma: no cover - capture support depends on the RCCL build
                    print(f"# hipGraph capture failed ({e!r}); timing eager launches", file=sys.stderr)
                    self.graph_mode = False

    def run(self, k):
        eng, gs = self.eng, self.gsteps
        if not self.graph_mode:
            for _ in range(k):
                eng.train_step()
            return
        if gs > 1 and k >= gs:
            eng.replay("trainN", k // gs)
        if k % gs or gs == 1:
            eng.replay("train", k % gs if gs > 1 else k)

    def close(self):
        """Tear down after every rank's kernels finished (a peer may still read our IPC staging)."""
        import torch

        torch.cuda.synchronize(self.ctx.device)
        self.ctx.barrier()
        for name in ("train", "trainN", "timed", "phases"):
            self.eng.drop_graph(name)
        self.tr.close()
        self.ctx.barrier()
        self.eng = None


def _probe_once(a, ctx, data, labels, sched) -> float:
    """Local ms/step of ``sched``: fresh engine + transport, ``--probe_warmup`` untimed steps, then
    ``--probe_steps`` graph-replayed steps between barriers. Setup failures are agreed on first, so
    no rank enters the timing collectives alone."""
    import torch

    job, err = None, None
    try:
        job = _Job(a, ctx, data, labels, sched, a.graph_steps)
    except Exception as e:  # noqa: BLE001 - agreed below
        err = e
    if ctx.max_scalar(1.0 if err is not None else 0.0) > 0:
        if job is not None:
            job.close()
        raise RuntimeError(f"setup failed on at least one rank (here: {err!r})")
    _CUR["tr"] = job.tr
    dt, err = 0.0, None
    try:
        with torch.cuda.stream(job.stream):
            job.run(a.probe_warmup)
        torch.cuda.synchronize(ctx.device)
        ctx.barrier()
        t0 = time.perf_counter()
        with torch.cuda.stream(job.stream):
            job.run(a.probe_steps)
        torch.cuda.synchronize(ctx.device)
        dt = time.perf_counter() - t0
        job.tr.check(f"schedule probe {sched}")
    except Exception as e:  # noqa: BLE001 - agreed after the teardown barriers
        err = e
    job.close()
    _CUR["tr"] = None
    # a timed-section failure (an IPC timeout caught by check) on one rank is raised on EVERY rank,
    # so no rank goes on alone into the next candidate's collectives
    if ctx.max_scalar(1.0 if err is not None else 0.0) > 0:
        raise RuntimeError(f"schedule probe {sched} failed on at least one rank (here: {err!r})")
    return dt * 1e3 / max(1, a.probe_steps)


_CUR = {"tr": None}  # the live DP transport, for the watchdog's error-word report


def _watchdog(rank):
    from tensorflow_distributed_amd.utils.tracing import PhaseWatchdog

    return PhaseWatchdog(rank, err_fn=lambda: _CUR["tr"].error() if _CUR["tr"] is not None else 0, tag="bench.py")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    a = _args(argv)
    from tensorflow_distributed_amd.parallel import spawn

    if spawn.needs_self_launch(a.gpus):
        # no launcher environment: this process only spawns the N ranks (it never touches the GPU)
        return spawn.self_launch(os.path.abspath(__file__), argv, a.gpus)
    if a.cpu:
        return _cpu_dry_run(a)

    import torch

    from tensorflow_distributed_amd import _native
    from tensorflow_distributed_amd.parallel import dist as D
    from tensorflow_distributed_amd.parallel import schedule as SCH

    wd = _watchdog(int(os.environ.get("RANK", "0")))
    wd.phase("setup: native library, process group, RCCL/IPC bootstrap, dataset", 600)
    _native.require()
    ctx = D.init_from_env(use_gpu=True)
    world, rank = ctx.world, ctx.rank
    spawn.check_world(a.gpus, world)
    dev = ctx.device
    B = a.batch_size
    n_data = 55000
    if a.data == "strokes":  # the learnable synthetic MNIST set (same images on every rank, like the
        # reference's workers that all read the full training split, mnist_python_m.py:291)
        from tensorflow_distributed_amd.utils.input_data import synthetic_mnist

        xi, yi = synthetic_mnist(n_data, 0)
        data = torch.from_numpy(xi.reshape(n_data, 784)).to(dev).float().div_(255.0)
        labels = torch.from_numpy(yi.astype("int32")).to(dev)
    else:
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        data = torch.rand(n_data, 784, device=dev, generator=g)
        labels = torch.randint(0, 10, (n_data,), device=dev, generator=g, dtype=torch.int32)
    torch.cuda.synchronize(dev)

    dp = world > 1 or bool(a.force_dp)
    cands, source = _candidates(a, dp)
    probe_ms = None
    if source == "probe" and len(cands) > 1:
        log = (lambda m: print(m, file=sys.stderr, flush=True)) if rank == 0 else None

        def probe_one(name):
            wd.phase(f"schedule probe {name} (setup, {a.probe_warmup} + {a.probe_steps} steps, teardown)",
                     180 + 0.05 * (a.probe_warmup + a.probe_steps))
            return _probe_once(a, ctx, data, labels, name)

        probe_ms = SCH.probe(cands, probe_one, ctx.max_scalar, log)
        sched = SCH.pick(probe_ms)
    else:
        sched = cands[0]

    res = _measure(a, ctx, data, labels, sched, wd, "bf16" if a.dtype == "bf16" else "fp32")
    job, tr, eng = res["job"], res["job"].tr, res["job"].eng
    topo = _job_topology(ctx, dev, tr, eng)
    phases = _phase_breakdown(eng, job.stream, job.graph_mode, world, ctx) if a.phases else None
    # the phase steps ran on the job's stream: wait for them before reading the state on the default
    # stream (without this the last step's loss rows could be read mid-write: two runs of the same
    # binary printed the loss of step N or N - 1)
    torch.cuda.synchronize(dev)
    _finish_losses(res)
    res_g = {k: v for k, v in res.items() if k not in ("job", "loss0_t")}
    ms = res["dt"] * 1e3 / a.steps
    img_s = world * B * a.steps / res["dt"]
    graph_mode, gsteps = job.graph_mode, job.gsteps
    kind, zero = tr.kind, job.zero
    tr.close()
    # The reference's precision (fp32 variables and arithmetic, /root/reference/mnist_python_m.py:185-200)
    # timed in the same process after the bf16 headline: same steps, warm-up and learning-state
    # protocol, reported beside it. World 1 by default (--fp32_also -1).
    fp32 = None
    if a.dtype == "bf16" and (a.fp32_also == 1 or (a.fp32_also < 0 and world == 1)):
        job.eng = None
        del res, job, eng
        torch.cuda.synchronize(dev)
        a32 = argparse.Namespace(**vars(a))
        a32.dtype, a32.lead_steps = "fp32", 0
        r32 = _measure(a32, ctx, data, labels, "allreduce" if dp else None, wd, "fp32")
        torch.cuda.synchronize(dev)
        _finish_losses(r32)
        fp32 = {"ms_per_step": round(r32["dt"] * 1e3 / a.steps, 5),
                "images_per_s": round(world * B * a.steps / r32["dt"], 1),
                "gpu_event_ms_per_step": round(r32["gpu_ms"] / a.steps, 5),
                "steps": a.steps, "warmup": a.warmup, "warmup_extra_steps": r32["extra"],
                "train_state": {"global_step": r32["gstep"], "loss_before_timed": round(r32["loss0"], 4),
                                "loss_after_timed": round(r32["loss1"], 4),
                                "minibatch_accuracy": round(r32["acc1"], 4)},
                "schedule": "allreduce" if dp else None,
                "what": "fp32 operands, fp32 MFMA (v_mfma_f32_16x16x4_f32), fp32 master/Adam: the reference's precision"}
        r32["job"].tr.close()
        if rank == 0:
            print(f"# fp32 (reference precision): {fp32['ms_per_step']:.4f} ms/step, {fp32['images_per_s']:.0f} img/s",
                  file=sys.stderr)
    if rank == 0:
        print(f"# world={world} B/gpu={B} schedule={sched} steps={a.steps} global_step={res_g['gstep']} "
              f"loss {res_g['loss0']:.3f}->{res_g['loss1']:.3f} acc {res_g['acc1']:.3f} {ms:.4f} ms/step",
              file=sys.stderr)
        print(json.dumps({
            "metric": METRIC,
            "value": round(img_s, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_extra_steps": res_g["extra"],
            "train_state": {"global_step": res_g["gstep"], "loss_before_timed": round(res_g["loss0"], 4),
                            "loss_after_timed": round(res_g["loss1"], 4),
                            "minibatch_accuracy": round(res_g["acc1"], 4), "state_steps": a.state_steps},
            "ms_per_step": round(ms, 5),
            "gpu_event_ms_per_step": round(res_g["gpu_ms"] / a.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / BASELINE_IMG_PER_S, 1),
            "dtype": a.dtype,
            "data": DATA_DESC[a.data],
            "phases_ms": phases,
            "schedule": {"chosen": sched, "source": source,
                         "candidates_ms_per_step": ({k: round(v, 5) for k, v in probe_ms.items()}
                                                    if probe_ms else None),
                         "probe_steps": a.probe_steps if probe_ms else 0},
            **topo,
            "fp32": fp32,
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
                "dp_transport": kind,
                "force_dp": bool(a.force_dp),
                "zero1_fc1": zero,
                "fc_grads": ("fp32" if a.dtype == "fp32" else
                             "summed from all-gathered factors (sfb), bf16" if "sfb" in kind else
                             "bf16" if (a.local_bf16_grads or world > 1) and not a.fp32_grads else "fp32"),
            },
        }), flush=True)
    wd.stop()
    ctx.shutdown()
    if not topo["replicas_identical"]:
        print("error: DP replicas diverged (parameter digests differ across ranks)", file=sys.stderr)
        return 3
    return 0


def _finish_losses(res):
    """Host reads of the losses / accuracy / step of a measured job (after its stream is drained)."""
    eng = res["job"].eng
    if res["loss0"] is None:
        res["loss0"] = float(res["loss0_t"].item())
    res["loss1"] = float(eng.loss_rows().mean().item())
    res["acc1"] = float(eng.correct_rows().mean().item())  # last timed step's minibatch accuracy (train mode)
    res["gstep"] = int(eng.step_tensor().item())


def _measure(a, ctx, data, labels, sched, wd, label):
    """Set up one job (engine, transport, graphs) and run the timing protocol on it: ``--state_steps``
    steps from init (snapshotted), ``--warmup`` + clock-ramp warm-up steps, state restored, then
    EXACTLY ``--steps`` replayed steps between a barrier + synchronize on both sides; ``dt`` is the
    max over ranks."""
    import torch

    dev, rank = ctx.device, ctx.rank
    wd.phase(f"{label} job setup ({sched}): engine, transport, graph capture", 300)
    lead = max(0, min(a.lead_steps, a.steps - 1)) if not a.eager else 0
    lead_e = max(0, min(a.lead_eager, a.steps - 1)) if not a.eager and not lead else 0
    job = _Job(a, ctx, data, labels, sched, a.graph_steps,
               extra_graph=(a.steps - lead - lead_e) if (lead or lead_e) else 0)
    eng, tr, s, run = job.eng, job.tr, job.stream, job.run
    _CUR["tr"] = tr
    wd.phase(f"{label} warm-up ({a.state_steps} state + {a.warmup} steps + {a.min_warmup_ms:.0f} ms)",
             180 + 0.05 * (a.state_steps + a.warmup) + a.min_warmup_ms / 1e3)
    if not job.graph_mode:
        lead = lead_e = 0
    loss0_t = None
    with torch.cuda.stream(s):
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

    wd.phase(f"{label} timed region ({a.steps} steps)", 120 + 0.05 * a.steps)
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
        elif lead_e:
            for _ in range(lead_e):
                eng.train_step()
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
    wd.phase(f"{label} report: replica digests, phase breakdown, teardown", 300)
    gpu_ms = ev0.elapsed_time(ev1)  # device time of the same K steps (diagnostic: host/sync overhead = dt - this)
    if job.zero:
        with torch.cuda.stream(s):
            eng.sync_params()
    dt = ctx.max_scalar(dt)
    tr.check("after the timed steps")
    return {"job": job, "dt": dt, "gpu_ms": gpu_ms, "extra": extra, "loss0": loss0, "loss0_t": loss0_t}


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
    from tensorflow_distributed_amd.parallel import schedule as SCH
    from tensorflow_distributed_amd.parallel import spawn
    from tensorflow_distributed_amd.parallel.sync_replicas import SyncReplicasStepper, broadcast_state
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer

    ctx = D.init_from_env(use_gpu=False)
    world, rank = ctx.world, ctx.rank
    spawn.check_world(a.gpus, world)
    g = torch.Generator().manual_seed(1000 + rank)
    x = torch.rand(a.batch_size, 784, generator=g)
    y = torch.randint(0, 10, (a.batch_size,), generator=g)

    def make():
        r = TorchMnistRunner(a.batch_size, AdamOptimizer(a.lr), keep_prob=0.75, seed=a.seed, rank=rank)
        if rank == 0:
            r.load_flat(M.flat_from_dict(M.init_params(a.seed)), {}, 0)
        if world > 1:
            broadcast_state(r, 0)
        return SyncReplicasStepper(r, rank, world, world)

    # the same probe/choose protocol as the GPU path, over CPU "schedules" (the Gloo all-reduce of
    # the whole flat gradient, or of the conv and fc buckets separately), so its collective
    # discipline is covered by the CPU suite
    from tensorflow_distributed_amd.parallel.sync_replicas import GlooGradAverager

    def configure(st, name):
        if world > 1:
            st.runner.comm = GlooGradAverager(None, world, [M.BUCKET_SPLIT] if name == "buckets" else None)

    probe_ms = None
    if world > 1 and a.schedule == "auto":
        def one(name):
            st = make()
            configure(st, name)
            st.step(x, y)
            ctx.barrier()
            t0 = time.perf_counter()
            for _ in range(max(1, min(a.probe_steps, 5))):
                st.step(x, y)
            return (time.perf_counter() - t0) * 1e3 / max(1, min(a.probe_steps, 5))

        probe_ms = SCH.probe(["flat", "buckets"], one, ctx.max_scalar)
        chosen = SCH.pick(probe_ms)
    else:
        chosen = "flat"
    st = make()
    configure(st, chosen)
    for _ in range(a.warmup):
        st.step(x, y)
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st.step(x, y)
    ctx.barrier()
    dt = ctx.max_scalar(time.perf_counter() - t0)
    digest = float(st.runner.params().double().sum())
    hi, lo = ctx.max_scalar(digest), -ctx.max_scalar(-digest)
    if rank == 0:
        print(json.dumps({"metric": "images/sec (whole node) MNIST CNN DP [CPU dry-run]", "value": world * a.batch_size * a.steps / dt,
                          "unit": "images/s", "n_gpus": 0, "n_ranks": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": dt * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
                          "schedule": {"chosen": chosen, "candidates_ms_per_step": probe_ms},
                          "replicas_identical": hi == lo,
                          "config": {"model": "mnist_cnn", "global_batch": world * a.batch_size, "seq_len": None,
                                     "parallelism": f"dp{world}", "device": "cpu"}}), flush=True)
    ctx.shutdown()
    return 0 if hi == lo else 3


if __name__ == "__main__":
    sys.exit(main())
