"""The distributed trainer behind ``mnist_python_m.py`` / ``mnist_python_w1.py`` / ``mnist_python_w2.py``
(``/root/reference/mnist_python_m.py:49-326``): same 14 flags and defaults, same roles, same stdout.

Roles:
  * ``--job_name=ps``: hosts the rendezvous store at ``--ps_hosts[task_index]`` (task 0), joins the
    control group and runs ``server.join()`` -- the async parameter-server service when
    ``--sync_replicas=False``, otherwise it just waits for the workers' completion signal.
  * ``--job_name=worker``: task 0 is the chief. GPU ``task_index % num_gpus`` (``--num_gpus>0``)
    or CPU. Chief initialises (or restores) and broadcasts; the loop runs until the GLOBAL step
    reaches ``--train_steps``; then a 5 x 1000 validation pass.

Sync mode = all-reduce DP with SyncReplicasOptimizer semantics (parallel/sync_replicas.py); async
mode = Hogwild PS over Gloo point-to-point (parallel/async_ps.py).
"""
from __future__ import annotations

import os
import sys
import tempfile
import time

import numpy as np
import torch

from ..utils import flags as flags_mod
from ..utils.flags import FLAGS

_DEFINED = False


def define_flags(task_index_default: int = 0, job_name_default: str = "ps") -> None:
    """The reference's 14 flags (mnist_python_m.py:49-87) + framework extras."""
    global _DEFINED
    f = flags_mod
    if _DEFINED:
        FLAGS._flags["task_index"].default = task_index_default
        FLAGS._flags["job_name"].default = job_name_default
        FLAGS.reset()
        return
    _DEFINED = True
    f.DEFINE_string("data_dir", "/tmp/mnist-data", "Directory for storing mnist data")
    f.DEFINE_boolean("download_only", False, "Only perform downloading of data; Do not proceed to "
                     "session preparation, model definition or training")
    f.DEFINE_integer("task_index", task_index_default, "Worker task index, should be >= 0. task_index=0 is "
                     "the master worker task the performs the variable initialization ")
    f.DEFINE_integer("num_gpus", 0, "Total number of gpus for each machine. If you don't use GPU, please set it to '0'")
    f.DEFINE_integer("replicas_to_aggregate", 2, "Number of replicas to aggregate before parameter update"
                     "is applied (For sync_replicas mode only; default: num_workers)")
    f.DEFINE_integer("hidden_units", 100, "Number of units in the hidden layer of the NN (unused by the CNN, "
                     "kept for flag compatibility)")
    f.DEFINE_integer("train_steps", 4, "Number of (global) training steps to perform")
    f.DEFINE_integer("batch_size", 128, "Training batch size")
    f.DEFINE_float("learning_rate", 0.01, "Learning rate")
    f.DEFINE_boolean("sync_replicas", True, "Use the sync_replicas (synchronized replicas) mode, "
                     "wherein the parameter updates from workers are aggregated before applied to "
                     "avoid stale gradients")
    f.DEFINE_boolean("existing_servers", False, "Whether servers already exists. If True, will use "
                     "the worker hosts via their GRPC URLs (one client process per worker host). "
                     "Otherwise, will create an in-process TensorFlow server.")
    f.DEFINE_string("ps_hosts", "10.0.1.3:2222", "Comma-separated list of hostname:port pairs")
    f.DEFINE_string("worker_hosts", "10.0.1.6:2223,10.0.1.2:2224", "Comma-separated list of hostname:port pairs")
    f.DEFINE_string("job_name", job_name_default, "job name: worker or ps")
    # ---- framework extras ----
    f.DEFINE_string("logdir", "", "Supervisor logdir (checkpoints, events). Empty = tempfile.mkdtemp() "
                    "like the reference; set it to a stable path to enable resume")
    f.DEFINE_float("save_model_secs", 600.0, "Checkpoint period (chief)")
    f.DEFINE_float("save_summaries_secs", 120.0, "Summary (global_step/sec) period (chief)")
    f.DEFINE_integer("seed", 0, "Init seed (normal(0,1) params, chief)")
    f.DEFINE_float("keep_prob", 0.75, "Dropout keep probability during training")
    f.DEFINE_enum("optimizer", "adam", ["adam", "sgd", "momentum"], "Optimizer (reference: adam)")
    f.DEFINE_float("momentum", 0.9, "Momentum for --optimizer=momentum")
    f.DEFINE_boolean("synthetic_data", False, "Use the synthetic MNIST-shaped dataset even if IDX files exist")
    f.DEFINE_boolean("bf16_grads", True, "All-reduce gradients in bf16 (GPU)")
    f.DEFINE_boolean("use_graph", True, "Replay the captured hipGraph of the train step (GPU)")
    f.DEFINE_integer("eval_batches", 5, "Validation batches after training")
    f.DEFINE_integer("eval_batch_size", 1000, "Validation batch size")
    f.DEFINE_string("metrics_file", "", "Chief: JSONL metrics per step")
    f.DEFINE_string("trace_file", "", "Chrome-trace JSON of host step phases")
    f.DEFINE_integer("check_consistency_every", 0, "Every N steps all-reduce a param checksum and "
                     "fail on cross-worker desync (sync mode)")
    f.DEFINE_integer("fault_inject_step", -1, "Test hook: the worker --fault_inject_task exits abruptly "
                     "when its global step reaches this value (first attempt only)")
    f.DEFINE_integer("fault_inject_task", -1, "Worker task index for --fault_inject_step")
    f.DEFINE_string("straggler_delay", "", "Test hook: 'task:seconds,...' artificial per-step delay "
                    "(backup-worker tests)")
    f.DEFINE_float("rendezvous_timeout", 600.0, "Seconds to wait for the cluster to assemble")
    f.DEFINE_boolean("quiet", False, "Suppress per-step prints")
    f.DEFINE_boolean("debug_sync", False, "Serialise every HIP launch/copy (AMD_SERIALIZE_KERNEL=3, "
                     "HIP_LAUNCH_BLOCKING=1): race-hunting mode")
    f.DEFINE_float("step_timeout_secs", 0.0, "Watchdog: abort the communicator and exit non-zero when no step "
                   "completes for this long (0 = off); the launcher then restarts from the last checkpoint")
    f.DEFINE_string("eval_at_steps", "", "Chief: comma-separated global steps at which to run the validation "
                    "pass and print a 'performance' table row (steps, training seconds, accuracy %, lr)")
    f.DEFINE_boolean("log_device_placement", False, "Print where every variable and the compute live "
                     "(ConfigProto.log_device_placement, mnist_python_m.py:257)")
    f.DEFINE_enum("dp_transport", "auto", ["auto", "rccl", "ipc"], "GPU sync gradient transport: auto = "
                  "peer-to-peer IPC when workers share a GPU (--num_gpus < workers; RCCL refuses that), else "
                  "RCCL over xGMI (+ IPC one-shot for the small conv bucket)")
    f.DEFINE_string("dp_schedule", "fixed", "Sync DP schedule (workers > 1). fixed (default) = one schedule per "
                    "device/dtype, so two identical runs train the same trajectory (GPU bf16 sfb+zero+mr, GPU fp32 "
                    "allreduce, CPU flat); auto = before training every worker times each candidate for "
                    "--dp_probe_steps steps and all keep the fastest (max over workers) -- the schedules round "
                    "differently, so auto trades bit-reproducibility across runs for speed; or "
                    "a name. GPU bf16: sfb+zero+mr, sfb+mr, sfb+zero, sfb, allreduce (parallel/schedule.py: "
                    "sufficient-factor fc gradients, ZeRO-1 fc1 sharding, slab reduce merged into the SFB GEMM, "
                    "bucketed all-reduce); GPU fp32: allreduce; CPU (Gloo): flat, buckets")
    f.DEFINE_integer("dp_probe_steps", 200, "Timed steps per --dp_schedule=auto candidate (CPU: at most 5)")
    f.DEFINE_integer("dp_probe_warmup", 30, "Untimed steps before each candidate's timing (CPU: 1)")
    f.DEFINE_integer("zero_sync_every", 100, "ZeRO-1 schedules: every this many global steps all workers agree "
                     "whether the chief's checkpoint is due and, if so, gather the sharded fc1 state first")
    f.DEFINE_boolean("phase_timing", False, "GPU: HIP timing events at the step's phase boundaries (forward, fc "
                     "backward, conv backward, optimizer, all-reduce), written to --metrics_file (always on when "
                     "--metrics_file is set on the chief)")
    f.DEFINE_enum("dtype", "bf16", ["bf16", "fp32"], "GPU compute precision: bf16 MFMA operands (fp32 accumulate, "
                  "master weights and optimizer), or fp32 everywhere (the reference's precision, "
                  "mnist_python_m.py:185-200)")
    f.DEFINE_float("bucket_mb", 0.0, "Gradient all-reduce bucketing: 0 = the MNIST engine's two buckets (fc 12.9 "
                   "MB over RCCL, conv 0.2 MB over the IPC one-shot kernel); > 0 = bucket size for the "
                   "generic bucket reducer (--model resnet*)")
    f.DEFINE_enum("model", "mnist_cnn", ["mnist_cnn", "resnet18", "resnet50"], "Model: the reference CNN, or the "
                  "synthetic-ImageNet ResNet family (BASELINE configs 4-5; trained by bench_resnet.py)")
    f.DEFINE_integer("image_size", 224, "--model resnet*: synthetic image height = width")
    f.DEFINE_boolean("bn_deterministic", False, "--model resnet*: batch-norm statistics in row mode (fixed summation "
                     "order, bit-reproducible runs) instead of slot mode's fp32 atomics (~3 % faster, order varies)")
    f.DEFINE_boolean("ps_on_gpu", True, "Parameter-server modes (async, backup workers) with --num_gpus > 0: each "
                     "ps task keeps its variables, optimizer slots and accumulator on GPU task_index % num_gpus; "
                     "workers push gradients into its GPU mailbox and the ps writes fresh values straight into "
                     "the workers' engine parameters (IPC peer memory, no host copies). False = the reference's "
                     "CPU ps (ps_device=/job:ps/cpu:0)")
    f.DEFINE_boolean("device_input", True, "GPU: upload the training split once and index it on the device "
                     "by a per-epoch shuffle (no per-step host feed); False = host next_batch + H2D per step")


def _make_optimizer():
    from .optimizers import AdamOptimizer, GradientDescentOptimizer, MomentumOptimizer

    if FLAGS.optimizer == "sgd":
        return GradientDescentOptimizer(FLAGS.learning_rate)
    if FLAGS.optimizer == "momentum":
        return MomentumOptimizer(FLAGS.learning_rate, FLAGS.momentum)
    return AdamOptimizer(FLAGS.learning_rate)


def host_identity() -> str:
    """This machine as far as IPC peer memory is concerned: hostname + kernel boot id."""
    import socket

    boot = ""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        pass
    return f"{socket.gethostname()}|{boot}"


def gpu_ps_capable() -> bool:
    """This task could run its side of the GPU-resident PS (flags + a visible GPU)."""
    return bool(FLAGS.ps_on_gpu and FLAGS.num_gpus > 0 and FLAGS.model == "mnist_cnn" and torch.cuda.is_available())


def agree_gpu_ps(capable: bool, host: str, group=None):
    """All-gather (host identity, capable) over every ps and worker task of ``group``. Returns
    (use the GPU-resident PS, reason if not): yes only if every task is capable and all share one
    host; otherwise every task falls back to the host parameter server -- the same answer on all."""
    import torch.distributed as dist

    rows = [(host, bool(capable))]
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        rows = [None] * dist.get_world_size(group)
        dist.all_gather_object(rows, (host, bool(capable)), group=group)
    if len({h for h, _ in rows}) > 1:
        return False, "tasks on different hosts"
    if not all(c for _, c in rows):
        return False, "a task without a GPU or with --ps_on_gpu=False"
    return True, ""


def _agree_gpu_ps() -> bool:
    ok, why = agree_gpu_ps(gpu_ps_capable(), host_identity())
    if FLAGS.ps_on_gpu and not ok:
        print("%s %d: --ps_on_gpu needs every task on one host with a GPU (%s); using the host parameter server"
              % (FLAGS.job_name, FLAGS.task_index, why))
    return ok


def _set_bn_mode(deterministic: bool) -> None:
    """--bn_deterministic: batch-norm statistics in row mode (fixed summation order). The switch is an
    op of _C.so, which nothing on the path to here has loaded yet: load it first."""
    if deterministic:
        from .. import _native

        _native.ops().set_bn_part_slots(0)


def _resnet_worker(server, cluster, num_workers: int, is_chief: bool) -> int:
    """``--model resnet18|resnet50``: the same cluster roles, stdout and Supervisor services as the MNIST
    path, training the synthetic-ImageNet ResNet family (BASELINE configs 4-5) with synchronous DP --
    bucketed bf16 gradient all-reduce (``--bucket_mb``, default 8) overlapped with the backward, fused
    SGD-momentum (lr = ``--learning_rate``). RCCL between GPUs; the IPC transport when workers share a
    GPU. Synthetic data: one device-resident random ``--image_size``^2 x 3 batch per worker.

    Supervisor (/root/reference/mnist_python_m.py:235-253): the chief restores the newest checkpoint
    in ``--logdir`` or keeps its seeded init, then params, momentum, BN running statistics and the
    global step go to every worker; timed checkpoints (``--save_model_secs``) in the MNIST layout
    (models/resnet.ResNetRunner); after training an inference-mode validation pass over
    ``--eval_batches`` synthetic batches and a final checkpoint."""
    import torch.distributed as dist

    from ..models.resnet import ResNet, ResNetRunner
    from ..parallel.ipc import IpcCollectives, make_ipc_comm
    from ..parallel.transport import devices_shared, make_rccl
    from .supervisor import Supervisor

    if not FLAGS.sync_replicas or FLAGS.num_gpus <= 0:
        raise ValueError("--model %s: synchronous data parallelism on GPUs only (--num_gpus > 0)" % FLAGS.model)
    _set_bn_mode(FLAGS.bn_deterministic)
    gpu = FLAGS.task_index % FLAGS.num_gpus
    torch.cuda.set_device(gpu)
    device = torch.device("cuda", gpu)
    depth = int(FLAGS.model.replace("resnet", ""))
    m = ResNet(depth, num_classes=1000, device=device, seed=FLAGS.seed)
    runner = ResNetRunner(m)
    comm = None
    grp = server.worker_group
    if num_workers > 1:
        if devices_shared(device, num_workers, grp):
            comm = IpcCollectives(make_ipc_comm(FLAGS.task_index, num_workers, gpu, m.fp.total, group=grp))
        else:
            comm = make_rccl(FLAGS.task_index, num_workers, gpu, group=grp, src=cluster.num_ps)
    m.set_comm(comm, FLAGS.bucket_mb or 8.0)

    def broadcast_fn():  # chief's (restored or seeded) state -> every worker (reference M6)
        if num_workers <= 1:
            return
        for t in [m.fp.master, m.fp.momentum] + [b for bn in m.bns for b in (bn.rmean, bn.rvar)]:
            host = t.detach().cpu()
            dist.broadcast(host, cluster.num_ps, group=grp)
            t.copy_(host.to(device))
        m.fp.shadow.copy_(m.fp.master)
        st = torch.tensor([runner.global_step()], dtype=torch.int64)
        dist.broadcast(st, cluster.num_ps, group=grp)
        runner.set_global_step(int(st.item()))

    logdir = FLAGS.logdir or tempfile.mkdtemp()
    sv = Supervisor(is_chief=is_chief, logdir=logdir, runner=runner, init_fn=lambda: None, broadcast_fn=broadcast_fn,
                    save_model_secs=FLAGS.save_model_secs, save_summaries_secs=FLAGS.save_summaries_secs,
                    recovery_wait_secs=1)
    if is_chief:
        print("Worker %d: Initializing session..." % FLAGS.task_index)
    else:
        print("Worker %d: Waiting for session to be initialized..." % FLAGS.task_index)
    sys.stdout.flush()
    sv.prepare_or_wait_for_session()
    print("Worker %d: Session initialization complete." % FLAGS.task_index)
    S = FLAGS.image_size
    g = torch.Generator(device=device).manual_seed(100 + FLAGS.task_index)
    x = torch.randn(FLAGS.batch_size, S, S, 3, device=device, generator=g)
    y = torch.randint(0, 1000, (FLAGS.batch_size,), device=device, generator=g, dtype=torch.int32)
    time_begin = time.time()
    print("Training begins @ %f" % time_begin)
    local_step = 0
    step = runner.global_step()
    while step < FLAGS.train_steps:
        loss = runner.train_step(x, y, lr=FLAGS.learning_rate)
        step = runner.global_step()
        local_step += 1
        if not FLAGS.quiet:
            print("%f: Worker %d: training step %d done (global step: %d) loss %.4f" % (
                time.time(), FLAGS.task_index, local_step, step, float(loss)))
        sv.on_step(step)
    torch.cuda.synchronize(device)
    time_end = time.time()
    print("Training ends @ %f" % time_end)
    el = time_end - time_begin
    print("Training elapsed time: %f s" % el)
    print("Worker %d: %.1f images/sec (this worker)" % (FLAGS.task_index, FLAGS.batch_size * local_step / max(el, 1e-9)))
    # validation (reference: 5 x 1000 images, mnist_python_m.py:309-320): synthetic batches of at most
    # --batch_size images through the inference-mode network (running BN statistics)
    gv = torch.Generator(device=device).manual_seed(7 + FLAGS.task_index)
    accs = []
    nb = min(FLAGS.eval_batch_size, FLAGS.batch_size)
    for _ in range(FLAGS.eval_batches):
        vx = torch.randn(nb, S, S, 3, device=device, generator=gv)
        vy = torch.randint(0, 1000, (nb,), device=device, generator=gv, dtype=torch.int32)
        _, correct = m.evaluate(vx, vy)
        print("After %d training step(s)", FLAGS.train_steps)  # verbatim reference line (quirk Q3)
        print("Accuracy : %f" % (correct / float(nb)))
        accs.append(correct / float(nb))
    print("Mean Accuracy : %f" % (sum(accs) / len(accs) if accs else float("nan")))
    sys.stdout.flush()
    if num_workers > 1:
        dist.barrier(group=grp)
    sv.stop(save=True)
    if isinstance(comm, IpcCollectives):
        if comm.ipc.error():
            raise RuntimeError("IPC collective barrier timed out")
        comm.ipc.close()
    server.mark_done()
    server.shutdown()
    return 0


def _max_over(group, v: float) -> float:
    import torch.distributed as dist

    t = torch.tensor([float(v)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def dp_candidates(device_type: str, dtype: str):
    """The sync DP schedules this worker device can run (parallel/schedule.py), in probe order."""
    from ..parallel import schedule as SCH

    if device_type == "cuda":
        return list(SCH.MNIST_SCHEDULES) if dtype == "bf16" else ["allreduce"]
    return list(SCH.CPU_SCHEDULES)


def choose_dp_schedule(run_one, rank: int, num_workers: int, device_type: str, group=None, log=None):
    """(schedule, {candidate: ms/step max over workers} or None, how it was chosen).

    ``--dp_schedule=auto`` with more than one candidate: every worker times every candidate with
    ``run_one(name)`` (same names, same order), the slowest worker's time counts and all keep the
    fastest -- the same in-job probe as bench.py (parallel/schedule.py). The reference has one
    schedule, the PS star (/root/reference/mnist_python_m.py:177,210-233)."""
    from ..parallel import schedule as SCH

    known = dp_candidates(device_type, FLAGS.dtype)
    want = FLAGS.dp_schedule
    if want == "fixed":
        return known[0], None, "fixed"
    if want != "auto":
        if want not in known:
            raise ValueError("--dp_schedule=%s: not a %s schedule (known: %s)" % (want, device_type, ", ".join(known)))
        return want, None, "flag"
    if num_workers <= 1 or len(known) == 1:
        return known[0], None, "only"
    times = SCH.probe(known, run_one, lambda v: _max_over(group, v), log)
    return SCH.pick(times), times, "probe"


def _probe_gpu_schedule(name, mnist, device, num_workers, group, src, comm):
    """Local ms/step of one GPU DP schedule: a throwaway engine + transport on the worker's device,
    chief-style init, the device-resident split, --dp_probe_warmup untimed then --dp_probe_steps
    timed graph replays between barriers. Setup failures are agreed on first (no worker may enter
    the timing collectives alone)."""
    import torch.distributed as dist

    from ..models import mnist_cnn as M
    from ..models.mnist_runner import make_runner
    from ..parallel.schedule import MNIST_SCHEDULES
    from ..parallel.transport import attach_engine

    cfg = MNIST_SCHEDULES.get(name, {"fc_sfb": 0, "zero": 0, "merge_reduce": 0})
    r, tr, err = None, None, None
    try:
        r = make_runner(FLAGS.batch_size, _make_optimizer(), device, keep_prob=FLAGS.keep_prob, seed=FLAGS.seed,
                        rank=FLAGS.task_index, bf16_grads=FLAGS.bf16_grads, use_graph=True, dtype=FLAGS.dtype)
        tr = attach_engine(r.eng, FLAGS.task_index, num_workers, device, group=group, src=src, mode=FLAGS.dp_transport,
                           comm=comm, bf16=FLAGS.bf16_grads, sfb=bool(cfg["fc_sfb"]) and FLAGS.dtype == "bf16",
                           zero=bool(cfg["zero"]))
        if cfg["zero"]:
            r.eng.set_zero(True)
        r.eng.set_sfb_merge_reduce(bool(cfg["merge_reduce"]))
        r.comm, r.transport = tr.comm, tr
        r.set_device_dataset(mnist.train.images, mnist.train.labels, seed=FLAGS.seed * 1000 + FLAGS.task_index + 31)
        r.load_flat(M.flat_from_dict(M.init_params(FLAGS.seed)), {}, 0)
    except Exception as e:  # noqa: BLE001 - agreed below
        err = e
    if _max_over(group, 1.0 if err is not None else 0.0) > 0:
        if tr is not None:
            tr.close()
        raise RuntimeError("schedule probe setup failed on a worker (here: %r)" % (err,))
    try:
        r.train_step(None, None)  # eager step + capture of the step graph
        with torch.cuda.stream(r.stream):
            r.eng.replay("train", max(1, FLAGS.dp_probe_warmup))
        torch.cuda.synchronize(device)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        n = max(1, FLAGS.dp_probe_steps)
        with torch.cuda.stream(r.stream):
            r.eng.replay("train", n)
        torch.cuda.synchronize(device)
        dt = time.perf_counter() - t0
        tr.check("schedule probe %s" % name)
    except Exception as e:  # noqa: BLE001 - agreed after the teardown barriers
        err = e
    torch.cuda.synchronize(device)
    dist.barrier(group=group)  # a peer may still read this engine's IPC staging
    r.eng.drop_graph("train")
    tr.close()
    dist.barrier(group=group)
    # a timed-section failure (replay, or an IPC timeout caught by check) on one worker is raised on
    # EVERY worker, so none goes on alone into the next candidate's collectives
    if _max_over(group, 1.0 if err is not None else 0.0) > 0:
        raise RuntimeError("schedule probe %s failed on a worker (here: %r)" % (name, err))
    return dt * 1e3 / n


def _probe_cpu_schedule(name, num_workers, group):
    """Local ms/step of one Gloo schedule on the CPU runner (random batch, 1 + min(5, steps) steps)."""
    import torch.distributed as dist

    from ..models import mnist_cnn as M
    from ..models.mnist_runner import TorchMnistRunner
    from ..parallel.sync_replicas import GlooGradAverager

    r = TorchMnistRunner(FLAGS.batch_size, _make_optimizer(), FLAGS.keep_prob, FLAGS.seed, FLAGS.task_index)
    r.load_flat(M.flat_from_dict(M.init_params(FLAGS.seed)), {}, 0)
    r.comm = GlooGradAverager(group, num_workers, [M.BUCKET_SPLIT] if name == "buckets" else None)
    g = torch.Generator().manual_seed(FLAGS.task_index + 5)
    x = torch.rand(FLAGS.batch_size, 784, generator=g)
    y = torch.randint(0, 10, (FLAGS.batch_size,), generator=g)
    r.train_step(x, y)
    dist.barrier(group=group)
    n = max(1, min(FLAGS.dp_probe_steps, 5))
    t0 = time.perf_counter()
    for _ in range(n):
        r.train_step(x, y)
    return (time.perf_counter() - t0) * 1e3 / n


def main(argv=None) -> int:
    from ..models import mnist_cnn as M
    from ..models.mnist_runner import make_runner
    from ..parallel import async_ps, sync_replicas
    from ..parallel.cluster import ClusterSpec, Server
    from ..utils import input_data
    from ..utils.metrics import MetricsLogger, StepTimer
    from .optimizers import SyncReplicasOptimizer
    from .supervisor import Supervisor

    if FLAGS.download_only:
        # no network on MI355X boxes: materialise the IDX files (synthetic if absent) and stop
        print("MNIST data in %s: %s" % (FLAGS.data_dir, input_data.maybe_download(FLAGS.data_dir)))
        sys.exit(0)
    if FLAGS.debug_sync:
        from ..utils.tracing import enable_debug_sync

        enable_debug_sync()
    mnist = input_data.read_data_sets(FLAGS.data_dir, one_hot=True, fake_data=FLAGS.synthetic_data,
                                      seed=FLAGS.seed * 1000 + max(FLAGS.task_index, 0) + 17)

    if FLAGS.job_name is None or FLAGS.job_name == "":
        raise ValueError("Must specify an explicit `job_name`")
    if FLAGS.task_index is None or FLAGS.task_index == "":
        raise ValueError("Must specify an explicit `task_index`")

    print("job name = %s" % FLAGS.job_name)
    print("task index = %d" % FLAGS.task_index)

    ps_spec = FLAGS.ps_hosts.split(",")
    worker_spec = FLAGS.worker_hosts.split(",")
    num_workers = len(worker_spec)
    cluster = ClusterSpec({"ps": ps_spec, "worker": worker_spec})

    server = Server(cluster, job_name=FLAGS.job_name, task_index=FLAGS.task_index,
                    existing_servers=FLAGS.existing_servers, timeout_s=FLAGS.rendezvous_timeout)
    opt = _make_optimizer()
    layout = async_ps.mnist_layout(cluster.num_ps) if cluster.num_ps else None
    if not FLAGS.sync_replicas and layout is None:
        raise ValueError("--sync_replicas=False (async parameter-server mode) needs at least one --ps_hosts task")

    sync = FLAGS.sync_replicas
    r2a = num_workers
    if sync:
        r2a = FLAGS.replicas_to_aggregate if FLAGS.replicas_to_aggregate is not None else num_workers
        if r2a > num_workers:
            # TF1 would wait forever for gradients that never come; clamp instead (and say so)
            print("Worker %d: replicas_to_aggregate=%d > %d workers; aggregating %d" %
                  (FLAGS.task_index, r2a, num_workers, num_workers))
            r2a = num_workers
    # backup workers (R < N) with a ps task: TF's accumulator semantics on the PS (stale gradients of
    # stragglers dropped, the first R fresh ones averaged); without a ps task: the all-gather stepper
    backup_ps = sync and r2a < num_workers and layout is not None
    ps_mode = (not sync) or backup_ps

    # GPU-resident PS only when EVERY task (ps and worker) can take part: same host (the data path is
    # IPC peer memory) and a GPU on each. Decided collectively so the PS and the workers never pick
    # different protocols (the reference's default cluster spans three hosts, mnist_python_m.py:81-84).
    use_gpu_ps = ps_mode and _agree_gpu_ps()

    if FLAGS.job_name == "ps":
        # (reference quirk Q9: ps + existing_servers fell through to the worker code; a PS here
        #  always serves and then exits once every worker has finished)
        service = None
        if use_gpu_ps:
            from ..parallel.gpu_ps import GpuParameterServerService

            ps_gpu = FLAGS.task_index % FLAGS.num_gpus
            torch.cuda.set_device(ps_gpu)
            service = GpuParameterServerService(FLAGS.task_index, cluster.num_ps, num_workers, layout, opt,
                                                torch.device("cuda", ps_gpu), sync=backup_ps,
                                                replicas_to_aggregate=r2a)
        elif ps_mode:
            service = async_ps.ParameterServerService(FLAGS.task_index, cluster.num_ps, num_workers, layout, opt,
                                                      sync=backup_ps, replicas_to_aggregate=r2a)
        server.join(service)
        server.shutdown()
        if service is not None and backup_ps:
            print("ps %d: %d synchronous updates, %d stale gradients dropped" % (FLAGS.task_index, service.updates,
                                                                               service.dropped))
        return 0

    is_chief = FLAGS.task_index == 0
    if FLAGS.model != "mnist_cnn":
        return _resnet_worker(server, cluster, num_workers, is_chief)
    if FLAGS.num_gpus > 0:
        gpu = FLAGS.task_index % FLAGS.num_gpus
        torch.cuda.set_device(gpu)
        device = torch.device("cuda", gpu)
    else:
        device = torch.device("cpu")

    sopt = None
    if sync:
        sopt = SyncReplicasOptimizer(opt, replicas_to_aggregate=r2a, total_num_replicas=num_workers).resolve(num_workers)

    # Sync all-reduce DP: which schedule (parallel/schedule.py) -- probed in-job by every worker, or
    # fixed by --dp_schedule. One RCCL communicator serves every probe and the training run.
    dp_sched, dp_probe, dp_source, rccl = None, None, None, None
    allreduce_dp = sync and num_workers > 1 and not backup_ps
    if allreduce_dp:
        grp = server.worker_group
        if device.type == "cuda":
            from ..parallel.transport import devices_shared, make_rccl

            if FLAGS.dp_transport != "ipc" and not devices_shared(device, num_workers, grp):
                rccl = make_rccl(FLAGS.task_index, num_workers, device.index or 0, group=grp, src=cluster.num_ps)
            run_one = lambda name: _probe_gpu_schedule(name, mnist, device, num_workers, grp,  # noqa: E731
                                                       cluster.num_ps, rccl)
        else:
            run_one = lambda name: _probe_cpu_schedule(name, num_workers, grp)  # noqa: E731
        log = (lambda m: print(m, file=sys.stderr, flush=True)) if is_chief else None
        dp_sched, dp_probe, dp_source = choose_dp_schedule(run_one, FLAGS.task_index, num_workers, device.type,
                                                           grp, log)
        if is_chief:
            print("Worker %d: DP schedule %s (%s%s)" % (
                FLAGS.task_index, dp_sched, dp_source,
                (": " + ", ".join("%s %.4f ms/step" % kv for kv in dp_probe.items())) if dp_probe else ""))
    runner = make_runner(FLAGS.batch_size, opt, device, keep_prob=FLAGS.keep_prob, seed=FLAGS.seed,
                         rank=FLAGS.task_index, comm=None, bf16_grads=FLAGS.bf16_grads,
                         use_graph=FLAGS.use_graph and (sopt is None or not sopt.has_backup_workers or backup_ps),
                         dtype=FLAGS.dtype)
    comm = None
    transport = None
    zero = False
    if allreduce_dp and device.type == "cuda":
        from ..parallel.schedule import MNIST_SCHEDULES
        from ..parallel.transport import attach_engine

        cfg = MNIST_SCHEDULES.get(dp_sched, {"fc_sfb": 0, "zero": 0, "merge_reduce": 0})
        zero = bool(cfg["zero"]) and FLAGS.dtype == "bf16"
        transport = attach_engine(runner.eng, FLAGS.task_index, num_workers, device, group=server.worker_group,
                                  src=cluster.num_ps, mode=FLAGS.dp_transport, comm=rccl, bf16=FLAGS.bf16_grads,
                                  sfb=bool(cfg["fc_sfb"]) and FLAGS.dtype == "bf16", zero=zero)
        if zero:
            runner.eng.set_zero(True)
        runner.eng.set_sfb_merge_reduce(bool(cfg["merge_reduce"]))
        comm = transport.comm
        runner.comm = comm
        runner.transport = transport
    # PS modes overwrite the runner's step with the PS global step after every push, and the device
    # permutation is indexed by that step: each worker would see ~1/N of its epoch. Those modes keep
    # the reference's per-worker sequential next_batch (mnist_python_m.py:291) on the host instead.
    device_input = device.type == "cuda" and FLAGS.device_input and not ps_mode
    if device_input:
        runner.set_device_dataset(mnist.train.images, mnist.train.labels,
                                  seed=FLAGS.seed * 1000 + FLAGS.task_index + 31)

    def init_fn():
        flat = M.flat_from_dict(M.init_params(FLAGS.seed))
        runner.load_flat(flat, {}, 0)

    client = None
    gpu_ps = use_gpu_ps
    if not ps_mode:
        def broadcast_fn():
            if num_workers > 1:
                sync_replicas.broadcast_state(runner, 0, group=server.worker_group, group_src_rank=cluster.num_ps)
    elif gpu_ps:
        from ..parallel.gpu_ps import GpuPSClient
        from .optimizers import FlatApplier

        client = GpuPSClient(FLAGS.task_index, layout, runner.params(), runner.sync_shadow,
                             slot_names=list(FlatApplier(opt, 0).slots()))
        runner.ps_client = client  # the chief's checkpoints read the PS-resident state (params + slots)

        def broadcast_fn():
            if is_chief:
                # the ps tasks read the initial / restored values from the chief's engine (peer memory);
                # restored moments follow as host tensors, fresh ones start at zero
                slots = {("m" if k == "accum" else k): v.detach().float().cpu()
                         for k, v in runner.slot_tensors().items()} if sv.restored_from else None
                client.init(step=runner.global_step(), t=runner.global_step(), slots=slots)
            runner.set_global_step(client.pull())
    else:
        from .optimizers import FlatApplier

        client = async_ps.AsyncPSClient(FLAGS.task_index, layout, slot_names=list(FlatApplier(opt, 0).slots()))
        runner.ps_client = client  # the chief's checkpoints read the PS-resident state (params + slots)

        def broadcast_fn():
            flat = runner.params().detach().float().cpu()
            if is_chief:
                # restored moments go back to the PS (fresh init: zeros); t = global_step
                slots = {("m" if k == "accum" else k): v.detach().float().cpu()
                         for k, v in runner.slot_tensors().items()} if sv.restored_from else None
                client.init(flat, step=runner.global_step(), t=runner.global_step(), slots=slots)
            gs = client.pull(flat)
            runner.set_params(flat)
            runner.set_global_step(gs)

    logdir = FLAGS.logdir or tempfile.mkdtemp()
    sv = Supervisor(is_chief=is_chief, logdir=logdir, runner=runner, init_fn=init_fn, broadcast_fn=broadcast_fn,
                    save_model_secs=FLAGS.save_model_secs, save_summaries_secs=FLAGS.save_summaries_secs,
                    recovery_wait_secs=1)

    if is_chief:
        print("Worker %d: Initializing session..." % FLAGS.task_index)
    else:
        print("Worker %d: Waiting for session to be initialized..." % FLAGS.task_index)
    if FLAGS.existing_servers:
        server_grpc_url = "grpc://" + worker_spec[FLAGS.task_index]
        print("Using existing server at: %s" % server_grpc_url)
    sys.stdout.flush()
    sv.prepare_or_wait_for_session()
    print("Worker %d: Session initialization complete." % FLAGS.task_index)

    if FLAGS.log_device_placement:
        from ..parallel.cluster import replica_device_setter

        names = ["global_step"] + [tf for _, tf, _ in M.PARAM_SPECS]
        wdev = "/job:worker/task:%d/%s:%d" % (FLAGS.task_index, "gpu" if device.type == "cuda" else "cpu",
                                              device.index or 0)
        placed = replica_device_setter(cluster, names, wdev) if ps_mode else {n: wdev + " (replicated)" for n in names}
        if gpu_ps:  # each ps task's shard lives on its GPU (task % num_gpus), not on the reference's ps cpu
            from ..parallel.cluster import ps_task_of

            placed = {n: "/job:ps/task:%d/gpu:%d" % (ps_task_of(placed, n), ps_task_of(placed, n) % FLAGS.num_gpus)
                      for n in names}
        for n in names:
            print("%s: %s" % (n, placed[n]))
        print("compute (conv_net, loss, gradients): %s; gradient sync: %s" % (
            wdev, (("GPU ps mailbox push / peer-memory pull" if gpu_ps else "async PS push/pull") if not sync else
                   "PS accumulator (%d of %d replicas)" % (r2a, num_workers) if backup_ps else
                   (transport.kind.replace("+sfb", "") + " all-reduce"
                    + (" (fc layers: all-gathered sufficient factors)" if "+sfb" in transport.kind else ""))
                   if transport is not None else "Gloo all-reduce")))

    eval_at = sorted(int(v) for v in FLAGS.eval_at_steps.split(",") if v.strip()) if FLAGS.eval_at_steps else []
    eval_time = 0.0
    perf_rows = []

    delays = {}
    if FLAGS.straggler_delay:
        for item in FLAGS.straggler_delay.split(","):
            k, v = item.split(":")
            delays[int(k)] = float(v)
    stepper = None
    if sync and not backup_ps:
        stepper = sync_replicas.SyncReplicasStepper(runner, FLAGS.task_index, num_workers, sopt.replicas_to_aggregate,
                                                    group=server.worker_group, straggler_delay_s=delays,
                                                    splits=[M.BUCKET_SPLIT] if dp_sched == "buckets" else None)
    metrics = MetricsLogger(FLAGS.metrics_file if is_chief else "")
    if dp_sched is not None:
        metrics.log(event="dp_schedule", chosen=dp_sched, source=dp_source,
                    candidates_ms_per_step=({k: round(v, 5) for k, v in dp_probe.items()} if dp_probe else None))
    phase_timing = FLAGS.phase_timing or (is_chief and bool(FLAGS.metrics_file))
    if phase_timing:
        runner.set_phase_timing(True)
    timer = StepTimer(pid=FLAGS.task_index, enabled=bool(FLAGS.trace_file))
    restart_attempt = int(os.environ.get("TFD_RESTART_COUNT", "0"))

    from ..utils.tracing import Watchdog, trace_range

    watchdog = Watchdog(FLAGS.step_timeout_secs, on_timeout=(comm.abort if comm is not None else None))
    time_begin = time.time()
    print("Training begins @ %f" % time_begin)
    local_step = 0
    step = runner.global_step()
    grad_cpu = None
    while True:
        if step >= FLAGS.train_steps:
            break
        with timer.phase("input"):
            if device_input:
                batch_xs = batch_ys = None  # the engine gathers the batch on the device
            else:
                batch_xs, batch_ys = mnist.train.next_batch(FLAGS.batch_size)
        t0 = time.time()
        with timer.phase("step"), trace_range("train_step"):
            if not ps_mode:
                stepper.step(batch_xs, batch_ys)
                step = runner.global_step()
            elif gpu_ps:
                g, _ = runner.compute_grads(batch_xs, batch_ys, with_loss=False)
                if FLAGS.task_index in delays:
                    time.sleep(delays[FLAGS.task_index])  # test hook: a straggling worker
                # the gradient goes GPU -> the ps tasks' GPU mailboxes, the fresh values come back into
                # the engine's parameters; only the 32-byte control messages touch the host
                step = client.push_pull(g, local_step=step)
                runner.set_global_step(step)
            else:
                g, _ = runner.compute_grads(batch_xs, batch_ys)
                if grad_cpu is None:
                    grad_cpu = torch.zeros(M.TOTAL)
                grad_cpu.copy_(g.detach().float().cpu())
                if FLAGS.task_index in delays:
                    time.sleep(delays[FLAGS.task_index])  # test hook: a straggling worker
                flat = runner.params().detach().float().cpu()
                # sync: the gradient is tagged with the global step it was computed at (stale ones
                # are dropped by the PS accumulator); async: applied as it comes
                step = client.push_pull(flat, grad_cpu, local_step=step)
                runner.set_params(flat)
                runner.set_global_step(step)
        local_step += 1
        watchdog.kick()
        now = time.time()
        if not FLAGS.quiet:
            print("%f: Worker %d: training step %d done (global step: %d)" % (now, FLAGS.task_index, local_step, step))
            if backup_ps and client.last_dropped:
                print("Worker %d: stale gradient dropped (a backup replica finished this step first)" % FLAGS.task_index)
        if metrics.path:
            rec = dict(step=local_step, global_step=step, step_ms=1e3 * (now - t0), loss=runner.last_loss(),
                       images_per_sec=FLAGS.batch_size * (num_workers if sync else 1) / max(now - t0, 1e-9))
            if phase_timing:
                ph = runner.phase_times()
                rec.update(ph)
                timer.add_gpu_phases(now, ph)
            rec.setdefault("allreduce_ms", 0.0 if (not sync or num_workers == 1) else None)
            metrics.log(**rec)
        if FLAGS.check_consistency_every and sync and local_step % FLAGS.check_consistency_every == 0:
            if zero:
                runner.sync_state()  # every worker: the fc1 shards -> whole fp32 state
            _check_consistency(runner, server, num_workers)
        if zero:
            # the fp32 fc1 master and its Adam slots are sharded over the workers: the chief's timed
            # checkpoint needs a gather that every worker joins, at agreed global steps
            save_now = False
            if step % max(1, FLAGS.zero_sync_every) == 0:
                due = torch.tensor([1 if sv.save_due() else 0], dtype=torch.int64)
                import torch.distributed as dist

                dist.all_reduce(due, op=dist.ReduceOp.MAX, group=server.worker_group)
                save_now = bool(due.item())
                if save_now:
                    runner.sync_state()
            sv.on_step(step, allow_save=save_now)
        else:
            sv.on_step(step)
        while is_chief and eval_at and step >= eval_at[0]:
            te = time.time()
            accs = []
            for _ in range(FLAGS.eval_batches):
                vx, vy = mnist.validation.next_batch(FLAGS.eval_batch_size)
                accs.append(runner.evaluate(vx, vy)[1] / float(len(vx)))
            acc = 100.0 * sum(accs) / len(accs)
            eval_time += time.time() - te
            row = dict(steps=eval_at.pop(0), time=time.time() - time_begin - eval_time, accuracy=round(acc, 2),
                       lr=FLAGS.learning_rate)
            perf_rows.append(row)
            print("Performance row: %d %.1f %.2f %g" % (row["steps"], row["time"], row["accuracy"], row["lr"]))
            metrics.log(event="performance", **row)
        if (FLAGS.fault_inject_step >= 0 and FLAGS.task_index == FLAGS.fault_inject_task and restart_attempt == 0
                and step >= FLAGS.fault_inject_step):
            print("Worker %d: fault injection at global step %d" % (FLAGS.task_index, step), flush=True)
            os._exit(17)

    watchdog.stop()
    if zero:
        runner.sync_state()  # whole replicas again: final checksum, eval and the chief's last checkpoint
    if FLAGS.check_consistency_every and sync:
        pp = runner.params().detach().double()
        print("Worker %d: parameter checksum %.17g %.17g" % (FLAGS.task_index, float(pp.sum().item()),
                                                             float((pp * pp).sum().item())))
    if transport is not None:
        transport.check("training")  # a timed-out IPC barrier must not pass as a finished run
    time_end = time.time()
    print("Training ends @ %f" % time_end)
    training_time = time_end - time_begin - eval_time
    print("Training elapsed time: %f s" % training_time)

    accuracy_arr = []
    nt = FLAGS.eval_batches
    for counter in range(1, nt + 1):
        val_x, val_y = mnist.validation.next_batch(FLAGS.eval_batch_size)
        _, correct = runner.evaluate(val_x, val_y)
        val_xent = correct / float(len(val_x))
        print("After %d training step(s)", FLAGS.train_steps)  # verbatim reference line (quirk Q3)
        print("Accuracy : %f" % val_xent)
        accuracy_arr.append(val_xent)
    mean_accuracy = sum(accuracy_arr) / len(accuracy_arr) if accuracy_arr else float("nan")
    print("Mean Accuracy : %f" % mean_accuracy)
    sys.stdout.flush()

    metrics.log(event="final", global_step=step, training_time_s=training_time, mean_accuracy=mean_accuracy)
    if perf_rows:
        from ..utils.metrics import performance_table

        print(performance_table(perf_rows), end="")
    metrics.close()
    if FLAGS.trace_file:
        timer.write_chrome_trace(FLAGS.trace_file.replace("{task}", str(FLAGS.task_index)))
    sv.stop(save=True)
    if client is not None:
        client.stop()
    if transport is not None:
        transport.close()
    server.mark_done()
    if sync and num_workers > 1:
        import torch.distributed as dist

        dist.barrier(group=server.worker_group)
    server.shutdown()
    return 0


def _check_consistency(runner, server, num_workers):
    """Race/desync detector: max |checksum_i - checksum_0| across workers."""
    import torch.distributed as dist

    p = runner.params().detach().double()
    cs = torch.tensor([float(p.sum().item()), float((p * p).sum().item())], dtype=torch.float64)
    mx, mn = cs.clone(), cs.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=server.worker_group)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=server.worker_group)
    if not torch.equal(mx, mn):
        raise RuntimeError(f"worker parameter desync detected: checksum range {mn.tolist()} .. {mx.tolist()}")


def run_script(task_index_default: int, job_name_default: str, argv=None) -> int:
    define_flags(task_index_default, job_name_default)
    argv = list(sys.argv if argv is None else argv)
    if "--help" in argv or "-h" in argv:
        print(f"usage: {argv[0]} [flags]\n{FLAGS.help_text()}")
        return 0
    FLAGS.parse(argv)
    return main(argv) or 0
