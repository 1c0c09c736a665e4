"""Convnet-at-scale benchmark for BASELINE.json configs 4-5: synthetic 224x224x3 ResNet-18 /
ResNet-50 (v1.5, bf16, NHWC) data-parallel training, images/sec (whole node).

One process per GPU (torchrun env, or self-launched: ``--gpus N`` without a launcher environment
spawns the N ranks from a GPU-clean parent, see parallel/spawn.py), native HIP conv/BN/pool kernels, bucketed RCCL gradient
all-reduce overlapped with the backward, fused flat SGD-momentum, the whole step captured in a
hipGraph and replayed. Synthetic data: one fixed device-resident random batch per rank.

With N > 1 the ranks first probe every gradient bucket size of ``--bucket_candidates`` (SURVEY.md
§5.8 item 5: 2/4/8/16/25 MB), untimed, each with its own captured graph, and time the fastest
(parallel/schedule.py); ``--bucket_mb X`` skips the probes. The job exits non-zero if the
replicas' weights differ after the timed steps.

    python bench_resnet.py [--depth 50] [--batch_size 128] [--steps 20] [--warmup 5] [--bucket_mb auto]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--batch_size", type=int, default=128, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bucket_mb", default="auto", help="gradient bucket size in MB (N > 1), or auto = probe "
                    "--bucket_candidates at this N and time the fastest")
    ap.add_argument("--bucket_candidates", default="2,4,8,16,25")
    ap.add_argument("--probe_steps", type=int, default=10, help="timed steps per bucket-size probe")
    ap.add_argument("--probe_warmup", type=int, default=3)
    ap.add_argument("--small_ipc_mb", type=float, default=1.0, help="gradient buckets of at most this many MB "
                    "(bf16 wire) take the IPC one-shot all-reduce beside RCCL (N > 1; 0: every bucket on RCCL)")
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--bn_stats", type=int, default=1, help="1: batch-norm statistics summed in the conv "
                    "forward epilogue (no separate statistics pass over the conv output)")
    ap.add_argument("--relu_bits", type=int, default=1, help="1: residual BNs keep their relu mask as bits for "
                    "the backward instead of re-reading the block output")
    ap.add_argument("--mask_from_y", type=int, default=1, help="1: residual-free BN backward recomputes its relu "
                    "mask from the conv output instead of reading the BN output")
    ap.add_argument("--fuse_joins", type=int, default=1, help="1: residual-join gradient sums in the dgrad "
                    "epilogue (0: autograd adds; measured faster, see resnet.GradJoin)")
    ap.add_argument("--bn_bwd_stats", type=int, default=1, help="1: batch-norm backward statistics summed in the "
                    "epilogue of the dgrad that produces the BN's gradient (no separate partial pass)")
    ap.add_argument("--masked_join", type=int, default=1, help="1: identity-shortcut gradients reach the joining "
                    "conv's dgrad epilogue as (dout, relu bits), the residual BN backward writes no dres tensor")
    ap.add_argument("--fuse_stem_pool", type=int, default=1, help="1: the stem's bn + relu + max pool in one pass "
                    "(the BN output is never written)")
    ap.add_argument("--stem_w2", type=int, default=1, help="1: the stem conv on width-paired input pixels "
                    "(7x4x8 instead of 7x7x8 MACs per output, models/resnet.py _StemW2); 0: channel-padded input")
    ap.add_argument("--bn_slots", type=int, default=-1, help="BN statistics partials: S > 0 fp32 atomics into S "
                    "zeroed slots, finalized inside the apply passes (no bn_final launches); 0 per-block rows + "
                    "bn_final (fixed order); -1 the library default")
    ap.add_argument("--deterministic", action="store_true", help="BN statistics in row mode (= --bn_slots 0): every "
                    "sum of the step in a fixed order, so a run repeats bit for bit (slot mode's fp32 atomics vary the "
                    "summation order run to run; measured 13.57 vs 13.22 ms/step for ResNet-50 b128, "
                    "profiles/resnet50_bn_slots_ab_r4.log)")
    ap.add_argument("--conv_halo", type=int, default=-1, help="3x3 stride-1 convs on LDS halo tiles (csrc/conv_halo.h): "
                    "0 off (im2col gather), 1 where measured faster (the library default), 2 every eligible shape; "
                    "-1 the library default")
    ap.add_argument("--fold_bn", type=int, default=0, help="1: single-consumer relu batch norms applied inside the "
                    "consuming conv's operand loader (no bn_apply pass; 0: the separate pass; 2: 1x1 consumers only)")
    ap.add_argument("--lr", type=float, default=0.1)
    argv = list(sys.argv[1:] if argv is None else argv)
    a = ap.parse_args(argv)
    from tensorflow_distributed_amd.parallel import spawn

    if spawn.needs_self_launch(a.gpus):
        return spawn.self_launch(os.path.abspath(__file__), argv, a.gpus)

    import torch

    from tensorflow_distributed_amd import _native
    from tensorflow_distributed_amd.models.resnet import ResNet
    from tensorflow_distributed_amd.parallel import dist as D

    from tensorflow_distributed_amd.utils.tracing import PhaseWatchdog

    live = {"ipc": None}  # the IPC communicator in use, for the watchdog's error-word report
    wd = PhaseWatchdog(int(os.environ.get("RANK", "0")), tag="bench_resnet.py",
                       err_fn=lambda: live["ipc"].error() if live["ipc"] is not None else 0)
    wd.phase("setup: native library, process group, RCCL/IPC bootstrap, model", 600)
    _native.require()
    ctx = D.init_from_env(use_gpu=True)
    spawn.check_world(a.gpus, ctx.world)
    dev = ctx.device
    if a.deterministic:
        if a.bn_slots > 0:
            raise SystemExit("error: --deterministic is row mode (--bn_slots 0)")
        a.bn_slots = 0
    if a.bn_slots >= 0:
        torch.ops.tfd.set_bn_part_slots(a.bn_slots)
    if a.conv_halo >= 0:
        torch.ops.tfd.conv_halo_mode(a.conv_halo)
    m = ResNet(a.depth, num_classes=1000, device=dev, seed=0, fuse_joins=bool(a.fuse_joins),
               bn_stats=bool(a.bn_stats), bn_bwd_stats=bool(a.bn_bwd_stats), fold_bn=a.fold_bn)
    m.mask_from_y = bool(a.mask_from_y)
    m.relu_bits = bool(a.relu_bits)
    m.masked_join = bool(a.masked_join)
    m.fuse_stem_pool = bool(a.fuse_stem_pool)
    m.stem_w2 = bool(a.stem_w2)
    comm, transport, small = None, "none", None
    if ctx.world > 1:
        if ctx.comm is not None:  # one rank per GPU: RCCL over xGMI
            comm, transport = ctx.comm, "rccl"
            comm.broadcast(m.fp.master, 0)
            from tensorflow_distributed_amd.parallel.transport import small_bucket_ipc

            small = small_bucket_ipc(ctx.rank, ctx.world, dev, comm, int(a.small_ipc_mb * (1 << 20)))
            if small is not None:
                transport = "rccl+ipc(small buckets)"
                live["ipc"] = small.ipc
        elif ctx.shared_device:  # ranks share a GPU (RCCL refuses that): the IPC transport
            from tensorflow_distributed_amd.parallel.ipc import IpcCollectives, make_ipc_comm

            comm, transport = IpcCollectives(make_ipc_comm(ctx.rank, ctx.world, dev.index, m.fp.total)), "ipc"
            live["ipc"] = comm.ipc
            host = m.fp.master.detach().cpu()
            ctx.broadcast_tensor_cpu(host, 0)  # chief init -> every rank over Gloo
            m.fp.master.copy_(host.to(dev))
        else:
            raise RuntimeError(f"world {ctx.world} but no gradient transport: refusing to report non-DP throughput")
        m.fp.shadow.copy_(m.fp.master)
    g = torch.Generator(device=dev).manual_seed(100 + ctx.rank)
    x = torch.randn(a.batch_size, a.image, a.image, 3, device=dev, generator=g)
    y = torch.randint(0, 1000, (a.batch_size,), device=dev, generator=g, dtype=torch.int32)
    s = torch.cuda.Stream(dev)
    pool = torch.cuda.graph_pool_handle()  # every captured step (probes + the timed one) shares one pool

    def agree(err, what):
        """Every rank learns whether a local step failed on ANY rank before the next collective, so no
        rank enters the step's collectives (RCCL / IPC / the probes' barriers) alone."""
        if ctx.max_scalar(1.0 if err is not None else 0.0) > 0:
            raise RuntimeError(f"{what} failed on at least one rank (here: {err!r})")

    def configure(mb):
        """Reducer with ``mb``-MB buckets, two eager steps, the step captured; returns run(k)."""
        err = None
        try:
            if comm is not None:
                m.set_comm(comm, mb, small=small, small_mb=a.small_ipc_mb)
        except Exception as e:  # noqa: BLE001 - agreed below
            err = e
        agree(err, f"bucket reducer setup ({mb} MB)")
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(2):
                m.train_step(x, y, lr=a.lr)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        if a.eager:
            def run(k):
                for _ in range(k):
                    out = m.train_step(x, y, lr=a.lr)
                return out
            return run, None
        graph, out_static, err = torch.cuda.CUDAGraph(), None, None
        try:
            with torch.cuda.graph(graph, pool=pool):
                out_static = m.train_step(x, y, lr=a.lr)
        except Exception as e:  # noqa: BLE001 - a capture fails locally (nothing is launched): agreed below
            err = e
        agree(err, f"step capture ({mb} MB buckets)")

        def run(k):
            for _ in range(k):
                graph.replay()
            return out_static
        return run, graph

    probe_ms, source = None, "single"
    if comm is None:
        bucket_mb = None
    elif a.bucket_mb != "auto":
        bucket_mb, source = float(a.bucket_mb), "flag"
    else:
        from tensorflow_distributed_amd.parallel import schedule as SCH

        cands = [float(c) for c in a.bucket_candidates.split(",") if c.strip()]
        # every probe trains: start the timed job from the same weights afterwards (every rank alike)
        snap = [t.clone() for t in (m.fp.master, m.fp.momentum, m.fp.shadow)]

        def one(name):
            wd.phase(f"bucket probe {name} MB (setup, capture, {a.probe_warmup} + {a.probe_steps} steps)",
                     240 + 2.0 * (a.probe_warmup + a.probe_steps))
            run_p, graph_p = configure(float(name))
            run_p(a.probe_warmup)
            torch.cuda.synchronize(dev)
            ctx.barrier()
            t0 = time.perf_counter()
            run_p(a.probe_steps)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            del run_p, graph_p
            return dt * 1e3 / max(1, a.probe_steps)

        log = (lambda msg: print(msg, file=sys.stderr, flush=True)) if ctx.rank == 0 else None
        probe_ms = SCH.probe([f"{c:g}" for c in cands], one, ctx.max_scalar, log)
        bucket_mb, source = float(SCH.pick(probe_ms)), "probe"
        for dst, src in zip((m.fp.master, m.fp.momentum, m.fp.shadow), snap):
            dst.copy_(src)
        del snap
        torch.cuda.synchronize(dev)
    wd.phase(f"job setup + warm-up ({bucket_mb} MB buckets, {a.warmup} steps)", 240 + 2.0 * a.warmup)
    run, graph = configure(bucket_mb)
    run(a.warmup)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    wd.phase(f"timed region ({a.steps} steps)", 120 + 2.0 * a.steps)
    t0 = time.perf_counter()
    loss = run(a.steps)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    dt = ctx.max_scalar(time.perf_counter() - t0)
    wd.phase("report: replica digests, teardown", 300)
    img_s = ctx.world * a.batch_size * a.steps / dt
    topo = _topology(ctx, dev, comm, m)
    if ctx.rank == 0:
        print(f"# resnet{a.depth} world={ctx.world} B/gpu={a.batch_size} loss={float(loss):.3f} "
              f"{dt * 1e3 / a.steps:.2f} ms/step", file=sys.stderr)
        print(json.dumps({
            "metric": f"images/sec (whole node) synthetic-ImageNet ResNet-{a.depth} DP training",
            "value": round(img_s, 1), "unit": "images/s", "n_gpus": ctx.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt * 1e3 / a.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": f"synthetic (random {a.image}x{a.image}x3 fp32 images, random labels; He init)",
            **topo,
            "config": {"model": f"resnet{a.depth} v1.5 NHWC", "global_batch": ctx.world * a.batch_size,
                       "per_gpu_batch": a.batch_size, "seq_len": None, "parallelism": f"dp{ctx.world}",
                       "dp_transport": transport,
                       "bucket_mb": bucket_mb, "small_bucket_mb": a.small_ipc_mb if small is not None else None,
                       "small_buckets": m.reducer.small_buckets if small is not None else 0,
                       "bucket_schedule": {"source": source, "candidates_ms_per_step": (
                           {k: round(v, 4) for k, v in probe_ms.items()} if probe_ms else None)},
                       "optimizer": "sgd-momentum 0.9 wd 1e-4",
                       "hipgraph": not a.eager, "fuse_joins": bool(a.fuse_joins), "bn_stats": bool(a.bn_stats),
                       "mask_from_y": bool(a.mask_from_y), "relu_bits": bool(a.relu_bits),
                       "bn_bwd_stats": bool(a.bn_bwd_stats), "fold_bn": a.fold_bn, "masked_join": bool(a.masked_join),
                       "fuse_stem_pool": bool(a.fuse_stem_pool),
                       "stem_w2": bool(a.stem_w2),
                       "bn_slots": int(torch.ops.tfd.bn_part_slots()),
                       "conv_halo": int(torch.ops.tfd.conv_halo_mode(-1)),
                       "bn_stats_mode": ("row: fixed summation order, bit-reproducible"
                                         if int(torch.ops.tfd.bn_part_slots()) == 0 else
                                         "slots: fp32 atomics, summation order varies run to run")}}), flush=True)
    for c in (comm if transport == "ipc" else None, small):
        if c is not None:
            if c.ipc.error():
                raise RuntimeError("IPC collective barrier timed out: replicas may have diverged")
            c.ipc.close()
    live["ipc"] = None
    wd.stop()
    ctx.shutdown()
    if not topo["replicas_identical"]:
        print("error: DP replicas diverged (parameter digests differ across ranks)", file=sys.stderr)
        return 3
    return 0


def _topology(ctx, dev, comm, m):
    """comm world as the transport reports it, every rank's device, and whether the replicas'
    fp32 master weights are bit-identical after the timed steps."""
    import hashlib

    import torch

    from tensorflow_distributed_amd.parallel.transport import device_label

    torch.cuda.synchronize(dev)
    mine = {"device": device_label(dev),
            "sha1": hashlib.sha1(m.fp.master.detach().cpu().numpy().tobytes()).hexdigest()[:16]}
    rows = [mine]
    if ctx.world > 1:
        import torch.distributed as dist

        rows = [None] * ctx.world
        dist.all_gather_object(rows, mine)
    return {"comm_world": int(comm.world()) if comm is not None else 1, "devices": [r["device"] for r in rows],
            "replicas_identical": len({r["sha1"] for r in rows}) == 1, "params_sha1": rows[0]["sha1"]}


if __name__ == "__main__":
    sys.exit(main())
