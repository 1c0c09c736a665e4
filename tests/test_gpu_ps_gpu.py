"""GPU-resident parameter server (parallel/gpu_ps.py, csrc/runtime/gpu_ps.cpp): the reference's async
and backup-worker modes (/root/reference/mnist_python_m.py:62-75, 210-222, 247-253) with the
variables, Adam slots and accumulator on the ps task's GPU and every gradient / parameter byte
moving device-to-device (IPC peer memory; here the reference quick-start topology: 1 ps + 2 workers
sharing one GPU)."""
import json
import os
import re

import numpy as np
import pytest
import torch

from dist_util import run_ranks
from tensorflow_distributed_amd.models import mnist_cnn as M

pytestmark = pytest.mark.gpu


def _padded_zero(flat):
    n = M.OFFSETS["out_b"] + 10  # end of the last variable; [n, TOTAL) is alignment padding
    flat[n:] = 0
    return flat


def _shard_worker(rank, world, kind):
    """rank 0 = ps (one shard = every variable), ranks 1..2 = workers with fixed gradients."""
    from tensorflow_distributed_amd import _native
    from tensorflow_distributed_amd.parallel.async_ps import mnist_layout
    from tensorflow_distributed_amd.parallel.gpu_ps import GpuParameterServerService, GpuPSClient
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer, MomentumOptimizer

    _native.require()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    opt = AdamOptimizer(0.01) if kind == "adam" else MomentumOptimizer(0.01, 0.9)
    layout = mnist_layout(1)
    sync = True
    if rank == 0:
        svc = GpuParameterServerService(0, 1, 2, layout, opt, dev, sync=sync, replicas_to_aggregate=2)
        svc.serve()
        return {"updates": svc.updates, "t": svc.t, "dropped": svc.dropped}
    w = rank - 1
    params = torch.zeros(M.TOTAL, device=dev)
    refreshed = []
    client = GpuPSClient(w, layout, params, lambda: refreshed.append(1), slot_names=["m", "v"] if kind == "adam" else ["m"])
    g0 = torch.Generator().manual_seed(11)
    init = _padded_zero(torch.randn(M.TOTAL, generator=g0) * 0.05)  # the flat buffer's tail padding is no variable
    if w == 0:
        params.copy_(init.to(dev))
        client.init(step=0, t=0)
    client.pull()
    assert torch.equal(params.cpu(), init), "pull did not deliver the chief's values"
    steps = []
    for s in range(3):
        g = torch.Generator().manual_seed(100 + 10 * s + w)
        grad = _padded_zero(torch.randn(M.TOTAL, generator=g) * 1e-2).to(dev)
        steps.append(client.push_pull(grad, local_step=s))
    torch.cuda.synchronize()
    out = params.cpu().clone()
    state = None
    if w == 0:
        flat = torch.zeros(M.TOTAL)
        slots, t, step = client.pull_state(flat)
        state = {"flat": flat, "t": t, "step": step, **{k: v for k, v in slots.items()}}
    client.stop()
    return {"params": out, "steps": steps, "refreshed": len(refreshed), "state": state}


@pytest.mark.parametrize("kind", ["adam", "momentum"])
def test_gpu_ps_sync_accumulator_matches_host_optimizer(cuda, kind):
    """1 ps + 2 workers, replicas_to_aggregate = 2: three global steps of (g0 + g1) / 2 applied on
    the ps GPU equal the host FlatApplier on the same gradients; both workers receive the fresh
    values straight into their parameter buffers, and the checkpoint read returns them with the
    optimizer slots."""
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer, FlatApplier, MomentumOptimizer

    res = run_ranks(_shard_worker, 3, kind, timeout=300)
    opt = AdamOptimizer(0.01) if kind == "adam" else MomentumOptimizer(0.01, 0.9)
    ref = _padded_zero(torch.randn(M.TOTAL, generator=torch.Generator().manual_seed(11)) * 0.05)
    ap = FlatApplier(opt, M.TOTAL)
    for s in range(3):
        gs = [_padded_zero(torch.randn(M.TOTAL, generator=torch.Generator().manual_seed(100 + 10 * s + w)) * 1e-2)
              for w in range(2)]
        ap.apply(ref, gs[0] + gs[1], 0.5)
    assert res[0]["updates"] == 3 and res[0]["t"] == 3 and res[0]["dropped"] == 0
    for w in (1, 2):
        assert res[w]["steps"] == [1, 2, 3]
        assert res[w]["refreshed"] == 4  # the pull + three push_pulls
        torch.testing.assert_close(res[w]["params"], ref, rtol=1e-5, atol=1e-6)
    assert torch.equal(res[1]["params"], res[2]["params"])
    st = res[1]["state"]
    assert st["t"] == 3 and st["step"] == 3 and torch.equal(st["flat"], res[1]["params"])
    torch.testing.assert_close(st["m"], ap.m, rtol=1e-5, atol=1e-7)
    if kind == "adam":
        torch.testing.assert_close(st["v"], ap.v, rtol=1e-5, atol=1e-10)


def _run_cluster(tmp_path, name, extra, workers=2, steps=30):
    from tensorflow_distributed_amd import launch

    mf = os.path.join(tmp_path, f"{name}.jsonl")
    args = ["--num_gpus=1", f"--train_steps={steps}", f"--logdir={tmp_path}/{name}", "--synthetic_data",
            "--eval_batches=1", "--data_dir=/nonexistent", f"--metrics_file={mf}"] + extra
    r = launch.launch(1, workers, args, echo=False, timeout_s=300)
    assert r["ok"], r["outputs"]
    recs = [json.loads(line) for line in open(mf) if line.strip()]
    ms = sorted(x["step_ms"] for x in recs if "step_ms" in x)
    return r, ms


def test_gpu_ps_async_and_backup_workers_and_speedup(cuda, tmp_path):
    """The reference quick start (1 ps + 2 workers on one GPU) in async mode with the ps on the GPU
    vs the reference's CPU ps: both train to the last global step; the GPU ps worker step is >= 5x
    faster (median over the run). Then backup workers (1 ps + 3 workers, replicas_to_aggregate 2)
    with the GPU ps."""
    rg, ms_gpu = _run_cluster(tmp_path, "gpu", ["--sync_replicas=False", "--log_device_placement"])
    rc, ms_cpu = _run_cluster(tmp_path, "cpu", ["--sync_replicas=False", "--ps_on_gpu=False"])
    outg = "".join(v for k, v in rg["outputs"].items() if k.startswith("worker:0#"))
    assert "/job:ps/task:0/gpu:0" in outg and "GPU ps mailbox push" in outg, outg[-2000:]
    steps = [int(x) for x in re.findall(r"global step: (\d+)\)", outg)]
    assert steps and max(steps) >= 29
    med_g, med_c = ms_gpu[len(ms_gpu) // 2], ms_cpu[len(ms_cpu) // 2]
    print(f"async 1 ps + 2 workers, worker step median: GPU ps {med_g:.2f} ms, CPU ps {med_c:.2f} ms "
          f"({med_c / med_g:.1f}x)")
    assert med_c / med_g >= 5.0, (med_g, med_c)
    rb, _ = _run_cluster(tmp_path, "backup", ["--replicas_to_aggregate=2"], workers=3, steps=12)
    outb = "".join(rb["outputs"].values())
    assert "synchronous updates" in outb


@pytest.mark.parametrize("opt", ["adam", "momentum"])
def test_gpu_ps_restore_matches_host_ps_restore(cuda, tmp_path, opt):
    """Checkpoint under the GPU parameter server, then restore it into fresh clusters: one with the
    GPU ps (OP_INIT with host slot tensors, GpuPsShard.load_state, the pull_state checkpoint read;
    momentum's 'accum' slot renamed 'm' on the way in) and one with the host ps. Both restored
    clusters stop at once (train_steps below the restored step) and write their final checkpoint,
    which must hold exactly the saved params, optimizer slots and global step."""
    import shutil

    from tensorflow_distributed_amd.training import checkpoint as C

    base = ["--sync_replicas=False", f"--optimizer={opt}"]
    _run_cluster(tmp_path, "saved", base, steps=12)
    saved_dir = os.path.join(tmp_path, "saved")
    def latest(d):
        path = C.read_checkpoint_state(d)["model_checkpoint_path"]
        return path if os.path.isabs(path) else os.path.join(d, path)

    saved = C.load_bundle(latest(saved_dir))
    gs = int(np.asarray(saved["global_step"]).item())
    assert gs >= 12
    outs = {}
    for name, extra in (("gpu", []), ("host", ["--ps_on_gpu=False"])):
        d = os.path.join(tmp_path, name)
        shutil.copytree(saved_dir, d)
        _run_cluster(tmp_path, name, base + extra, steps=1)
        path = latest(d)
        assert os.path.dirname(os.path.abspath(path)) == os.path.abspath(d), path  # its own final save
        outs[name] = C.load_bundle(path)
    for name, got in outs.items():
        assert sorted(got) == sorted(saved), (name, sorted(got), sorted(saved))
        for k, v in saved.items():
            assert np.array_equal(np.asarray(got[k]), np.asarray(v)), (name, k)
    slot_keys = [k for k in saved if "/" in k]
    assert slot_keys, sorted(saved)  # the optimizer slots are in the checkpoint and were compared
