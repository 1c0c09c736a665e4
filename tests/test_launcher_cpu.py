"""End-to-end launcher / script smoke tests on CPU: the three reference
roles on localhost, sync and async modes, fault injection + restart + resume, mnist_single.py,
--download_only and --existing_servers."""
import os
import subprocess
import sys

import pytest

from tensorflow_distributed_amd import launch
from tensorflow_distributed_amd.training.checkpoint import latest_checkpoint

pytestmark = pytest.mark.slow
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--synthetic_data", "--eval_batches=1", "--data_dir=/nonexistent"]


def _out(r, name):
    return "".join(v for k, v in r["outputs"].items() if k.startswith(name + "#"))


def test_sync_cluster_reference_lines(tmp_path):
    mf = tmp_path / "m.jsonl"
    r = launch.launch(1, 2, ["--train_steps=3", f"--logdir={tmp_path}", f"--metrics_file={mf}",
                             f"--trace_file={tmp_path}/trace{{task}}.json"] + COMMON, echo=False, timeout_s=300)
    assert r["ok"], r["outputs"]
    w0, w1, ps = _out(r, "worker:0"), _out(r, "worker:1"), _out(r, "ps:0")
    assert "job name = ps" in ps and "task index = 0" in ps
    assert "Worker 0: Initializing session..." in w0 and "Worker 1: Waiting for session to be initialized..." in w1
    for w, i in ((w0, 0), (w1, 1)):
        assert f"Worker {i}: Session initialization complete." in w
        assert "Training begins @" in w and "Training elapsed time:" in w and "Mean Accuracy :" in w
        assert f"Worker {i}: training step 3 done (global step: 3)" in w
    # default --dp_schedule=fixed: one schedule per device/dtype, no probes (reproducible runs)
    assert "Worker 0: DP schedule flat (fixed)" in w0, w0
    assert latest_checkpoint(str(tmp_path)).endswith("model.ckpt-3")
    assert any(f.startswith("events.out.tfevents.") for f in os.listdir(tmp_path))
    import json
    recs = [json.loads(ln) for ln in open(mf)]
    steps = [rec for rec in recs if "step" in rec and "event" not in rec]
    assert len(steps) == 3 and all(rec["loss"] > 0 and rec["allreduce_ms"] > 0 for rec in steps), steps
    assert os.path.exists(tmp_path / "trace0.json")


def test_sync_cluster_probes_dp_schedule(tmp_path):
    """--dp_schedule=auto at 2 workers over Gloo: both workers time every CPU candidate
    before training, the chief prints and logs the choice (the fastest by max over workers), and the
    run trains with it; a pinned schedule skips the probes."""
    import json

    mf = tmp_path / "m.jsonl"
    r = launch.launch(1, 2, ["--train_steps=3", f"--logdir={tmp_path}/a", f"--metrics_file={mf}",
                             "--dp_schedule=auto", "--dp_probe_steps=2"] + COMMON, echo=False, timeout_s=300)
    assert r["ok"], r["outputs"]
    w0 = _out(r, "worker:0")
    rec = [json.loads(ln) for ln in open(mf) if '"dp_schedule"' in ln]
    assert len(rec) == 1 and rec[0]["source"] == "probe", rec
    c = rec[0]["candidates_ms_per_step"]
    assert set(c) == {"flat", "buckets"} and all(v > 0 for v in c.values()), c
    assert rec[0]["chosen"] == min(c, key=c.get)
    assert f"Worker 0: DP schedule {rec[0]['chosen']} (probe: " in w0, w0
    assert "training step 3 done (global step: 3)" in w0
    r = launch.launch(1, 2, ["--train_steps=2", f"--logdir={tmp_path}/b", "--dp_schedule=buckets"] + COMMON,
                      echo=False, timeout_s=300)
    assert r["ok"], r["outputs"]
    assert "Worker 0: DP schedule buckets (flag)" in _out(r, "worker:0")


def test_async_cluster_two_ps(tmp_path):
    r = launch.launch(2, 2, ["--train_steps=4", "--sync_replicas=False", f"--logdir={tmp_path}"] + COMMON,
                      echo=False, timeout_s=300)
    assert r["ok"], r["outputs"]
    out = _out(r, "worker:0") + _out(r, "worker:1")
    assert out.count("training step") >= 4  # global step advances once per worker step


def test_fault_injection_restart_resumes(tmp_path):
    args = ["--train_steps=6", f"--logdir={tmp_path}", "--save_model_secs=0.3", "--fault_inject_step=4",
            "--fault_inject_task=1"] + COMMON
    r = launch.launch(1, 2, args, max_restarts=1, echo=False, timeout_s=300)
    assert r["ok"] and r["attempts"] == 2, r["outputs"]
    first = r["outputs"]["worker:1#0"]
    assert "fault injection at global step 4" in first
    second = r["outputs"]["worker:0#1"]
    assert "Restored from checkpoint" in second
    assert latest_checkpoint(str(tmp_path)).endswith("model.ckpt-6")


def test_fault_without_restart_fails(tmp_path):
    args = ["--train_steps=5", f"--logdir={tmp_path}", "--fault_inject_step=2", "--fault_inject_task=0"] + COMMON
    r = launch.launch(1, 2, args, max_restarts=0, echo=False, timeout_s=300)
    assert not r["ok"] and r["failed"] == "worker:0"


def test_mnist_single_cpu(tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "mnist_single.py"), "--cpu", "--training_iters=1400",
                        "--eval_batches=5", f"--data_dir={tmp_path}/none"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert "Iter 1280, Minibatch Loss= " in p.stdout and "Optimization Finished!" in p.stdout
    assert "Mean Accuracy :" in p.stdout and "seconds Time for Inference ---" in p.stdout


def test_download_only(tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "mnist_python_w1.py"), "--download_only",
                        f"--data_dir={tmp_path}"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert sorted(os.listdir(tmp_path)) == sorted(f + ".gz" for f in (
        "train-images-idx3-ubyte", "train-labels-idx1-ubyte", "t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"))


def test_existing_servers_mode(tmp_path):
    port = launch.free_port()
    addr = f"127.0.0.1:{port}"
    srv = subprocess.Popen([sys.executable, "-m", "tensorflow_distributed_amd.server", "--address", addr,
                            "--num_workers", "1"], cwd=ROOT, stdout=subprocess.PIPE, text=True)
    try:
        base = [sys.executable, os.path.join(ROOT, "mnist_python_w1.py"), f"--ps_hosts={addr}",
                f"--worker_hosts=127.0.0.1:{launch.free_port()}", "--existing_servers=True", "--train_steps=2",
                f"--logdir={tmp_path}"] + COMMON
        ps = subprocess.Popen(base[:1] + [os.path.join(ROOT, "mnist_python_m.py")] + base[2:], cwd=ROOT,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        w = subprocess.run(base, cwd=ROOT, capture_output=True, text=True, timeout=300)
        assert w.returncode == 0, w.stdout + w.stderr
        assert "Using existing server at: grpc://" in w.stdout
        assert ps.wait(60) == 0
        assert srv.wait(60) == 0
    finally:
        for p in (srv,):
            if p.poll() is None:
                p.kill()


@pytest.mark.parametrize("n", [2, 8])
def test_bench_torchrun_cpu_dry_run(n):
    """bench.py's multi-rank contract (torchrun env, barrier, max over ranks, one JSON line on rank 0),
    up to the 8 ranks of the driver's 8-GPU job: probes over Gloo, identical replicas."""
    import json

    port = launch.free_port()
    env = dict(os.environ, OMP_NUM_THREADS=str(max(1, (os.cpu_count() or 8) // n)))
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", str(n), "--steps", "2", "--warmup", "1", "--cpu", "--batch_size", "16"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_ranks"] == n and rec["config"]["global_batch"] == 16 * n and rec["value"] > 0
    assert rec["replicas_identical"] and set(rec["schedule"]["candidates_ms_per_step"]) == {"flat", "buckets"}


def test_performance_table_tool(tmp_path):
    out = tmp_path / "performance"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "performance.py"), "--steps", "2,4",
                        "--out", str(out), "--", "--synthetic_data", "--eval_batches=1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = out.read_text().splitlines()
    assert lines[0] == "Steps ,Time ,Accuracy, Learning rate" and lines[1].split()[0] == "2" and len(lines) == 3


def test_watchdog_exits_nonzero():
    code = ("import time,sys; sys.path.insert(0, %r)\n"
            "from tensorflow_distributed_amd.utils.tracing import Watchdog\n"
            "w = Watchdog(0.5)\ntime.sleep(5)\n" % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3 and "watchdog" in p.stderr


def test_phase_watchdog_names_rank_phase_and_error_word():
    """bench.py / bench_resnet.py's rank-side watchdog: a phase past its limit prints the rank, the
    phase and the transport's error word, then exits non-zero; a finished phase never fires."""
    code = ("import time,sys; sys.path.insert(0, %r)\n"
            "from tensorflow_distributed_amd.utils.tracing import PhaseWatchdog\n"
            "w = PhaseWatchdog(3, err_fn=lambda: 7)\n"
            "w.phase('setup', 0.3); time.sleep(0.1); w.done(); time.sleep(1.0)\n"
            "w.phase('timed region (20 steps)', 0.5); time.sleep(10)\n" % ROOT)
    env = dict(os.environ, TFD_WATCHDOG_SCALE="1")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, env=env)
    assert p.returncode == 5, p.stderr
    assert "rank 3 phase 'timed region (20 steps)'" in p.stderr and "ipc error word 7" in p.stderr, p.stderr
    assert "'setup'" not in p.stderr


def test_bn_deterministic_flag_loads_the_library_first():
    """dist_main --bn_deterministic: in a fresh process nothing has loaded _C.so when the
    ResNet worker switches the BN statistics mode; the switch must load it and land in row mode."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from tensorflow_distributed_amd.training.dist_main import _set_bn_mode\n"
            "_set_bn_mode(True)\n"
            "import torch; print('slots', int(torch.ops.tfd.bn_part_slots()))\n" % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "slots 0" in p.stdout, p.stdout + p.stderr


def test_log_device_placement_round_robin():
    r = launch.launch(2, 1, ["--train_steps=1", "--sync_replicas=False", "--log_device_placement"] + COMMON,
                      echo=False, timeout_s=300)
    assert r["ok"]
    w = _out(r, "worker:0")
    assert "global_step: /job:ps/task:0/cpu:0" in w and "Variable: /job:ps/task:1/cpu:0" in w


def test_profile_prefix_puts_program_right_after_dashdash():
    from tensorflow_distributed_amd.launch import profiler_prefix

    p = profiler_prefix("/tmp/prof/worker0")
    assert p[0] == "rocprofv3" and p[-1] == "--" and "--stats" in p and "--pmc" not in p
    q = profiler_prefix("/tmp/prof/worker1", "SQ_WAVES,SQ_INSTS_VALU_MFMA_MOPS_BF16")
    assert q[q.index("--pmc") + 1:q.index("--pmc") + 3] == ["SQ_WAVES", "SQ_INSTS_VALU_MFMA_MOPS_BF16"]
    assert "--stats" not in q and "--sys-trace" not in q


def test_backup_workers_tolerate_a_straggler(tmp_path):
    """1 ps + 3 workers, replicas_to_aggregate=2, worker 2 stalls 12 s per step: the fast workers
    finish without waiting for it (TF accumulator semantics on the PS), its stale gradient is
    dropped, and everyone exits (mnist_python_m.py:62-65,216-220)."""
    import re

    args = ["--train_steps=6", "--replicas_to_aggregate=2", "--straggler_delay=2:12", "--batch_size=16",
            f"--logdir={tmp_path}"] + COMMON
    r = launch.launch(1, 3, args, echo=False, timeout_s=300)
    assert r["ok"], r["outputs"]
    def done_times(task):  # "<unix time>: Worker i: training step k done (global step: g)"
        return [float(t) for t in re.findall(r"^([0-9.]+): Worker \d+: training step \d+ done", _out(r, task), re.M)]

    fast_end = max(done_times("worker:0")[-1], done_times("worker:1")[-1])
    slow_first = done_times("worker:2")[0]
    slow = float(re.search(r"Training elapsed time: ([0-9.]+) s", _out(r, "worker:2")).group(1))
    # the fast workers finish every step while the straggler is still inside its first 12 s stall
    # (ordering, not a wall-clock ratio: CPU steps take 0.7-1.4 s depending on host load)
    assert slow > 12.0 and fast_end < slow_first, (fast_end, slow_first, slow)
    assert "stale gradient dropped" in _out(r, "worker:2")
    m = re.search(r"(\d+) synchronous updates, (\d+) stale gradients dropped", _out(r, "ps:0"))
    assert m and int(m.group(1)) == 6 and int(m.group(2)) >= 1, _out(r, "ps:0")
    for i in range(3):
        assert "global step: 6)" in _out(r, f"worker:{i}")


def test_async_checkpoint_holds_ps_adam_slots(tmp_path):
    """in async mode the optimizer state lives on the PS; the chief's checkpoint must
    hold those moments (not the worker's zero slots) so a resume continues Adam correctly."""
    import numpy as np

    from tensorflow_distributed_amd.training.checkpoint import load_bundle

    r = launch.launch(1, 2, ["--train_steps=4", "--sync_replicas=False", "--batch_size=16",
                             f"--logdir={tmp_path}"] + COMMON, echo=False, timeout_s=300)
    assert r["ok"], r["outputs"]
    ck = load_bundle(latest_checkpoint(str(tmp_path)))
    assert np.abs(ck["Variable_2/Adam"]).sum() > 0 and np.abs(ck["Variable_2/Adam_1"]).sum() > 0
    assert int(ck["global_step"]) >= 4
    assert abs(float(ck["beta1_power"]) - 0.9 ** int(ck["global_step"])) < 1e-6
    # resume: the restored moments go back to the PS (no restart of Adam from zero)
    r2 = launch.launch(1, 2, ["--train_steps=6", "--sync_replicas=False", "--batch_size=16",
                              f"--logdir={tmp_path}"] + COMMON, echo=False, timeout_s=300)
    assert r2["ok"], r2["outputs"]
    assert "Restored from checkpoint" in _out(r2, "worker:0")
    ck2 = load_bundle(latest_checkpoint(str(tmp_path)))
    assert int(ck2["global_step"]) >= 6
    assert abs(float(ck2["beta1_power"]) - 0.9 ** int(ck2["global_step"])) < 1e-6


def test_launcher_nproc_alias(monkeypatch):
    """--nproc N (SURVEY 5.6 launcher flag) is the worker count; the rest after -- reaches the script."""
    seen = {}

    def fake(num_ps, num_workers, rest, *a, **k):
        seen.update(num_ps=num_ps, num_workers=num_workers, rest=rest)
        return {"ok": True, "attempts": 1}

    monkeypatch.setattr(launch, "launch", fake)
    assert launch.main(["--num_ps", "1", "--nproc", "3", "--", "--train_steps=2"]) == 0
    assert seen == {"num_ps": 1, "num_workers": 3, "rest": ["--train_steps=2"]}
