"""Self-launch contract of bench.py / bench_resnet.py (parallel/spawn.py): ``--gpus N`` without a
launcher environment spawns N ranks from a parent that never imports torch (so it never
initialises HIP), relays exactly one JSON line, and fails when a rank fails or when the job's
WORLD_SIZE differs from --gpus."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _clean_env():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    return env


def test_bench_self_launch_parent_stays_gpu_clean():
    code = textwrap.dedent("""
        import sys
        sys.path.insert(0, %r)
        import bench
        rc = bench.main(["--cpu", "--gpus", "2", "--steps", "2", "--warmup", "1"])
        assert rc == 0, rc
        bad = [m for m in sys.modules if m == "torch" or m.startswith("torch.")]
        assert not bad, "parent imported torch: " + str(bad[:5])
        print("PARENT_CLEAN", file=sys.stderr)
    """ % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=_clean_env(),
                       cwd=ROOT)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PARENT_CLEAN" in p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    r = json.loads(lines[0])
    assert r["n_ranks"] == 2 and r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 256


def test_bench_refuses_wrong_world():
    env = dict(_clean_env(), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2", "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr and not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_spawn_fails_fast_when_a_rank_fails(tmp_path):
    script = tmp_path / "job.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        r = int(os.environ["RANK"])
        assert os.environ["WORLD_SIZE"] == "3" and os.environ["MASTER_ADDR"] == "127.0.0.1"
        if r == 1:
            sys.exit(7)
        time.sleep(60)  # the others would hang on a collective; the parent must tear them down
    """))
    sys.path.insert(0, ROOT)
    from tensorflow_distributed_amd.parallel import spawn

    import time

    t0 = time.time()
    rc = spawn.self_launch(str(script), [], 3)
    assert rc == 7
    assert time.time() - t0 < 30


def test_spawn_relays_rank0_stdout_only(tmp_path):
    script = tmp_path / "job.py"
    script.write_text("import os\nprint('LINE', os.environ['RANK'], os.environ['LOCAL_RANK'], flush=True)\n")
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from tensorflow_distributed_amd.parallel import spawn\n"
            "sys.exit(spawn.self_launch(%r, [], 2))\n") % (ROOT, str(script))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, env=_clean_env())
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip() == "LINE 0 0"
    assert "LINE 1 1" in p.stderr
