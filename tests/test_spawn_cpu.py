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
    # the ranks probed both CPU schedules (the parent above still never imported torch) and kept the
    # faster one; the replicas agree after the timed steps
    c = r["schedule"]["candidates_ms_per_step"]
    assert set(c) == {"flat", "buckets"} and r["schedule"]["chosen"] == min(c, key=c.get)
    assert r["replicas_identical"]


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


def test_schedule_pick_takes_max_over_ranks_and_fastest():
    """probe() reports each candidate's MAX over ranks (a step is as slow as its slowest rank) and
    pick() the fastest of those; a failing candidate is +inf, never chosen; all failing raises."""
    import math

    import pytest

    sys.path.insert(0, ROOT)
    from tensorflow_distributed_amd.parallel import schedule as S

    local = {"a": 1.0, "b": 2.0, "c": 0.5}
    other_rank = {"a": 3.0, "b": 2.5, "c": 9.0}  # rank 1 is slow on c
    order = ["a", "b", "c"]
    got = S.probe(order, lambda n: local[n], lambda x, it=iter(order): max(x, other_rank[next(it)]))
    assert got == {"a": 3.0, "b": 2.5, "c": 9.0} and S.pick(got) == "b"

    def flaky(n):
        if n == "x":
            raise RuntimeError("capture failed")
        return 4.0
    got = S.probe(["x", "y"], flaky, lambda v: v)
    assert math.isinf(got["x"]) and S.pick(got) == "y"
    assert S.pick({"p": 1.0, "q": 1.0}) == "p"  # ties: probe order
    with pytest.raises(RuntimeError):
        S.pick({"x": math.inf})


def test_bench_schedule_flags_resolve():
    """--schedule NAME and the --fc_sfb/--zero/--merge_reduce overrides fix the schedule without probes; a one-GPU
    job without --force_dp has no DP schedule at all."""
    sys.path.insert(0, ROOT)
    import bench

    a = bench._args(["--gpus", "4"])
    assert bench._candidates(a, True) == (list(bench.SCHEDULES), "probe")
    assert bench._candidates(a, False) == ([None], "single")
    assert bench._candidates(bench._args(["--schedule", "sfb"]), True) == (["sfb"], "flag")
    assert bench._candidates(bench._args(["--fc_sfb", "0", "--zero", "0"]), True) == (["allreduce"], "flag")
    assert bench._candidates(bench._args(["--fc_sfb", "1", "--zero", "1"]), True) == (["sfb+zero+mr"], "flag")
    assert bench._candidates(bench._args(["--fc_sfb", "1", "--zero", "1", "--merge_reduce", "0"]), True) == \
        (["sfb+zero"], "flag")
    assert bench._candidates(bench._args(["--fc_sfb", "1", "--merge_reduce", "1"]), True) == (["sfb+mr"], "flag")
    assert bench._candidates(bench._args(["--candidates", "sfb,allreduce"]), True) == (["sfb", "allreduce"], "probe")
