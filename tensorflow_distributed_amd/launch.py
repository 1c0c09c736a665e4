"""Local cluster launcher with failure detection and restart.

Starts every role of a ``ClusterSpec`` on this node -- what the reference did by hand with three
shells running ``mnist_python_m.py`` / ``_w1.py`` / ``_w2.py`` against ``10.0.1.x`` hosts -- on
127.0.0.1 with free ports, prefixes and collects their output, and watches them:

* a worker that exits non-zero (crash, ``--fault_inject_step``, OOM kill) tears the whole cluster
  down (process groups, SIGTERM then SIGKILL) and, up to ``--max_restarts`` times, starts it again
  with ``TFD_RESTART_COUNT`` set; with a stable ``--logdir`` in the script flags the chief resumes
  from the newest checkpoint (Supervisor restore), so training continues instead of restarting;
* the run succeeds when every worker exits 0 (the ps tasks exit on their own afterwards).

    python -m tensorflow_distributed_amd.launch --num_ps 1 --num_workers 2 [--num_gpus 0] \\
        [--max_restarts 1] [--log_dir DIR] [--script mnist_python_m.py] -- --train_steps=20 --logdir=/tmp/run
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import threading
import time
from typing import List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    from .parallel.spawn import free_port as _free_port  # below the ephemeral range (see there)

    return _free_port()


class Proc:
    def __init__(self, role: str, index: int, cmd: List[str], env: dict, log_path: Optional[str], echo: bool):
        self.role, self.index = role, index
        self.name = f"{role}:{index}"
        self.lines: List[str] = []
        self._log = open(log_path, "a") if log_path else None
        self.p = subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                  text=True, bufsize=1, start_new_session=True)
        self._echo = echo
        self._t = threading.Thread(target=self._pump, daemon=True)
        self._t.start()

    def _pump(self):
        for line in self.p.stdout:
            self.lines.append(line)
            if self._log:
                self._log.write(line)
                self._log.flush()
            if self._echo:
                sys.stdout.write(f"[{self.name}] {line}")
                sys.stdout.flush()

    def poll(self):
        return self.p.poll()

    def kill(self, grace: float = 5.0):
        if self.p.poll() is not None:
            return
        try:
            os.killpg(self.p.pid, signal.SIGTERM)
        except ProcessLookupError:
            return
        try:
            self.p.wait(grace)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(self.p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            self.p.wait()

    def finish(self):
        self._t.join(timeout=5)
        if self._log:
            self._log.close()


def profiler_prefix(out_dir: str, pmc: str = "") -> List[str]:
    """rocprofv3 command prefix (SURVEY 5.1 ``--profile``): kernel trace + per-kernel stats, or one
    PMC counter pass (counters of one pass only; see scripts/gpu_run.sh pmc= and the per-block limits in docs/DESIGN.md)."""
    if pmc:
        return ["rocprofv3", "--kernel-trace", "--pmc", *pmc.split(","), "-d", out_dir, "-o", "run", "--"]
    return ["rocprofv3", "--kernel-trace", "--stats", "-d", out_dir, "-o", "run", "--"]


def launch(num_ps: int, num_workers: int, script_args: List[str], script: str = "mnist_python_m.py",
           max_restarts: int = 0, log_dir: Optional[str] = None, echo: bool = True, timeout_s: float = 3600.0,
           python: str = sys.executable, extra_env: Optional[dict] = None, profile_dir: Optional[str] = None,
           profile_pmc: str = "") -> dict:
    """Run the cluster to completion. Returns {"ok", "attempts", "outputs": {name: text}}.

    ``profile_dir``: run every worker under ``rocprofv3 --kernel-trace --stats`` (or, with
    ``profile_pmc``, a counter pass ``--pmc <counters>``; never combined with trace domains) into
    ``<profile_dir>/worker<i>``. The worker program comes directly after ``--`` (no shell or
    env hop: the profiler initialises the GPU before the program starts)."""
    attempt = 0
    outputs = {}
    while True:
        ps_hosts = ",".join(f"127.0.0.1:{free_port()}" for _ in range(num_ps))
        worker_hosts = ",".join(f"127.0.0.1:{free_port()}" for _ in range(num_workers))
        env = dict(os.environ)
        env.update(extra_env or {})
        env["TFD_RESTART_COUNT"] = str(attempt)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        base = [python, os.path.join(ROOT, script) if not os.path.isabs(script) else script,
                f"--ps_hosts={ps_hosts}", f"--worker_hosts={worker_hosts}"]
        procs: List[Proc] = []
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)
        for i in range(num_ps):
            lp = os.path.join(log_dir, f"ps{i}.attempt{attempt}.log") if log_dir else None
            procs.append(Proc("ps", i, base + ["--job_name=ps", f"--task_index={i}"] + script_args, env, lp, echo))
        for i in range(num_workers):
            lp = os.path.join(log_dir, f"worker{i}.attempt{attempt}.log") if log_dir else None
            cmd = base + ["--job_name=worker", f"--task_index={i}"] + script_args
            if profile_dir:
                cmd = profiler_prefix(os.path.join(profile_dir, f"worker{i}"), profile_pmc) + cmd
            procs.append(Proc("worker", i, cmd, env, lp, echo))
        t0 = time.time()
        failed = None
        while True:
            workers = [p for p in procs if p.role == "worker"]
            codes = [p.poll() for p in workers]
            bad = [p for p, c in zip(workers, codes) if c not in (None, 0)]
            bad += [p for p in procs if p.role == "ps" and p.poll() not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            if all(c == 0 for c in codes):
                # workers done: give the ps tasks a moment to observe completion and exit
                for p in procs:
                    if p.role == "ps":
                        try:
                            p.p.wait(30)
                        except subprocess.TimeoutExpired:
                            p.kill()
                break
            if time.time() - t0 > timeout_s:
                failed = workers[0]
                break
            time.sleep(0.05)
        for p in procs:
            if failed is not None:
                p.kill()
            p.finish()
            outputs[f"{p.name}#{attempt}"] = "".join(p.lines)
        if failed is None:
            return {"ok": True, "attempts": attempt + 1, "outputs": outputs}
        print(f"[launch] {failed.name} exited with {failed.poll()} (attempt {attempt}); "
              f"{'restarting' if attempt < max_restarts else 'giving up'}", flush=True)
        if attempt >= max_restarts:
            return {"ok": False, "attempts": attempt + 1, "outputs": outputs, "failed": failed.name}
        attempt += 1


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" in argv:
        i = argv.index("--")
        ours, rest = argv[:i], argv[i + 1:]
    else:
        ours, rest = argv, []
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--num_ps", type=int, default=1)
    ap.add_argument("--num_workers", type=int, default=2)
    ap.add_argument("--nproc", type=int, default=None, help="worker processes on this node (SURVEY 5.6 name; "
                    "overrides --num_workers)")
    ap.add_argument("--script", default="mnist_python_m.py")
    ap.add_argument("--max_restarts", type=int, default=0)
    ap.add_argument("--log_dir", default=None)
    ap.add_argument("--timeout", type=float, default=3600.0)
    ap.add_argument("--profile", default=None, metavar="DIR", help="run workers under rocprofv3 into DIR/worker<i>")
    ap.add_argument("--profile_pmc", default="", help="comma-separated PMC counters for one --profile pass")
    a = ap.parse_args(ours)
    if a.nproc is not None:
        a.num_workers = a.nproc
    r = launch(a.num_ps, a.num_workers, rest, a.script, a.max_restarts, a.log_dir, True, a.timeout,
               profile_dir=a.profile, profile_pmc=a.profile_pmc)
    print(f"[launch] {'ok' if r['ok'] else 'FAILED'} after {r['attempts']} attempt(s)", flush=True)
    return 0 if r["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
