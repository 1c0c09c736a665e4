"""Self-launch of one rank process per GPU from a GPU-clean parent.

``python bench.py --gpus N`` without a torchrun environment must still measure N GPUs (the
reference's headline is a real multi-process run: 1 PS + 2 workers,
``/root/reference/mnist_python_m.py:81-84,210-233``, ``/root/reference/performance:1-6``).
The parent here only ``Popen``s N children with the torchrun-style environment
(``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE`` / ``MASTER_ADDR=127.0.0.1`` / ``MASTER_PORT``),
relays rank 0's stdout (the one JSON line) to its own stdout, sends every other rank's stdout
to stderr, and exits non-zero as soon as any child fails (the rest are torn down).

This module must not import torch: the parent never initialises HIP (``tests/test_spawn_cpu.py``
checks that), so a child is never started from a process that already touched the GPU.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional, Sequence

SELF_LAUNCH_ENV = "TFD_SELF_LAUNCHED"


def free_port() -> int:
    """A port that binds now, taken BELOW the kernel's ephemeral range (Linux 32768-60999): a port
    from bind(0) is released and only bound again by the child a moment later, and in between an
    outgoing connection (another job's Gloo or TCPStore client) may take it as its local port --
    EADDRINUSE in a launched task. Ports under 32768 are never handed out that way."""
    import random

    rng = random.SystemRandom()
    for _ in range(64):
        port = rng.randrange(20000, 32000)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def under_launcher() -> bool:
    """True when this process already is one rank of a launched job (torchrun or self-launch)."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def needs_self_launch(n: int) -> bool:
    return n > 1 and not under_launcher()


def _pump(src, dst, lock: threading.Lock) -> None:
    for line in iter(src.readline, ""):
        with lock:
            dst.write(line)
            dst.flush()
    src.close()


def _kill_group(p: subprocess.Popen, grace: float = 10.0) -> None:
    if p.poll() is not None:
        return
    try:
        os.killpg(p.pid, signal.SIGTERM)
    except ProcessLookupError:
        return
    try:
        p.wait(grace)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.wait()


def self_launch(script: str, argv: Sequence[str], n: int, timeout_s: Optional[float] = None,
                python: str = sys.executable, extra_env: Optional[dict] = None) -> int:
    """Run ``python script *argv`` as ranks 0..n-1 of one job on this node; return the job's exit code
    (0 only if every rank exited 0). Each child is its own process group, so a failing rank's
    siblings (and anything they started) are torn down together."""
    port = free_port()
    base = dict(os.environ)
    base.update(extra_env or {})
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                **{SELF_LAUNCH_ENV: "1"})
    lock = threading.Lock()
    procs: List[subprocess.Popen] = []
    pumps: List[threading.Thread] = []
    try:
        for r in range(n):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
            p = subprocess.Popen([python, script, *argv], env=env, stdout=subprocess.PIPE, text=True, bufsize=1,
                                 start_new_session=True)
            procs.append(p)
            t = threading.Thread(target=_pump, args=(p.stdout, sys.stdout if r == 0 else sys.stderr, lock),
                                 daemon=True)
            t.start()
            pumps.append(t)
        t0 = time.time()
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print(f"[spawn] rank {r} exited with {c}; stopping the other ranks", file=sys.stderr, flush=True)
                return c if c > 0 else 1
            if all(c == 0 for c in codes):
                return 0
            if timeout_s is not None and time.time() - t0 > timeout_s:
                print(f"[spawn] job exceeded {timeout_s:.0f} s; stopping it", file=sys.stderr, flush=True)
                return 124
            time.sleep(0.05)
    except KeyboardInterrupt:
        return 130
    finally:
        for p in procs:
            _kill_group(p)
        for t in pumps:
            t.join(timeout=5)


def check_world(requested: int, world: int, what: str = "--gpus") -> None:
    """Fail loudly when the job does not have the rank count the caller asked for (a benchmark that
    silently measured fewer GPUs than its JSON claims would report a flat scaling curve)."""
    if requested != world:
        raise SystemExit(f"error: {what} {requested} but this job has WORLD_SIZE={world} ranks; launch it with "
                         f"--nproc-per-node {requested} or without a launcher environment (self-launch)")
