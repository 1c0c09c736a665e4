"""Trace ranges and debug switches.

* :func:`trace_range` -- roctx ranges (``torch.cuda.nvtx`` maps to roctx on ROCm) around host
  phases, visible in ``rocprofv3 --marker-trace`` timelines; a no-op without a GPU.
* :func:`enable_debug_sync` -- ``AMD_SERIALIZE_KERNEL=3`` + ``HIP_LAUNCH_BLOCKING=1``: every
  launch synchronous, the race-hunting mode; must run before the first HIP call.
* :class:`Watchdog` -- the collective/step timeout: if no step completes within ``timeout_s`` it
  aborts the communicator (unblocking a hung RCCL collective) and exits non-zero so the launcher
  tears the cluster down and restarts it from the last checkpoint.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from contextlib import contextmanager


@contextmanager
def trace_range(name: str):
    pushed = False
    try:
        import torch

        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:
        pushed = False
    try:
        yield
    finally:
        if pushed:
            import torch

            torch.cuda.nvtx.range_pop()


def enable_debug_sync() -> None:
    os.environ["AMD_SERIALIZE_KERNEL"] = "3"
    os.environ["HIP_LAUNCH_BLOCKING"] = "1"
    os.environ["AMD_SERIALIZE_COPY"] = "3"


class Watchdog:
    def __init__(self, timeout_s: float, on_timeout=None, name: str = "step"):
        self.timeout_s = timeout_s
        self.on_timeout = on_timeout
        self.name = name
        self._last = time.time()
        self._stop = threading.Event()
        self._t = None
        if timeout_s and timeout_s > 0:
            self._t = threading.Thread(target=self._run, daemon=True)
            self._t.start()

    def kick(self) -> None:
        self._last = time.time()

    def _run(self):
        while not self._stop.wait(min(1.0, self.timeout_s / 4)):
            if time.time() - self._last > self.timeout_s:
                sys.stderr.write(f"watchdog: no {self.name} progress for {self.timeout_s:.0f} s; aborting\n")
                sys.stderr.flush()
                try:
                    if self.on_timeout:
                        self.on_timeout()
                finally:
                    os._exit(3)

    def stop(self) -> None:
        self._stop.set()


class PhaseWatchdog:
    """Rank-side bound on every phase of a benchmark job (setup, each schedule probe, warm-up, the
    timed region, teardown).

    ``phase(name, limit_s)`` arms a deadline for the phase that starts now; ``done()`` disarms it. If
    a phase is still running at its deadline, the watchdog thread prints one line naming the rank,
    the phase, its limit and the transport's error word (``err_fn()``, read on a helper thread that
    may itself be stuck behind a hung GPU: then it says so), and ends the process with
    ``os._exit(code)`` -- no re-exec, nothing else runs. The launcher (torchrun or
    parallel/spawn.py) sees the non-zero exit and tears the job down, so a first-contact hang on a
    new world size ends with a diagnosis instead of at the driver's wall-clock limit.

    ``TFD_WATCHDOG_SCALE`` multiplies every limit (0 disables the watchdog)."""

    def __init__(self, rank: int, err_fn=None, code: int = 5, tag: str = "bench"):
        self.rank = rank
        self.err_fn = err_fn
        self.code = code
        self.tag = tag
        try:
            self.scale = float(os.environ.get("TFD_WATCHDOG_SCALE", "1"))
        except ValueError:
            self.scale = 1.0
        self._lock = threading.Lock()
        self._phase = None
        self._limit = 0.0
        self._deadline = None
        self._t0 = 0.0
        self._stop = threading.Event()
        self._t = None
        if self.scale > 0:
            self._t = threading.Thread(target=self._run, daemon=True, name="tfd-phase-watchdog")
            self._t.start()

    def phase(self, name: str, limit_s: float) -> None:
        now = time.time()
        with self._lock:
            self._phase, self._limit, self._t0 = name, limit_s * self.scale, now
            self._deadline = now + self._limit if self.scale > 0 else None

    def done(self) -> None:
        with self._lock:
            self._phase, self._deadline = None, None

    def current(self):
        with self._lock:
            return self._phase

    def _error_word(self) -> str:
        if self.err_fn is None:
            return "n/a"
        box = []

        def read():
            try:
                box.append(str(int(self.err_fn())))
            except Exception as e:  # noqa: BLE001 - diagnostic only
                box.append(f"unreadable ({e!r})")

        t = threading.Thread(target=read, daemon=True)
        t.start()
        t.join(3.0)
        return box[0] if box else "unreadable (the read is stuck behind the GPU)"

    def _run(self):
        while not self._stop.wait(0.25):
            with self._lock:
                name, dl, lim, t0 = self._phase, self._deadline, self._limit, self._t0
            if dl is None or time.time() <= dl:
                continue
            msg = (f"watchdog[{self.tag}]: rank {self.rank} phase '{name}' still running after "
                   f"{time.time() - t0:.1f} s (limit {lim:.0f} s); ipc error word {self._error_word()}; exiting "
                   f"with {self.code}\n")
            try:
                sys.stderr.write(msg)
                sys.stderr.flush()
                sys.stdout.flush()
            finally:
                os._exit(self.code)

    def stop(self) -> None:
        self.done()
        self._stop.set()
