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
