"""Metrics, step timing and trace export.

* :class:`MetricsLogger` -- ``--metrics_file`` JSONL on the chief: one record per step
  (step, global_step, loss, images/sec, step_ms, ...).
* :class:`StepTimer` -- host wall-clock phases; keeps a chrome-trace (``chrome://tracing`` /
  Perfetto JSON) of per-phase spans for ``--trace_file``. GPU phases (forward, fc/conv backward,
  optimizer, all-reduce) come from the engine's HIP timing events (``runner.phase_times()``,
  recorded inside the captured step graph) and are added to the same trace by :meth:`add_gpu_phases`.
* :func:`performance_table` -- the reference's ``performance`` file format
  (``Steps ,Time ,Accuracy, Learning rate``, ``/root/reference/performance:1-6``).
"""
from __future__ import annotations

import json
import os
import threading
import time
from contextlib import contextmanager
from typing import Dict, List, Optional


class MetricsLogger:
    def __init__(self, path: Optional[str]):
        self.path = path
        self._f = None
        self._lock = threading.Lock()
        if path:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._f = open(path, "a")

    def log(self, **rec) -> None:
        if self._f is None:
            return
        rec.setdefault("time", time.time())
        with self._lock:
            self._f.write(json.dumps(rec) + "\n")
            self._f.flush()

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None


class StepTimer:
    """Named host wall-time phases + GPU phase spans; chrome-trace events in µs."""

    def __init__(self, pid: int = 0, enabled: bool = True, max_events: int = 200000):
        self.pid = pid
        self.enabled = enabled
        self.events: List[dict] = []
        self.totals: Dict[str, float] = {}
        self.counts: Dict[str, int] = {}
        self.max_events = max_events

    @contextmanager
    def phase(self, name: str, tid: int = 0):
        if not self.enabled:
            yield
            return
        t0 = time.perf_counter()
        try:
            yield
        finally:
            t1 = time.perf_counter()
            self.totals[name] = self.totals.get(name, 0.0) + (t1 - t0)
            self.counts[name] = self.counts.get(name, 0) + 1
            if len(self.events) < self.max_events:
                self.events.append({"name": name, "ph": "X", "pid": self.pid, "tid": tid,
                                    "ts": t0 * 1e6, "dur": (t1 - t0) * 1e6})

    def add_gpu_phases(self, end_s: float, phases: Dict[str, float], tid: int = 1) -> None:
        """Lay the GPU phase durations (ms, in step order) back to back ending at host time ``end_s``
        on their own trace row."""
        if not self.enabled:
            return
        order = ["fwd_ms", "bwd_fc_ms", "bwd_conv_ms", "optim_ms"]
        total = sum(phases.get(k, 0.0) for k in order)
        t = end_s * 1e6 - total * 1e3
        for k in order:
            d = phases.get(k, 0.0) * 1e3
            if d > 0 and len(self.events) < self.max_events:
                self.events.append({"name": "gpu:" + k[:-3], "ph": "X", "pid": self.pid, "tid": tid, "ts": t, "dur": d})
            t += d
        ar = phases.get("allreduce_ms", 0.0)
        if ar and len(self.events) < self.max_events:
            self.events.append({"name": "gpu:allreduce", "ph": "X", "pid": self.pid, "tid": tid + 1,
                                "ts": end_s * 1e6 - ar * 1e3, "dur": ar * 1e3})

    def mean_ms(self, name: str) -> float:
        n = self.counts.get(name, 0)
        return 1e3 * self.totals.get(name, 0.0) / n if n else 0.0

    def write_chrome_trace(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events, "displayTimeUnit": "ms"}, f)


def performance_table(rows: List[dict]) -> str:
    """rows: dicts with steps, time, accuracy (%), lr -> the reference's whitespace table."""
    out = ["Steps ,Time ,Accuracy, Learning rate"]
    for r in rows:
        # the reference prints whole seconds; sub-10 s runs (one GPU) keep two decimals
        t = f"{r['time']:<4.0f}" if r["time"] >= 10 else f"{r['time']:<6.2f}"
        out.append(f"{r['steps']:<6}{t}{r['accuracy']:<7g}{r['lr']:g}")
    return "\n".join(out) + "\n"
