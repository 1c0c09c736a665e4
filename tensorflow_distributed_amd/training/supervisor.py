"""``tf.train.Supervisor`` re-expressed for the all-reduce world
(``/root/reference/mnist_python_m.py:235-253, 260-282``).

* ``prepare_or_wait_for_session``: the chief restores the newest checkpoint in ``logdir`` (a
  STABLE directory here -- the reference's ``tempfile.mkdtemp()`` logdir made resume impossible,
  SURVEY §5.3) or runs the init op (seeded ``normal(0, 1)``), then the state is broadcast to every
  worker (RCCL on GPUs, Gloo on CPUs). Non-chief workers block in that broadcast, which replaces
  the reference's 1-second readiness polling (``recovery_wait_secs``) with a collective wait.
* Services, chief only, as the TF defaults: checkpoint every ``save_model_secs`` (600) and the
  ``global_step/sec`` summary every ``save_summaries_secs`` (120). They are *cooperative*: timer
  threads only raise flags and :meth:`on_step` does the work between steps on the training thread,
  so a save never reads parameters in the middle of an update.
* :meth:`stop` (never called by the reference) writes a final checkpoint and closes the event file.
"""
from __future__ import annotations

import os
import threading
import time
from collections import OrderedDict
from typing import Callable, Optional

import numpy as np

from .checkpoint import Saver, latest_checkpoint, load_bundle
from .summary import EventFileWriter


class Supervisor:
    def __init__(self, is_chief: bool, logdir: Optional[str], runner, init_fn: Callable[[], None],
                 broadcast_fn: Optional[Callable[[], None]] = None, save_model_secs: float = 600.0,
                 save_summaries_secs: float = 120.0, recovery_wait_secs: float = 1.0, max_to_keep: int = 5,
                 summary_writer: bool = True, log=print):
        self.is_chief = is_chief
        self.logdir = logdir
        self.runner = runner
        self.init_fn = init_fn
        self.broadcast_fn = broadcast_fn
        self.save_model_secs = save_model_secs
        self.save_summaries_secs = save_summaries_secs
        self.recovery_wait_secs = recovery_wait_secs
        self.saver = Saver(max_to_keep=max_to_keep)
        self.writer = EventFileWriter(logdir) if (is_chief and logdir and summary_writer) else None
        self.log = log
        self._save_due = threading.Event()
        self._summary_due = threading.Event()
        self._stop = threading.Event()
        self._threads = []
        self._last_summary = (time.time(), 0)
        self.restored_from = None
        self.last_save_path = None

    # ---- session preparation ----
    def prepare_or_wait_for_session(self) -> None:
        if self.is_chief:
            ckpt = latest_checkpoint(self.logdir) if self.logdir else None
            if ckpt:
                self.runner.load_state_dict_tf(load_bundle(ckpt))
                self.restored_from = ckpt
                self.log(f"Restored from checkpoint {ckpt} (global step {self.runner.global_step()})")
            else:
                self.init_fn()
        if self.broadcast_fn is not None:
            self.broadcast_fn()
        self._last_summary = (time.time(), self.runner.global_step())
        if self.is_chief:
            self._start_services()

    def _start_services(self):
        def timer(ev: threading.Event, every: float):
            while not self._stop.wait(every):
                ev.set()

        if self.logdir and self.save_model_secs and self.save_model_secs > 0:
            t = threading.Thread(target=timer, args=(self._save_due, self.save_model_secs), daemon=True)
            t.start()
            self._threads.append(t)
        if self.writer is not None and self.save_summaries_secs and self.save_summaries_secs > 0:
            t = threading.Thread(target=timer, args=(self._summary_due, self.save_summaries_secs), daemon=True)
            t.start()
            self._threads.append(t)

    # ---- per-step services (training thread) ----
    def save_due(self) -> bool:
        """The chief's checkpoint timer has fired and the save has not happened yet."""
        return self.is_chief and self._save_due.is_set()

    def on_step(self, global_step: int, scalars: Optional[dict] = None, allow_save: bool = True) -> None:
        """``allow_save=False`` defers a due checkpoint (the flag stays set): a sharded run saves only at
        steps where every worker first gathered the shards (dist_main's ZeRO-1 sync points)."""
        if not self.is_chief:
            return
        if self._summary_due.is_set():
            self._summary_due.clear()
            self.write_summary(global_step, scalars)
        if allow_save and self._save_due.is_set():
            self._save_due.clear()
            self.save(global_step)

    def write_summary(self, global_step: int, scalars: Optional[dict] = None) -> None:
        if self.writer is None:
            return
        now = time.time()
        t0, s0 = self._last_summary
        vals = dict(scalars or {})
        if now > t0:
            vals["global_step/sec"] = (global_step - s0) / (now - t0)
        self.writer.add_scalars(vals, global_step)
        self._last_summary = (now, global_step)

    def save(self, global_step: Optional[int] = None) -> Optional[str]:
        if not (self.is_chief and self.logdir):
            return None
        gs = self.runner.global_step() if global_step is None else global_step
        self.last_save_path = self.saver.save(self.logdir, self.runner.state_dict_tf(), gs)
        return self.last_save_path

    def stop(self, save: bool = True) -> None:
        self._stop.set()
        if self.is_chief and save and self.logdir:
            self.save()
            self.write_summary(self.runner.global_step())
        if self.writer is not None:
            self.writer.close()
