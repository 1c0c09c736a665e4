"""Cluster description and in-process server: the ``tf.train.ClusterSpec`` / ``tf.train.Server`` /
``tf.train.replica_device_setter`` surface of ``/root/reference/mnist_python_m.py:145-177``.

MI355X-native re-expression:

* ``ClusterSpec({"ps": [...], "worker": [...]})`` keeps the reference's job/task naming. Global
  ranks are ``ps`` tasks first, then workers: ``rank(ps, i) = i``, ``rank(worker, j) = P + j``.
* ``Server`` does the rendezvous instead of starting a gRPC service: ``ps`` task 0 hosts a
  ``torch.distributed.TCPStore`` on its own ``host:port`` (``--ps_hosts[0]``); every task joins a
  Gloo control group over that store; the workers additionally form a worker sub-group (the sync
  gradient all-reduce group -- RCCL on GPUs, Gloo on CPUs). With ``existing_servers`` the store is
  hosted elsewhere (``python -m tensorflow_distributed_amd.server ...``) and tasks only attach.
* ``Server.join()`` on a ``ps`` task runs the parameter-server service (async mode, §5.8) or just
  waits for every worker's completion signal -- unlike the reference's ``join()``, which blocks
  forever (SURVEY quirk list, §5.3), the PS exits cleanly once all workers are done.
* :func:`replica_device_setter` returns the variable -> PS-task placement the TF device setter
  would produce: round-robin over PS tasks in variable-creation order (``:177``).
"""
from __future__ import annotations

import datetime
import os
import time
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist


class ClusterSpec:
    def __init__(self, cluster: Dict[str, Sequence[str]]):
        self._jobs = {k: [h.strip() for h in (v.split(",") if isinstance(v, str) else v) if h.strip()]
                      for k, v in cluster.items()}
        for k, v in self._jobs.items():
            if k not in ("ps", "worker", "chief", "evaluator"):
                raise ValueError(f"unknown job {k!r}")

    @property
    def jobs(self) -> List[str]:
        return list(self._jobs)

    def job_tasks(self, job: str) -> List[str]:
        return list(self._jobs.get(job, []))

    def num_tasks(self, job: str) -> int:
        return len(self._jobs.get(job, []))

    def task_address(self, job: str, index: int) -> str:
        return self._jobs[job][index]

    def as_dict(self) -> Dict[str, List[str]]:
        return {k: list(v) for k, v in self._jobs.items()}

    @property
    def num_ps(self) -> int:
        return self.num_tasks("ps")

    @property
    def num_workers(self) -> int:
        return self.num_tasks("worker")

    @property
    def world_size(self) -> int:
        return self.num_ps + self.num_workers

    def rank(self, job: str, index: int) -> int:
        if not 0 <= index < self.num_tasks(job):
            raise ValueError(f"task_index {index} out of range for job {job!r} ({self.num_tasks(job)} tasks)")
        return index if job == "ps" else self.num_ps + index

    def coordinator(self) -> str:
        """The rendezvous address: the first ps task (or the first worker when there is no ps job)."""
        return (self._jobs.get("ps") or self._jobs["worker"])[0]

    def __repr__(self):
        return f"ClusterSpec({self._jobs})"


def split_hostport(addr: str):
    host, _, port = addr.rpartition(":")
    if not host:
        raise ValueError(f"expected host:port, got {addr!r}")
    if host in ("localhost", ""):
        host = "127.0.0.1"
    return host, int(port)


def replica_device_setter(cluster: ClusterSpec, variable_names: Sequence[str], worker_device: str = "",
                          ps_device: str = "/job:ps/cpu:0") -> Dict[str, str]:
    """Variable -> device map of ``tf.train.replica_device_setter``: round-robin over PS tasks in
    creation order; without ps tasks every variable stays on the worker device."""
    p = cluster.num_ps
    if p == 0:
        return {n: worker_device for n in variable_names}
    base = ps_device.split("/task:")[0].replace("/job:ps", "")
    return {n: f"/job:ps/task:{i % p}{base}" for i, n in enumerate(variable_names)}


def ps_task_of(placement: Dict[str, str], name: str) -> int:
    dev = placement[name]
    if "/task:" not in dev:
        return -1
    return int(dev.split("/task:")[1].split("/")[0])


class Server:
    """``tf.train.Server(cluster, job_name, task_index)`` re-expressed as store + process groups."""

    def __init__(self, cluster: ClusterSpec, job_name: str, task_index: int, existing_servers: bool = False,
                 timeout_s: float = 600.0, start: bool = True):
        if job_name not in ("ps", "worker"):
            raise ValueError(f"job_name must be 'ps' or 'worker', got {job_name!r}")
        self.cluster = cluster
        self.job_name = job_name
        self.task_index = task_index
        self.rank = cluster.rank(job_name, task_index)
        self.world = cluster.world_size
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.existing_servers = existing_servers
        self.host, self.port = split_hostport(cluster.coordinator())
        self.store = None
        self.worker_group = None
        self._started = False
        if start:
            self.start()

    @property
    def target(self) -> str:
        return f"tfd://{self.host}:{self.port}"

    @property
    def is_store_host(self) -> bool:
        return (not self.existing_servers) and self.rank == 0

    def start(self) -> None:
        if self._started:
            return
        self.store = dist.TCPStore(self.host, self.port, world_size=None if self.existing_servers else self.world,
                                   is_master=self.is_store_host, timeout=self.timeout, wait_for_workers=False)
        pre = dist.PrefixStore("tfd/pg", self.store)
        if self.world > 1 and not dist.is_initialized():
            dist.init_process_group("gloo", store=pre, rank=self.rank, world_size=self.world, timeout=self.timeout)
        workers = list(range(self.cluster.num_ps, self.world))
        if self.world > 1:
            # every task must take part in new_group(); the PS tasks simply never use it
            self.worker_group = dist.new_group(ranks=workers, backend="gloo") if self.cluster.num_ps else dist.group.WORLD
        self._started = True

    # ---- signalling over the store ----
    def mark_done(self) -> None:
        self.store.add("tfd/workers_done", 1)

    def workers_done(self) -> int:
        return int(self.store.add("tfd/workers_done", 0))

    def join(self, service=None, poll_s: float = 0.2) -> None:
        """PS role: run ``service`` (async parameter server) or wait until every worker is done."""
        if service is not None:
            service.serve()
            return
        n = self.cluster.num_workers
        while self.workers_done() < n:
            time.sleep(poll_s)

    def shutdown(self) -> None:
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass
        self.store = None
        self._started = False
