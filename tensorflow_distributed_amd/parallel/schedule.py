"""Schedule probes: the multi-GPU job times its own candidate DP schedules and keeps the fastest.

Which data-parallel schedule wins depends on N and on the node (xGMI link count, RCCL's channel
choice, how much of the collective hides behind compute), so it cannot be settled on a one-GPU
box. A benchmark or training job with N > 1 therefore runs a short untimed probe of every
candidate at its real N -- fresh engine and transport per candidate, graph-replayed steps timed
between barriers -- takes the MAX over ranks of each candidate's ms/step (a step is as slow as
its slowest rank), and keeps the fastest. Every rank computes the identical choice from the
identical all-reduced numbers, so the collectives of the timed job stay matched.

The probes run inside the ranks, not in a parent process: the round driver launches the
benchmark under ``torch.distributed.run`` (one process per GPU, no parent of ours), and a
self-launched job (``parallel/spawn.py``) behaves the same way.

The reference has one schedule (the PS star of ``/root/reference/mnist_python_m.py:177,210-233``);
the candidates here are the all-reduce-world re-expressions of it.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Optional, Sequence, Tuple

# The bf16 MNIST engine's DP schedules (name -> MnistEngine switches), in probe order (ties go to the
# earlier one). "sfb": fc-region gradients by sufficient-factor broadcasting (all-gather the fc
# factors, 1.33 MB/rank at B = 128, and form the summed gradient locally); "+zero": ZeRO-1 sharding of
# the fc1 weight on top; "+mr": the conv slab reduce merged into the SFB GEMM's launch (the conv
# bucket's all-reduce then hides behind the fc-region optimizer instead of the GEMM); "allreduce": the
# bucketed bf16 gradient all-reduce (6.4 MB fc bucket + IPC one-shot conv bucket).
MNIST_SCHEDULES = {
    "sfb+zero+mr": {"fc_sfb": 1, "zero": 1, "merge_reduce": 1},
    "sfb+mr": {"fc_sfb": 1, "zero": 0, "merge_reduce": 1},
    "sfb+zero": {"fc_sfb": 1, "zero": 1, "merge_reduce": 0},
    "sfb": {"fc_sfb": 1, "zero": 0, "merge_reduce": 0},
    "allreduce": {"fc_sfb": 0, "zero": 0, "merge_reduce": 0},
}
# CPU (Gloo) sync DP: the flat gradient in one all-reduce, or the conv and fc buckets separately
CPU_SCHEDULES = ("flat", "buckets")


def probe(candidates: Sequence[str], run_one: Callable[[str], float], max_over_ranks: Callable[[float], float],
          log: Optional[Callable[[str], None]] = None) -> Dict[str, float]:
    """Run ``run_one(name)`` (local ms/step of one candidate; every rank calls it for the same names
    in the same order) and return {name: max over ranks of ms/step}. A candidate whose probe raised
    on this rank reports +inf; the exception's text goes to ``log``. Non-finite or non-positive
    times count as failures."""
    out: Dict[str, float] = {}
    for name in candidates:
        try:
            ms = float(run_one(name))
            if not (ms > 0 and math.isfinite(ms)):
                raise ValueError(f"probe of {name!r} returned {ms!r}")
        except Exception as e:  # noqa: BLE001 - a failed candidate is reported, not fatal, if others work
            if log:
                log(f"# schedule probe {name!r} failed: {e!r}")
            ms = math.inf
        out[name] = max_over_ranks(ms)
        if log:
            log(f"# schedule probe {name}: {out[name]:.4f} ms/step (max over ranks)")
    return out


def pick(times: Dict[str, float]) -> str:
    """Fastest candidate; ties go to the earlier candidate (dict order = probe order). Raises if no
    candidate produced a finite time."""
    best: Tuple[float, int, str] = (math.inf, 0, "")
    for i, (name, ms) in enumerate(times.items()):
        if ms < best[0]:
            best = (ms, i, name)
    if not math.isfinite(best[0]):
        raise RuntimeError(f"every schedule candidate failed its probe: {times}")
    return best[2]
