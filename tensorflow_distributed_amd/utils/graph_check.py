"""Dependency check of a captured multi-stream training-step graph.

``MnistEngine.capture_topology(n)`` captures ``n`` consecutive training steps exactly as the
benchmark's replayed graph (compute stream, comm stream, optimizer stream, every RCCL / IPC
collective, every cross-stream event edge) and returns its nodes, edges and, per schedule
operation, the nodes that operation added (``tag <label>@<step> <node>...``). This module turns
that text into a DAG and checks the schedule's data dependencies:

* read-after-write: a collective starts only after the kernel that produced its operand, and its
  consumers start only after it (e.g. ``slab_reduce -> ar_conv -> opt_conv``);
* write-after-read across steps: the next step must not overwrite a buffer a collective of this
  step still reads (e.g. ``gather_p2@i -> conv_fwd@i+1``: the next conv forward rewrites this
  rank's p2 slot that the all-gather reads).

A missing ``hipStreamWaitEvent`` between the comm and compute streams is invisible on one GPU
whose ranks time-slice (the collective happens to finish first) and a data race with real peers;
here it is a missing path in the DAG. ``A -> B`` means: every node of A reaches every node of B.

The reference's equivalent ordering is implicit in TF's graph executor plus the sync token queue
(``/root/reference/mnist_python_m.py:216-233``); SURVEY.md §5.2 asks for the stream-ordering
discipline to be checked.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Optional, Sequence, Set, Tuple


class Topology:
    def __init__(self, lines: Sequence[str]):
        self.types: Dict[int, int] = {}
        self.succ: Dict[int, Set[int]] = defaultdict(set)
        self.tags: List[Tuple[str, int, List[int]]] = []  # (label, step, nodes) in host issue order
        for ln in lines:
            f = ln.split()
            if not f:
                continue
            if f[0] == "node":
                self.types[int(f[1])] = int(f[2])
            elif f[0] == "edge":
                self.succ[int(f[1])].add(int(f[2]))
            elif f[0] == "tag":
                label, step = f[1].rsplit("@", 1)
                self.tags.append((label, int(step), [int(x) for x in f[2:]]))
        self._reach: Dict[int, Set[int]] = {}

    def reach(self, a: int) -> Set[int]:
        """Nodes reachable from ``a`` (excluding ``a``)."""
        if a not in self._reach:
            seen: Set[int] = set()
            stack = list(self.succ.get(a, ()))
            while stack:
                x = stack.pop()
                if x in seen:
                    continue
                seen.add(x)
                stack.extend(self.succ.get(x, ()))
            self._reach[a] = seen
        return self._reach[a]

    def ordered(self, a_nodes: Sequence[int], b_nodes: Sequence[int]) -> bool:
        """Every node of A reaches every node of B (A finishes before B starts)."""
        return all(set(b_nodes) <= self.reach(a) for a in a_nodes)

    def find(self, label: str, step: int, after: int = -1) -> Optional[int]:
        """Index (in issue order) of the first tag ``label@step`` after position ``after``."""
        for i, (lb, st, _) in enumerate(self.tags):
            if i > after and lb == label and st == step:
                return i
        return None

    def steps(self) -> List[int]:
        return sorted({st for _, st, _ in self.tags})


def _first(t: Topology, labels: Sequence[str], step: int) -> Optional[int]:
    for lb in labels:
        i = t.find(lb, step)
        if i is not None:
            return i
    return None


def required(t: Topology) -> List[Tuple[int, int, str]]:
    """(producer tag index, consumer tag index, reason) pairs the schedule must order."""
    labels = {lb for lb, _, _ in t.tags}
    steps = t.steps()
    req: List[Tuple[int, int, str]] = []

    def add(a: Optional[int], b: Optional[int], why: str):
        if a is not None and b is not None:
            req.append((a, b, why))

    opt_any = ("opt", "opt_fc", "opt_conv")
    for k, i in enumerate(steps):
        nxt = steps[k + 1] if k + 1 < len(steps) else None
        f = lambda lb, st=i: t.find(lb, st)  # noqa: E731
        if "gather_p2" in labels:  # sufficient-factor schedule
            add(f("conv_fwd"), f("gather_p2"), "RAW p2 slot -> all-gather")
            add(f("gather_p2"), f("sfb_gemm"), "RAW gathered p2 -> SFB GEMM")
            add(f("fc_fwd"), f("gather_dr"), "RAW dh/hd/dlogits slot -> all-gather")
            add(f("gather_dr"), f("sfb_gemm"), "RAW gathered dh/hd/dlogits -> SFB GEMM")
            add(f("slab_reduce"), f("ar_conv"), "RAW conv bucket -> all-reduce")
            add(f("ar_conv"), _first(t, ("opt_conv", "opt"), i), "RAW reduced conv bucket -> optimizer")
            add(f("sfb_gemm"), _first(t, ("opt_fc", "opt"), i), "RAW fc gradient -> optimizer")
            if nxt is not None:
                add(f("gather_p2"), t.find("conv_fwd", nxt), "WAR next conv fwd rewrites the gathered p2 slot")
                add(f("gather_dr"), t.find("fc_fwd", nxt), "WAR next head rewrites the gathered dh slot")
                add(f("ar_conv"), t.find("slab_reduce", nxt), "WAR next slab reduce rewrites the conv bucket")
                add(f("sfb_gemm"), t.find("gather_p2", nxt), "WAR next p2 gather rewrites rows the GEMM reads")
                add(f("sfb_gemm"), t.find("gather_dr", nxt), "WAR next dh gather rewrites rows the GEMM reads")
        elif "ar_fc" in labels:  # bucketed all-reduce schedule
            add(f("fc_bwd"), f("ar_fc"), "RAW fc bucket -> all-reduce")
            add(f("ar_fc"), f("opt_fc"), "RAW reduced fc bucket -> fc optimizer")
            add(f("slab_reduce"), f("ar_conv"), "RAW conv bucket -> all-reduce")
            add(f("ar_conv"), f("opt_conv"), "RAW reduced conv bucket -> conv optimizer")
            if nxt is not None:
                add(f("opt_fc"), t.find("fc_fwd", nxt), "RAW updated fc weights -> next fc fwd")
                add(f("ar_fc"), t.find("fc_bwd", nxt), "WAR next fc bwd rewrites the fc bucket")
                add(f("opt_fc"), t.find("fc_bwd", nxt), "WAR next fc bwd rewrites the gradients the optimizer reads")
                add(f("ar_conv"), t.find("slab_reduce", nxt), "WAR next slab reduce rewrites the conv bucket")
        else:  # one GPU: one stream, the plain chain
            chain = [x for x in (f("conv_fwd"), f("fc_fwd"), f("fc_bwd"), f("conv_bwd"), _first(t, opt_any, i))
                     if x is not None]
            for a, b in zip(chain[:-1], chain[1:]):
                add(a, b, "step order")
        if nxt is not None:  # the conv forward reads the conv region, the fc forward the fc region
            add(_first(t, ("opt", "opt_conv"), i), t.find("conv_fwd", nxt), "RAW updated conv weights -> next conv fwd")
            add(_first(t, ("opt", "opt_fc"), i), t.find("fc_fwd", nxt), "RAW updated fc weights -> next fc fwd")
    # ZeRO-1: every shard all-gather follows the optimizer that updated the shard (and the fc1 dX
    # that still read the old bf16 weights), and precedes the next fc forward that reads them
    for p, (lb, st, _) in enumerate(t.tags):
        if lb != "wag":
            continue
        prev_opt = max((q for q, (l2, _, _) in enumerate(t.tags[:p]) if l2 in ("opt", "opt_fc")), default=None)
        prev_dx = max((q for q, (l2, _, _) in enumerate(t.tags[:p]) if l2 == "fc1_dx"), default=None)
        nxt_fc = min((q for q, (l2, _, _) in enumerate(t.tags) if q > p and l2 == "fc_fwd"), default=None)
        add(prev_opt, p, "RAW updated shard -> weight all-gather")
        add(prev_dx, p, "WAR weight all-gather rewrites the bf16 weights fc1 dX read")
        add(p, nxt_fc, "RAW gathered weights -> next fc fwd")
    return req


def violations(t: Topology, collectives=("gather_p2", "gather_dr", "ar_conv", "ar_fc", "wag")) -> List[str]:
    """Human-readable list of every required ordering the DAG does not guarantee (empty = OK), plus
    collective operations whose tag recorded no node (nothing could be checked for them)."""
    out = []
    for lb, st, nodes in t.tags:
        if lb in collectives and not nodes:
            out.append(f"{lb}@{st}: no graph node recorded")
    for a, b, why in required(t):
        la, sa, na = t.tags[a]
        lb, sb, nb = t.tags[b]
        if not t.ordered(na, nb):
            out.append(f"{la}@{sa} -> {lb}@{sb} not ordered ({why})")
    return out
