"""The captured-graph dependency checker (utils/graph_check.py) on synthetic schedules: a small
stream/event simulator emits the same ``node / edge / tag`` text ``MnistEngine.capture_topology``
returns. The full sufficient-factor and all-reduce schedules pass; dropping one cross-stream wait
is reported as exactly the orderings it broke. The same checker runs on the real captured graphs
in tests/test_graph_topology_gpu.py."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tensorflow_distributed_amd.utils.graph_check import Topology, violations  # noqa: E402


class Sim:
    """Stream capture in miniature: an op depends on the previous op of its stream and on every
    event its stream waited for since; record() snapshots a stream's last op into an event."""

    def __init__(self, drop=()):
        self.n, self.last, self.pending, self.ev, self.lines, self.drop = 0, {}, {}, {}, [], set(drop)
        self.step = 0

    def op(self, stream, label):
        i = self.n
        self.n += 1
        self.lines.append(f"node {i} 0")
        deps = set(self.pending.pop(stream, set()))
        if stream in self.last:
            deps.add(self.last[stream])
        for d in sorted(deps):
            self.lines.append(f"edge {d} {i}")
        self.last[stream] = i
        self.lines.append(f"tag {label}@{self.step} {i}")

    def alias(self, label):
        """The last op's node under a second label (MnistEngine::tag_alias: one launch, two jobs)."""
        self.lines.append(f"tag {label}@{self.step} {self.n - 1}")

    def record(self, ev, stream):
        self.ev[ev] = self.last[stream]

    def wait(self, stream, ev, name):
        if name not in self.drop:
            self.pending.setdefault(stream, set()).add(self.ev[ev])


def sfb_schedule(sim, steps=2, zero=False, world=2, merged=False):
    """train_step_sfb_serial's operation/event order (csrc/runtime/mnist_engine.cpp). merged: the slab
    reduce runs inside the SFB GEMM's launch (set_sfb_merge_reduce)."""
    pending_wag = False
    for i in range(steps):
        sim.step = i
        join = i == steps - 1
        if zero and pending_wag and world == 1:
            sim.record("start", "s")
            sim.wait("c", "start", "wag<-opt")
            sim.op("c", "wag")
            sim.record("wag", "c")
        sim.op("s", "conv_fwd")
        sim.record("p2", "s")
        sim.wait("c", "p2", "gather_p2<-conv_fwd")
        sim.op("c", "gather_p2")
        if zero and pending_wag:
            sim.wait("s", "wag", "fc_fwd<-wag")
            pending_wag = False
        sim.op("s", "fc_fwd")
        sim.record("a", "s")
        sim.wait("c", "a", "gather_dr<-fc_fwd")
        sim.op("c", "gather_dr")
        sim.record("ag", "c")
        sim.op("s", "fc1_dx")
        sim.op("s", "conv_bwd")
        if merged:
            sim.wait("s", "ag", "sfb_gemm<-gather_dr")
            sim.op("s", "sfb_gemm")
            sim.alias("slab_reduce")
        else:
            sim.op("s", "slab_reduce")
        sim.record("b", "s")
        sim.wait("c", "b", "ar_conv<-slab_reduce")
        sim.op("c", "ar_conv")
        sim.record("done", "c")
        if not merged:
            sim.wait("s", "ag", "sfb_gemm<-gather_dr")
            sim.op("s", "sfb_gemm")
        if world > 1:
            sim.op("s", "opt_fc")
            if zero:
                sim.record("start", "s")
                sim.wait("c", "start", "wag<-opt_fc")
                sim.op("c", "wag")
                sim.record("wag", "c")
            sim.wait("s", "done", "opt_conv<-ar_conv")
            sim.op("s", "opt_conv")
        else:
            sim.wait("s", "done", "opt<-ar_conv")
            sim.op("s", "opt")
        if zero:
            pending_wag = True
            if join:
                if world == 1:
                    sim.record("start", "s")
                    sim.wait("c", "start", "wag<-opt")
                    sim.op("c", "wag")
                    sim.record("wag", "c")
                sim.wait("s", "wag", "end<-wag")
    return sim.lines


def allreduce_schedule(sim, steps=2):
    """train_step_dp's operation/event order: fc optimizer on its own stream."""
    pending = False
    for i in range(steps):
        sim.step = i
        sim.op("s", "conv_fwd")
        if pending:
            sim.wait("s", "opt_a", "fc_fwd<-opt_fc")
        sim.op("s", "fc_fwd")
        sim.op("s", "fc_bwd")
        sim.record("a", "s")
        sim.wait("c", "a", "ar_fc<-fc_bwd")
        sim.op("c", "ar_fc")
        sim.record("ag", "c")
        sim.wait("o", "ag", "opt_fc<-ar_fc")
        sim.op("o", "opt_fc")
        sim.record("opt_a", "o")
        sim.op("s", "conv_bwd")
        sim.op("s", "slab_reduce")
        sim.record("b", "s")
        sim.wait("c", "b", "ar_conv<-slab_reduce")
        sim.op("c", "ar_conv")
        sim.record("done", "c")
        sim.wait("s", "done", "opt_conv<-ar_conv")
        sim.op("s", "opt_conv")
        pending = i < steps - 1
        if not pending:
            sim.wait("s", "opt_a", "end<-opt_fc")
    return sim.lines


def test_full_schedules_have_no_violations():
    for world in (1, 2):
        for zero in (False, True):
            for merged in (False, True):
                assert violations(Topology(sfb_schedule(Sim(), 3, zero, world, merged))) == [], (world, zero, merged)
    assert violations(Topology(allreduce_schedule(Sim(), 3))) == []


def test_dropped_wait_is_reported():
    v = violations(Topology(sfb_schedule(Sim(drop={"sfb_gemm<-gather_dr"}), 2)))
    assert any(x.startswith("gather_dr@0 -> sfb_gemm@0") for x in v), v
    assert any(x.startswith("gather_dr@1 -> sfb_gemm@1") for x in v), v
    v = violations(Topology(sfb_schedule(Sim(drop={"sfb_gemm<-gather_dr"}), 2, merged=True)))
    assert any(x.startswith("gather_dr@1 -> sfb_gemm@1") for x in v), v
    v = violations(Topology(sfb_schedule(Sim(drop={"opt_conv<-ar_conv"}), 2, world=2, merged=True)))
    assert any(x.startswith("ar_conv@0 -> opt_conv@0") for x in v), v
    v = violations(Topology(sfb_schedule(Sim(drop={"gather_p2<-conv_fwd"}), 2)))
    assert any(x.startswith("conv_fwd@0 -> gather_p2@0") for x in v), v
    v = violations(Topology(sfb_schedule(Sim(drop={"fc_fwd<-wag"}), 3, zero=True, world=2)))
    assert any(x.startswith("wag@0 -> fc_fwd@1") for x in v), v
    v = violations(Topology(allreduce_schedule(Sim(drop={"fc_fwd<-opt_fc"}), 2)))
    assert any(x.startswith("opt_fc@0 -> fc_fwd@1") for x in v), v


def test_empty_collective_tag_is_reported():
    lines = sfb_schedule(Sim(), 1)
    lines = [ln if not ln.startswith("tag gather_p2@0") else "tag gather_p2@0" for ln in lines]
    assert "gather_p2@0: no graph node recorded" in violations(Topology(lines))
