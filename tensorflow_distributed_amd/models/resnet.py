"""ResNet-18 / ResNet-50 (v1.5, NHWC, bf16) on the native HIP kernel library -- the convnet
configs of BASELINE.json (4: synthetic 224x224x3 ResNet-18-style DP=8; 5: synthetic-ImageNet
ResNet-50 bf16 DP=8 with bucketed gradient all-reduce overlapped with backward).

Execution model (MI355X-first, not a framework-module port):

* Every trainable tensor lives in ONE flat fp32 master buffer with a bf16 shadow (the MFMA
  operand) and ONE flat fp32 gradient buffer, laid out in *reverse* forward order, so the backward
  pass fills the gradient buffer front to back and gradient buckets are contiguous ranges.
* Activations flow through ``torch.autograd`` only for bookkeeping; every op is a native kernel
  (``torch.ops.tfd.conv2d_* / bn_* / maxpool2d_* / linear_* / softmax_xent``). Weight gradients
  are written straight into their slice of the flat gradient buffer from inside the backward, and
  each write marks the parameter ready in the :class:`BucketReducer`, which launches that bucket's
  all-reduce on a dedicated communication stream as soon as the bucket is complete (overlap with
  the rest of the backward), exactly the bucket/backward overlap of config 5.
* One fused flat optimizer kernel (SGD-momentum by default, Adam available) updates master +
  shadow. The whole step can be captured into a hipGraph with ``torch.cuda.graph``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

ops = None


# Backward on autograd's device threads (True) or on the caller's thread (False, the library's
# choice: see ResNet.train_step). A module constant, not a switch: tools/debug/memset_resnet_probe.py
# flips it to rebuild the round-5 conditions.
BACKWARD_ON_AUTOGRAD_THREADS = False


def _ops():
    global ops
    if ops is None:
        from .. import _native

        _native.require()
        ops = torch.ops.tfd
    return ops


# ----------------------------------------------------------------------------- parameters
@dataclass
class PSpec:
    name: str
    shape: Tuple[int, ...]
    init: str  # "he" (conv/linear weight), "ones", "zeros"
    fan_in: int = 1
    offset: int = 0

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))


class FlatParams:
    """Flat master/shadow/grad buffers; slots padded to 64 elements (256-B aligned views)."""

    def __init__(self, specs: List[PSpec], device, seed: int = 0):
        self.specs = specs
        off = 0
        for s in reversed(specs):  # reverse forward order == backward production order
            s.offset = off
            off += (s.numel + 63) // 64 * 64
        self.total = off
        self.device = device
        self.master = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        self.momentum = torch.zeros(off, dtype=torch.float32, device=device)
        self.by_name: Dict[str, PSpec] = {s.name: s for s in specs}
        g = torch.Generator(device="cpu").manual_seed(seed)
        for s in specs:
            v = self.view(self.master, s)
            if s.init == "he":
                v.copy_((torch.randn(s.shape, generator=g) * math.sqrt(2.0 / s.fan_in)).to(device))
            elif s.init == "ones":
                v.fill_(1.0)
            else:
                v.zero_()
        self.shadow = self.master.to(torch.bfloat16)

    def view(self, buf: torch.Tensor, s: PSpec) -> torch.Tensor:
        return buf[s.offset:s.offset + s.numel].view(s.shape)

    def w(self, name: str) -> torch.Tensor:  # bf16 operand
        return self.view(self.shadow, self.by_name[name])

    def p(self, name: str) -> torch.Tensor:  # fp32 master
        return self.view(self.master, self.by_name[name])

    def g(self, name: str) -> torch.Tensor:  # fp32 grad slot
        return self.view(self.grad, self.by_name[name])


# ----------------------------------------------------------------------------- bucketed reducer
_EVENT_POOL: Dict[int, List[torch.cuda.Event]] = {}


def _reducer_events(device, n: int) -> List["torch.cuda.Event"]:
    """The first ``n`` events of the device's process-lifetime pool (grown on demand)."""
    idx = torch.device(device).index or 0
    pool = _EVENT_POOL.setdefault(idx, [])
    while len(pool) < n:
        pool.append(torch.cuda.Event())
    return pool[:n]


class BucketReducer:
    """Contiguous gradient buckets of ~``bucket_bytes``; a bucket's all-reduce is launched on the
    comm stream the moment its last parameter gradient has been written (backward overlap)."""

    def __init__(self, fp: FlatParams, comm=None, bucket_bytes: int = 8 << 20, bf16: bool = False,
                 force_dp: bool = False, small=None, small_bytes: int = 0):
        """``force_dp``: run the DP schedule (comm stream, per-bucket bf16 casts and collectives,
        1/N in the optimizer) even when the communicator has ONE rank -- the exact multi-GPU code
        path, rehearsed on a one-GPU box over a real world-1 RcclComm (MnistEngine.set_force_dp's
        analogue). ``small``: a second communicator (the IPC one-shot all-reduce,
        parallel/ipc.IpcCollectives) for buckets of at most ``small_bytes`` wire bytes -- latency-bound
        tails where RCCL's ring pays 2(N-1) link hops for a few hundred KB."""
        self.fp = fp
        self.comm = comm
        self.small = small
        self.small_bytes = small_bytes
        self.world = comm.world() if comm is not None else 1
        dp = comm is not None and (self.world > 1 or force_dp)
        self.buckets: List[Tuple[int, int]] = []
        self.bucket_of: Dict[str, int] = {}
        cur_lo, cur_n = 0, 0
        elt = 2 if (bf16 and dp) else 4  # wire bytes per gradient
        order = list(reversed(fp.specs))  # flat-buffer order
        for s in order:
            if cur_n and (s.offset + s.numel - cur_lo) * elt > bucket_bytes:
                self.buckets.append((cur_lo, s.offset))
                cur_lo, cur_n = s.offset, 0
            self.bucket_of[s.name] = len(self.buckets)
            cur_n += 1
        self.buckets.append((cur_lo, fp.total))
        self.need = [0] * len(self.buckets)
        for s in fp.specs:
            self.need[self.bucket_of[s.name]] += 1
        self.count = [0] * len(self.buckets)
        self.bucket_comm = [small if (small is not None and (hi - lo) * elt <= small_bytes) else comm
                            for lo, hi in self.buckets]
        self.small_buckets = sum(1 for c in self.bucket_comm if c is small and small is not None)
        self.stream = torch.cuda.Stream(fp.device) if dp else None
        # one event per bucket for the compute -> comm stream hand-off, from a per-device pool (no event
        # objects created or freed per reducer / per step; the host-heap corruption they were once
        # suspected of was the autograd-thread issuance fixed in mark_ready)
        ev = _reducer_events(fp.device, len(self.buckets) + 1) if dp else [None]
        self.bucket_events, self.join_event = ev[:-1], ev[-1]
        self.events = []
        self.ready: List[int] = []  # buckets whose ready event is recorded, collective not yet issued
        self.launched = 0
        # bf16 wire format halves the all-reduce bytes; the optimizer reads the bf16 sums directly
        self.bf16 = bf16 and self.stream is not None
        self.gbf = torch.empty(fp.total, dtype=torch.bfloat16, device=fp.device) if self.bf16 else None

    def reset(self):
        self.count = [0] * len(self.buckets)
        self.events = []
        self.ready = []
        self.launched = 0

    def mark_ready(self, name: str):
        """Called from inside backward (ResNet.train_step runs it on the caller's thread): a bucket
        whose last gradient just landed only records its ready event on the compute stream -- the
        point its collective will wait for. The side-stream work itself is issued by finish().

        Issuing it here instead (stream switch, wait, collective launch on the autograd thread)
        corrupted the host heap once a CUDA graph captured over it was destroyed: glibc aborts
        ("free(): invalid pointer", segfaults) within 1-30 capture / replay / destroy cycles, with
        the IPC collective, RCCL or a plain torch-op stand-in alike, never with the hand-offs issued
        from the main thread (80 cycles each) nor without the side stream; a torch-only twin issuing
        the same stream/event pattern from the main thread was clean too (tools/debug/heap_twin.py,
        tools/debug/rn_configure_loop.py, profiles/heap_bisect_r5.log). The overlap is unchanged:
        the collective still waits only for its bucket's event, recorded at the same point of the
        backward."""
        b = self.bucket_of[name]
        self.count[b] += 1
        if self.count[b] == self.need[b] and self.stream is not None:
            self.bucket_events[b].record(torch.cuda.current_stream(self.fp.device))
            self.ready.append(b)

    def _launch(self, b: int):
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(self.bucket_events[b])
            lo, hi = self.buckets[b]
            c = self.bucket_comm[b]
            if self.bf16 and hasattr(c, "all_reduce_into"):
                # the IPC one-shot reads the fp32 gradients and writes the bf16 sums: no cast pass
                c.all_reduce_into(self.fp.grad[lo:hi], self.gbf[lo:hi], "sum")
            elif self.bf16:
                self.gbf[lo:hi].copy_(self.fp.grad[lo:hi])
                c.all_reduce(self.gbf[lo:hi], "sum")
            else:
                c.all_reduce(self.fp.grad[lo:hi], "sum")
        self.launched += 1

    def finish(self):
        """After backward, on the caller's thread: every ready bucket's collective on the comm stream (in
        readiness order, each behind its own event), then the join back into the compute stream."""
        if self.stream is not None:
            for b in self.ready:
                self._launch(b)
            self.ready = []
            ev = self.join_event  # from the pool too (wait_stream makes a temporary one)
            ev.record(self.stream)
            torch.cuda.current_stream(self.fp.device).wait_event(ev)

    def reduced_grads(self) -> torch.Tensor:
        return self.gbf if self.bf16 else self.fp.grad


# ----------------------------------------------------------------------------- autograd ops
# GradJoin defers a first-arriving conv whose dgrad can carry the BN-backward statistics (13.335 ->
# 13.25 ms, profiles/resnet50_join_defer_ab_r4.log); False = compute it at once -- the oracle form the
# tests and tools/debug/bn_bwd_stats_rel.py compare against (module attribute, not a run-time switch)
_JOIN_DEFER = True
# a 1x1 stride-2 shortcut dgrad stays on its own grid, added at the even pixels by the joining dgrad's
# epilogue (13.12 -> 13.04 ms, profiles/resnet50_shortcut_sub2_ab_r4.log); False = the full-grid
# dgrad with its zero phases written -- test_stride2_shortcut_gradient_on_its_own_grid's oracle
_JOIN_SUB2 = True


class GradJoin:
    """Sum of the gradients that reach one activation over several paths (a residual block's input
    feeds the first conv and the shortcut), without autograd's separate elementwise add: the
    first path to run parks its gradient here and hands autograd ``None``; the last one adds
    the parked tensor -- a conv adds it in its dgrad epilogue (``conv2d_dgrad(acc=...)``), so the sum
    costs no extra pass over the activation. Works for either execution order of the paths.

    On by default (``ResNet(fuse_joins=True)``). With the round-1 fragment-order epilogue the
    add's scalar bf16 loads serialised on memory latency (pointwise dgrad 77 -> 277 us, so it was
    off); the LDS-staged epilogue (csrc/kernels/conv_nhwc.hip ``lds_epilogue``) issues the add
    tile as 16-B loads before staging the accumulator and stores whole lines: ResNet-50 b128
    16.81 -> 16.28 ms/step on one MI355X (profiles/resnet50_epi_ab_r2.log)."""

    def __init__(self, n: int):
        self.n = n
        self.bn = None  # the batch norm whose output is the joined activation (its dout is the sum)
        self.reset()

    def reset(self):
        self.seen, self.acc, self.bits, self.deferred = 0, None, None, None
        self.sub = None  # full [N, H, W, C] when acc is a stride-2 shortcut dgrad on its own grid

    @staticmethod
    def _sub2(L) -> bool:
        """A 1x1 stride-2 unpadded conv: its dgrad is nonzero at the even pixels only."""
        return _JOIN_SUB2 and L.k == 1 and L.stride == 2 and L.pad == 0

    def _expand(self):
        """Materialise a parked stride-2 gradient on the full grid (an unusual arrival order)."""
        if self.sub is not None:
            full = torch.zeros(self.sub, dtype=self.acc.dtype, device=self.acc.device)
            full[:, ::2, ::2, :] = self.acc
            self.acc, self.sub = full, None

    @staticmethod
    def _unmask(dout, bits):
        """dout through the relu bits, as a tensor (the masked operand's explicit form)."""
        C = dout.shape[-1]
        keep = ((bits.view(-1, C // 8).unsqueeze(-1) >> torch.arange(8, device=bits.device, dtype=torch.uint8)) & 1)
        return dout * keep.reshape(dout.shape).to(dout.dtype)

    def _add(self, g):
        if self.acc is None:
            self.acc = g
            return
        self._expand()
        if self.bits is not None:  # a parked masked gradient meets a plain one: materialise it
            self.acc, self.bits = self._unmask(self.acc, self.bits), None
        self.acc = self.acc.add_(g)

    def _conv_into_acc(self, dy, L, xs, fid, fuse):
        """acc <- this conv's dgrad (+ acc): with the BN statistics in its epilogue when ``fuse``; a
        stride-2 parked acc rides the epilogue (every phase of a strided dgrad maps its rows to the
        full grid, so the odd pixels simply get no add)."""
        bits, self.bits = self.bits, None
        sub2 = self.sub is not None
        if fuse:
            self.acc = _dgrad_bn(dy, L, xs, self.acc, self.bn, fid, bits, sub2)
        elif self.acc is not None:
            self.acc = _ops().conv2d_dgrad(dy, L.w(), xs, L.stride, L.pad, self.acc, bits, sub2)
        elif self._sub2(L):  # nothing to add yet: the shortcut dgrad on its own grid, parked
            N, H, W, C = xs
            self.acc = _ops().conv2d_dgrad(dy, L.w(), [N, (H + 1) // 2, (W + 1) // 2, C], 1, 0)
            self.sub = list(xs)
            return
        else:
            self.acc = _ops().conv2d_dgrad(dy, L.w(), xs, L.stride, L.pad)
        self.sub = None

    def arrive(self, g=None, conv=None, masked=None):
        """``g``: a finished gradient; ``conv=(dy, layer, xshape, fwd_id)``: compute it as a dgrad;
        ``masked=(dout, relu_bits)``: the residual BN's gradient through its relu, never materialised
        -- a conv arriving after it adds dout masked by the bits in its dgrad epilogue
        (``acc_bits``), the dres write the BN backward skipped. Returns the total for the last
        arrival, else None.

        A conv whose dgrad can carry the BN-backward statistics (``_bn_stats_fusable``) arriving
        first is deferred and run last, after the other arrival: then its epilogue sees the whole
        dout and the BN backward needs no partial pass -- whichever order autograd delivers the two
        paths in (a downsample block's strided 1x1 shortcut dgrad, which cannot carry them, used to
        arrive last at 4 joins per ResNet-50 step)."""
        self.seen += 1
        last = self.seen == self.n
        if (_JOIN_DEFER and not last and conv is not None and self.deferred is None and self.acc is None
                and _bn_stats_fusable(conv[1], self.bn, conv[3])):
            self.deferred = conv
            return None
        fuse_now = last and self.deferred is None
        # fold this arrival into (acc, bits)
        if masked is not None:
            if self.acc is None and (not last or self.deferred is not None):
                self.acc, self.bits = masked  # consumed by a later (or the deferred) dgrad's epilogue
            else:
                self._add(self._unmask(*masked))
        elif conv is not None:
            dy, L, xs, fid = conv
            # the sum is the BN's whole dout when this is the last arrival
            self._conv_into_acc(dy, L, xs, fid, fuse_now and _bn_stats_fusable(L, self.bn, fid))
        elif g is not None:
            self._add(g)
        if not last:
            return None
        if self.deferred is not None:  # the deferred conv last: its epilogue sums the statistics
            dy, L, xs, fid = self.deferred
            self._conv_into_acc(dy, L, xs, fid, True)
        self._expand()
        out = self.acc if self.bits is None else self._unmask(self.acc, self.bits)
        self.acc, self.bits, self.deferred, self.sub = None, None, None, None
        return out


# strided (phase) dgrads carry BN-backward statistics too (profiles/resnet50_bn_stats_strided_ab_r3.log)
_BN_STATS_STRIDED = True


def _bn_stats_fusable(L, bn, fid) -> bool:
    """Can conv ``L``'s dgrad (the whole dout of batch norm ``bn``) emit that BN's backward
    statistics partials (``conv2d_dgrad_bn``)? Stride-1 dgrads and strided ones whose output phases all
    have taps (3x3 stride 2, by phase GEMMs), and a BN whose relu mask the epilogue
    can form the way the BN backward will: none, relu bits (residual BN), or recomputed from y
    (residual-free BN with ``mask_from_y``)."""
    if bn is None or not L.model.bn_bwd_stats or bn.fwd_state is None:
        return False
    if bn.fwd_state[6] != fid:  # the BN state is another forward's (a second forward before this backward)
        return False
    if L.stride != 1 and (L.k < L.stride or not _BN_STATS_STRIDED):  # tap-less phases (1x1 stride 2)
        return False
    _, _, _, mask, relu, has_res, _ = bn.fwd_state
    return (not relu) or mask is not None or (not has_res and L.model.mask_from_y)


def _dgrad_bn(dy, L, xs, acc, bn, fid, acc_bits=None, acc_sub2=False):
    """dX of conv ``L`` (+ ``acc``) with BN ``bn``'s backward partials summed in the same epilogue;
    the partials wait on the BN layer for its backward (which then skips its own partial pass),
    tagged with the forward they belong to."""
    y, mean, invstd, mask, relu, has_res, _ = bn.fwd_state
    beta = bn.beta() if (relu and mask is None) else None
    g, part = _ops().conv2d_dgrad_bn(dy, L.w(), xs, L.stride, L.pad, acc, y, mean, invstd, bn.gamma(), beta, mask,
                                     relu, acc_bits, part_out=bn.acc_b, acc_sub2=acc_sub2)
    bn.bwd_part = (part, fid)
    return g


class _Conv(torch.autograd.Function):
    # `token` is a 0-d tensor that requires grad: weights are not autograd leaves (their gradients
    # go straight into the flat buffer), so the stem needs it to put the graph on the tape.
    # With layer.model.bn_stats the conv also returns the batch-norm statistics partials of its
    # output ([row blocks, 2, K], summed in the GEMM epilogue), which the following BN consumes.
    @staticmethod
    def forward(ctx, x, token, layer):
        ctx.layer = layer
        ctx.fwd_id = layer.model.fwd_id
        ctx.save_for_backward(x)
        if layer.model.bn_stats:
            y, part = _ops().conv2d_fwd_stats(x, layer.w(), layer.stride, layer.pad, part_out=layer.acc)
            ctx.mark_non_differentiable(part)
            ctx.set_materialize_grads(False)  # no zero-filled gradient for `part` in the backward
            return y, part
        return _ops().conv2d_fwd(x, layer.w(), layer.stride, layer.pad)

    @staticmethod
    def backward(ctx, dy, *_dpart):
        (x,) = ctx.saved_tensors
        L = ctx.layer
        dy = dy.contiguous()
        _ops().conv2d_wgrad(x, dy, L.g(), L.stride, L.pad, L.model.grads_zeroed)
        L.model.reducer.mark_ready(L.name)
        dx = None
        if ctx.needs_input_grad[0]:
            if L.in_join is not None:
                dx = L.in_join.arrive(conv=(dy, L, list(x.shape), ctx.fwd_id))
            elif _bn_stats_fusable(L, L.in_bn, ctx.fwd_id):  # this conv is the BN output's only consumer
                dx = _dgrad_bn(dy, L, list(x.shape), None, L.in_bn, ctx.fwd_id)
            else:
                dx = _ops().conv2d_dgrad(dy, L.w(), list(x.shape), L.stride, L.pad)
        return dx, None, None


def pair_stem_weight(w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[R, S, 8, K] stem filter (3 real input channels, S odd, pad 3) -> the width-paired filter
    [R, (S + 1) // 2, 8, K] of ``conv2d_fwd_stats_w2``: channel p*3 + c of column s' is the original tap
    s = 2s' + p - 1 (tap -1 is zero), channels 6-7 zero. ``out``: a buffer of that shape whose
    never-written entries (tap -1, channels 6-7) are already zero -- two copies, no allocation."""
    R, S, _, K = w.shape
    if out is None:
        out = torch.zeros(R, (S + 1) // 2, 8, K, device=w.device, dtype=w.dtype)
    out[:, 1:, 0:3].copy_(w[:, 1::2, :3])  # p = 0: taps 1, 3, 5 (column 0 is tap -1)
    out[:, :, 3:6].copy_(w[:, 0::2, :3])  # p = 1: taps 0, 2, 4, 6
    return out


def unpair_stem_grad(dwp: torch.Tensor, dw: torch.Tensor) -> None:
    """Write the width-paired filter gradient ``dwp`` [R, S', 8, K] into ``dw`` [R, 2S' - 1, 8, K]
    (inverse map of ``pair_stem_weight``; the padded input channels 3-7 get zero gradient)."""
    dw[:, 1::2, :3].copy_(dwp[:, 1:, 0:3])
    dw[:, 0::2, :3].copy_(dwp[:, :, 3:6])
    dw[:, :, 3:].zero_()


class _StemW2(torch.autograd.Function):
    """The stem conv (7x7, stride 2, pad 3 over 3 channels) on width-paired input pixels
    (``stem_pack``): the paired filter covers two input columns per 8-channel chunk, so the implicit
    GEMM runs 7 x 4 x 8 = 224 MACs per output element instead of 7 x 7 x 8 = 392 over the channel-padded
    input, and the packed input is half the bytes of the padded one. The weights and their gradient
    stay in the [7, 7, 8, K] layout of ``ConvLayer`` (checkpoints, optimizer); ``evaluate`` keeps the
    padded form. Same BN-statistics epilogue as ``_Conv``."""

    @staticmethod
    def forward(ctx, xp, token, layer):
        ctx.layer = layer
        ctx.save_for_backward(xp)
        if layer.paired_w is None:  # eager warm-up steps allocate, captured steps reuse
            R, S, C, K = layer.w().shape
            layer.paired_w = torch.zeros(R, (S + 1) // 2, C, K, device=xp.device, dtype=layer.w().dtype)
            layer.paired_g = torch.zeros(R, (S + 1) // 2, C, K, device=xp.device, dtype=torch.float32)
        y, part = _ops().conv2d_fwd_stats_w2(xp, pair_stem_weight(layer.w(), layer.paired_w), layer.stride, layer.pad,
                                             part_out=layer.acc)
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, dy, *_dpart):
        (xp,) = ctx.saved_tensors
        L = ctx.layer
        _ops().conv2d_wgrad_w2(xp, dy.contiguous(), L.paired_g, L.stride, L.pad, False)
        unpair_stem_grad(L.paired_g, L.g())
        L.model.reducer.mark_ready(L.name)
        return None, None, None


def _take_bwd_part(bn, fid):
    """The BN-backward partials a dgrad epilogue left for ``bn`` -- only if they belong to the
    forward ``fid`` (else None: bn_bwd runs its own partial pass). Clears the layer's state when it
    is this forward's (its consumers' dgrads have run)."""
    tagged, bn.bwd_part = bn.bwd_part, None
    if bn.fwd_state is not None and bn.fwd_state[6] == fid:
        bn.fwd_state = None
    return tagged[0] if tagged is not None and tagged[1] == fid else None


class _BNReluConv(torch.autograd.Function):
    """relu(bn(y)) -> conv with the batch norm applied by the conv's operand loader (the forward BN
    fold, ``conv2d_fwd(..., mean, invstd, gamma, beta)``): the normalised activation is never written.
    The BN here is a residual-free relu BN whose output has this conv as its only consumer (a
    bottleneck's bn1 -> conv2 and bn2 -> conv3, a basic block's bn1 -> conv2). Its statistics come
    from the producing conv's epilogue partials (``bn_stats``: the finalize only, no apply pass); the
    backward rebuilds the conv's X operand the same way in the weight-gradient loader, takes the
    BN-backward partials from the dgrad epilogue (relu mask recomputed from y) and runs the BN
    backward -- the unfused _BN + _Conv pair, minus one full read + write of the activation per BN.
    Bit-identical forward (same bn_affine constants, same fmaf + relu + rounding)."""

    @staticmethod
    def forward(ctx, y, token, part, bn, conv):
        o = _ops()
        mean, invstd = o.bn_stats(y, part, bn.rmean, bn.rvar, bn.momentum, bn.eps)
        fid = conv.model.fwd_id
        bn.fwd_state = (y, mean, invstd, None, True, False, fid)
        ctx.bn, ctx.conv, ctx.fwd_id = bn, conv, fid
        ctx.save_for_backward(y, mean, invstd)
        act = (mean, invstd, bn.gamma(), bn.beta())
        if conv.model.bn_stats:
            out, p2 = o.conv2d_fwd_stats(y, conv.w(), conv.stride, conv.pad, *act, part_out=conv.acc)
            ctx.mark_non_differentiable(p2)
            ctx.set_materialize_grads(False)
            return out, p2
        return o.conv2d_fwd(y, conv.w(), conv.stride, conv.pad, *act)

    @staticmethod
    def backward(ctx, dout, *_dpart):
        y, mean, invstd = ctx.saved_tensors
        bn, L = ctx.bn, ctx.conv
        o = _ops()
        dout = dout.contiguous()
        o.conv2d_wgrad(y, dout, L.g(), L.stride, L.pad, L.model.grads_zeroed, mean, invstd, bn.gamma(), bn.beta())
        L.model.reducer.mark_ready(L.name)
        if _bn_stats_fusable(L, bn, ctx.fwd_id):  # the BN output's gradient + its backward statistics partials
            dbn = _dgrad_bn(dout, L, list(y.shape), None, bn, ctx.fwd_id)
        else:
            dbn = o.conv2d_dgrad(dout, L.w(), list(y.shape), L.stride, L.pad)
        part = _take_bwd_part(bn, ctx.fwd_id)
        # relu mask recomputed from y (beta given); `out` is never read
        dy, _ = o.bn_bwd(dbn, y, y, bn.gamma(), mean, invstd, True, False, bn.g_gamma(), bn.g_beta(), bn.beta(), None,
                         part)
        L.model.reducer.mark_ready(bn.name + "/gamma")
        L.model.reducer.mark_ready(bn.name + "/beta")
        return dy, None, None, None, None


_FOLD_MAX_C = None


def _fold_max_c() -> int:
    global _FOLD_MAX_C
    if _FOLD_MAX_C is None:
        _FOLD_MAX_C = int(_ops().bn_relu_max_channels())
    return _FOLD_MAX_C


class _BN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, res, layer, relu, part=None):
        args = (y, layer.gamma(), layer.beta(), res, relu, layer.rmean, layer.rvar, layer.momentum, layer.eps)
        # residual + relu: the relu mask cannot be recomputed from y; keep it as bits (1/16 of `out`)
        # so the backward never re-reads the block output
        mask = None
        if relu and res is not None and layer.model.relu_bits:
            mask = torch.empty(y.numel() // y.shape[-1], y.shape[-1] // 8, dtype=torch.uint8, device=y.device)
        out, mean, invstd = _ops().bn_fwd(*args, part, mask)
        ctx.layer, ctx.relu, ctx.has_res = layer, relu, res is not None
        ctx.fwd_id = layer.model.fwd_id
        # for the consuming conv's dgrad epilogue (conv2d_dgrad_bn): this forward's state, tagged
        layer.fwd_state = (y, mean, invstd, mask, relu, res is not None, ctx.fwd_id)
        ctx.save_for_backward(y, out if mask is None else mask, mean, invstd)
        ctx.bits = mask is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        y, out_or_mask, mean, invstd = ctx.saved_tensors
        L = ctx.layer
        # residual-free BN: pass beta, the kernels recompute the relu mask from y (no read of out);
        # residual BN: the forward's relu bits (no read of out either)
        beta = L.beta() if (ctx.relu and not ctx.has_res and L.model.mask_from_y) else None
        mask = out_or_mask if ctx.bits else None
        out = y if ctx.bits else out_or_mask  # not read when a mask (bits or from y) is given
        dout = dout.contiguous()
        # identity shortcut with relu bits: the join's conv adds dout masked by the bits in its dgrad
        # epilogue, so the residual gradient is never written (GradJoin.arrive(masked=...))
        masked = ctx.has_res and L.res_join is not None and mask is not None and L.model.masked_join
        args = (dout, out, y, L.gamma(), mean, invstd, ctx.relu, ctx.has_res and not masked, L.g_gamma(), L.g_beta())
        part = _take_bwd_part(L, ctx.fwd_id)  # partials from the dgrad that produced dout, if it made them
        dy, dres = _ops().bn_bwd(*args, beta, mask, part)
        L.model.reducer.mark_ready(L.name + "/gamma")
        L.model.reducer.mark_ready(L.name + "/beta")
        if masked:
            dres = L.res_join.arrive(masked=(dout, mask))
        elif ctx.has_res and L.res_join is not None:
            dres = L.res_join.arrive(dres)
        return dy, (dres if ctx.has_res else None), None, None, None


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, st, pad):
        y, am = _ops().maxpool2d_fwd(x, k, st, pad)
        ctx.save_for_backward(am)
        ctx.cfg = (list(x.shape), k, st, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (am,) = ctx.saved_tensors
        xs, k, st, pad = ctx.cfg
        return _ops().maxpool2d_bwd(dy.contiguous(), am, xs, k, st, pad), None, None, None


class _BNReluMaxPool(torch.autograd.Function):
    """The stem's relu(bn(y)) -> max pool in one pass (``bn_relu_maxpool``): the BN output, the
    largest activation of the network, is never written nor read back. Same output and argmax as
    _BN + _MaxPool bit for bit. The backward is theirs (maxpool2d_bwd, then bn_bwd with the relu mask
    recomputed from y; folding the statistics into the pool's backward measured no faster,
    csrc/kernels/norm.hip maxpool2_bwd_kernel)."""

    @staticmethod
    def forward(ctx, y, part, bn, k, st, pad):
        o = _ops()
        out, am, mean, invstd = o.bn_relu_maxpool(y, bn.gamma(), bn.beta(), bn.rmean, bn.rvar, bn.momentum, bn.eps, part,
                                                  k, st, pad)
        ctx.bn, ctx.cfg = bn, (list(y.shape), k, st, pad)
        ctx.save_for_backward(y, mean, invstd, am)
        ctx.mark_non_differentiable(am)
        return out

    @staticmethod
    def backward(ctx, dout):
        y, mean, invstd, am = ctx.saved_tensors
        bn = ctx.bn
        xs, k, st, pad = ctx.cfg
        o = _ops()
        dpre = o.maxpool2d_bwd(dout.contiguous(), am, xs, k, st, pad)
        dy, _ = o.bn_bwd(dpre, y, y, bn.gamma(), mean, invstd, True, False, bn.g_gamma(), bn.g_beta(), bn.beta(), None,
                         None)
        bn.model.reducer.mark_ready(bn.name + "/gamma")
        bn.model.reducer.mark_ready(bn.name + "/beta")
        return dy, None, None, None, None, None


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.xs = list(x.shape)
        return _ops().avgpool_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return _ops().avgpool_bwd(dy.contiguous(), ctx.xs)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, layer):
        ctx.layer = layer
        ctx.save_for_backward(x)
        return _ops().linear_fwd(x, layer.w(), layer.bias())

    @staticmethod
    def backward(ctx, dlogits):
        (x,) = ctx.saved_tensors
        L = ctx.layer
        dl = dlogits.to(torch.bfloat16).contiguous()
        _ops().linear_wgrad(x, dl, L.g())
        torch.sum(dlogits.float(), 0, out=L.g_bias())
        L.model.reducer.mark_ready(L.name)
        L.model.reducer.mark_ready(L.name + "/bias")
        return _ops().linear_dgrad(dl, L.w()), None


class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        loss_rows, correct, dl = _ops().softmax_xent(logits.contiguous(), labels)
        ctx.save_for_backward(dl)
        ctx.mark_non_differentiable(correct)
        return loss_rows.mean(), correct

    @staticmethod
    def backward(ctx, dloss, _dcorrect):
        (dl,) = ctx.saved_tensors
        return dl.float() * dloss, None  # dl already carries the 1/N of the mean


class StatArena:
    """Batch-norm statistics slots in slot mode (``bn_part_slots() = S > 0``, csrc/conv_kernels.h):
    the producer epilogues of BN statistics -- a conv's forward epilogue (``conv2d_fwd_stats``) and a
    dgrad's BN-backward epilogue (``conv2d_dgrad_bn``) -- add their tiles' column sums into an
    [S, 2, C] buffer with fp32 atomics, and the BN apply pass finalizes inline: no bn_final launch
    between them. The buffers must start at zero, so they are slices of one arena zeroed once per
    forward (one fill) instead of a fill per buffer. Each slice has one producer per forward /
    backward (a conv's output slots; the slots of the dgrad producing a BN's dout), so a second forward
    before a backward (whose BN states are refused, see _bn_stats_fusable) cannot mix sums. BNs
    without such a producer keep bn_fwd / bn_bwd's own partial pass (row layout + bn_final).
    S = 0 (row mode): no arena, the ops allocate per-tile partial rows that bn_final reduces."""

    def __init__(self, model):
        self.slots = int(_ops().bn_part_slots())
        self.buf = None
        if not self.slots:
            return
        S = self.slots
        layout = []  # (owner, attr, C)
        for L in model.convs:
            layout.append((L, "acc", L.cout))
        for bn in model.bns:
            layout.append((bn, "acc_b", bn.c))
        sizes = [(S * 2 * c + 63) // 64 * 64 for _, _, c in layout]  # 256-B aligned slices
        self.buf = torch.zeros(sum(sizes), dtype=torch.float32, device=model.device)
        off = 0
        for (owner, attr, c), n in zip(layout, sizes):
            setattr(owner, attr, self.buf[off:off + S * 2 * c].view(S, 2, c))
            off += n

    def zero(self):
        if self.buf is not None:
            self.buf.zero_()


# ----------------------------------------------------------------------------- layers
class ConvLayer:
    def __init__(self, model, name, cin, cout, k, stride, pad):
        self.model, self.name, self.stride, self.pad, self.k, self.cout = model, name, stride, pad, k, cout
        self.acc = None  # statistics-partials slots of this conv's output (StatArena), None: row mode
        self.in_join = None  # GradJoin of this conv's input (residual block inputs)
        self.in_bn = None  # the BN whose output is this conv's only input consumer (BN-backward stats)
        self.paired_w = self.paired_g = None  # the width-paired stem's filter / gradient buffers (_StemW2)
        model.specs.append(PSpec(name, (k, k, cin, cout), "he", fan_in=k * k * cin))
        model.convs.append(self)

    def w(self):
        return self.model.fp.w(self.name)

    def g(self):
        return self.model.fp.g(self.name)

    def __call__(self, x):
        return _Conv.apply(x, self.model.token, self)

    def after_bn(self, bn, yp):
        """This conv applied to relu(bn(y)) where ``yp`` is the (y, partials) pair of the producing
        conv: folded when the model allows it (ResNet(fold_bn=True)), else bn then conv."""
        m = self.model
        scope = int(m.fold_bn)  # 0 off, 1 every eligible conv, 2 1x1 consumers only
        if scope and (scope != 2 or self.k == 1) and m.mask_from_y and isinstance(yp, tuple) and bn.c <= _fold_max_c():
            y, part = yp
            return _BNReluConv.apply(y, m.token, part, bn, self)
        return self(bn(yp))


class BNLayer:
    def __init__(self, model, name, c, zero_init=False):
        self.model, self.name, self.c = model, name, c
        self.momentum, self.eps = 0.9, 1e-5
        self.res_join = None  # GradJoin of the residual input (identity shortcut)
        self.fwd_state = None  # (y, mean, invstd, relu bits, relu, has_res, fwd_id) of the latest forward
        self.bwd_part = None  # (partials, fwd_id) left by the dgrad that produced dout
        # statistics-partials slots of the dgrad epilogue that produces this BN's dout (StatArena)
        self.acc_b = None
        model.specs.append(PSpec(name + "/gamma", (c,), "zeros" if zero_init else "ones"))
        model.specs.append(PSpec(name + "/beta", (c,), "zeros"))
        model.bns.append(self)

    def gamma(self):
        return self.model.fp.p(self.name + "/gamma")

    def beta(self):
        return self.model.fp.p(self.name + "/beta")

    def g_gamma(self):
        return self.model.fp.g(self.name + "/gamma")

    def g_beta(self):
        return self.model.fp.g(self.name + "/beta")

    def __call__(self, y, relu=True, res=None):
        part = None
        if isinstance(y, tuple):  # (conv output, its statistics partials) from a stats conv
            y, part = y
        return _BN.apply(y, res, self, relu, part)


class LinearLayer:
    def __init__(self, model, name, cin, cout):
        self.model, self.name = model, name
        model.specs.append(PSpec(name, (cin, cout), "he", fan_in=cin))
        model.specs.append(PSpec(name + "/bias", (cout,), "zeros"))

    def w(self):
        return self.model.fp.w(self.name)

    def bias(self):
        return self.model.fp.p(self.name + "/bias")

    def g(self):
        return self.model.fp.g(self.name)

    def g_bias(self):
        return self.model.fp.g(self.name + "/bias")

    def __call__(self, x):
        return _Linear.apply(x, self)


# ----------------------------------------------------------------------------- model
class ResNet:
    """ResNet-{18,34,50,101} v1.5, NHWC, input fp32 [N,H,W,3] (padded to 8 channels on device)."""

    CFG = {18: ("basic", [2, 2, 2, 2]), 34: ("basic", [3, 4, 6, 3]), 50: ("bottleneck", [3, 4, 6, 3]),
           101: ("bottleneck", [3, 4, 23, 3])}

    def __init__(self, depth: int = 50, num_classes: int = 1000, device=None, seed: int = 0, width: int = 64,
                 zero_init_residual: bool = True, fuse_joins: bool = True, bn_stats: bool = True,
                 bn_bwd_stats: bool = True, fold_bn: int = 0, stem_w2: bool = True):
        kind, blocks = self.CFG[depth]
        if num_classes % 8 or width % 8:
            raise ValueError("num_classes and width must be multiples of 8 (16-byte MFMA operand chunks)")
        self.depth, self.kind, self.num_classes = depth, kind, num_classes
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.specs: List[PSpec] = []
        self.bns: List[BNLayer] = []
        self.convs: List[ConvLayer] = []
        self.stem = ConvLayer(self, "conv1", 8, width, 7, 2, 3)
        self.stem_bn = BNLayer(self, "bn1", width)
        self.blocks = []
        self.joins: List[GradJoin] = []
        self.grads_zeroed = False  # set by train_step: the flat grad buffer was zeroed this step
        self.fuse_joins = fuse_joins
        # BN statistics summed in the producing conv's epilogue (conv2d_fwd_stats) instead of a
        # separate read pass over every conv output
        self.bn_stats = bn_stats
        # BN-backward statistics summed in the epilogue of the dgrad that produces the BN's dout
        # (conv2d_dgrad_bn) instead of bn_bwd's separate read pass over dout and y
        self.bn_bwd_stats = bn_bwd_stats
        # residual-free BN backward recomputes its relu mask from y instead of reading the output
        self.mask_from_y = True
        # residual BN keeps its relu mask as bits for the backward instead of re-reading the output
        self.relu_bits = True
        # 1: single-consumer relu BNs applied inside the consuming conv's operand loader (_BNReluConv);
        # 2: only into 1x1 consumers (a 3x3 consumer's im2col loader re-applies the transform to every
        # input element 9 times); 0 (default): the separate bn_apply pass -- measured no slower than
        # either fold on ResNet-50 b128 (13.79 vs 14.15 / 13.83 ms, profiles/resnet50_bn_fold_ab_r4.log)
        self.fold_bn = int(fold_bn)
        # identity-shortcut gradient as (dout, relu bits) added in the joining conv's dgrad epilogue
        # instead of a dres tensor written by the residual BN's backward (GradJoin.arrive(masked=))
        self.masked_join = True
        # the stem's bn + relu + max pool as one pass (_BNReluMaxPool): its BN output is never written
        self.fuse_stem_pool = True
        # the stem conv on width-paired input pixels (_StemW2): 7 x 4 x 8 instead of 7 x 7 x 8 MACs per output
        self.stem_w2 = bool(stem_w2)
        cin = width
        exp = 4 if kind == "bottleneck" else 1
        prev_out_bn = None  # the BN that produced the current block input (None: the stem's maxpool)
        for li, nb in enumerate(blocks):
            w = width * (2 ** li)
            for bi in range(nb):
                st = 2 if (bi == 0 and li > 0) else 1
                nm = f"layer{li + 1}.{bi}"
                blk = {}
                if kind == "basic":
                    blk["c1"], blk["b1"] = ConvLayer(self, nm + ".conv1", cin, w, 3, st, 1), BNLayer(self, nm + ".bn1", w)
                    blk["c2"], blk["b2"] = ConvLayer(self, nm + ".conv2", w, w, 3, 1, 1), BNLayer(self, nm + ".bn2", w, zero_init_residual)
                    cout = w
                else:
                    blk["c1"], blk["b1"] = ConvLayer(self, nm + ".conv1", cin, w, 1, 1, 0), BNLayer(self, nm + ".bn1", w)
                    blk["c2"], blk["b2"] = ConvLayer(self, nm + ".conv2", w, w, 3, st, 1), BNLayer(self, nm + ".bn2", w)
                    blk["c3"], blk["b3"] = (ConvLayer(self, nm + ".conv3", w, w * exp, 1, 1, 0),
                                            BNLayer(self, nm + ".bn3", w * exp, zero_init_residual))
                    cout = w * exp
                if st != 1 or cin != cout:
                    blk["cd"] = ConvLayer(self, nm + ".downsample", cin, cout, 1, st, 0)
                    blk["bd"] = BNLayer(self, nm + ".downsample_bn", cout)
                blk["c2"].in_bn = blk["b1"]
                if kind != "basic":
                    blk["c3"].in_bn = blk["b2"]
                # the block input feeds conv1 and the shortcut: join their gradients in place
                j = GradJoin(2)
                j.bn = prev_out_bn
                if not fuse_joins:
                    j = None
                blk["c1"].in_join = j
                if "cd" in blk:
                    blk["cd"].in_join = j
                else:
                    blk["b2" if kind == "basic" else "b3"].res_join = j
                if j is not None:
                    self.joins.append(j)
                self.blocks.append(blk)
                prev_out_bn = blk["b2" if kind == "basic" else "b3"]
                cin = cout
        self.fc = LinearLayer(self, "fc", cin, num_classes)
        self.fp = FlatParams(self.specs, self.device, seed)
        for bn in self.bns:
            bn.rmean = torch.zeros(bn.c, device=self.device)
            bn.rvar = torch.ones(bn.c, device=self.device)
        self.reducer = BucketReducer(self.fp)
        self.stats = StatArena(self)
        self.token = torch.zeros((), device=self.device, requires_grad=True)
        self.fwd_id = 0

    @property
    def num_params(self) -> int:
        return sum(s.numel for s in self.specs)

    def set_comm(self, comm, bucket_mb: float = 8.0, bf16_grads: bool = True, force_dp: bool = False, small=None,
                 small_mb: float = 1.0):
        """Bucketed gradient all-reduce over ``comm``; buckets of at most ``small_mb`` MB of wire bytes
        go through ``small`` (the IPC one-shot communicator) when one is given."""
        self.reducer = BucketReducer(self.fp, comm, int(bucket_mb * (1 << 20)), bf16=bf16_grads, force_dp=force_dp,
                                     small=small, small_bytes=int(small_mb * (1 << 20)))

    def forward(self, x_nhwc_f32: torch.Tensor) -> torch.Tensor:
        self.fwd_id += 1  # tags the BN states this forward leaves for its own backward
        for j in self.joins:
            j.reset()
        for bn in self.bns:
            bn.fwd_state, bn.bwd_part = None, None
        self.stats.zero()
        if self.stem_w2 and self.bn_stats and x_nhwc_f32.shape[2] % 2 == 0:
            yp = _StemW2.apply(_ops().stem_pack(x_nhwc_f32), self.token, self.stem)
        else:
            yp = self.stem(_ops().pad_channels(x_nhwc_f32, 8))
        if self.fuse_stem_pool and isinstance(yp, tuple):  # (y, statistics partials) from a stats conv
            x = _BNReluMaxPool.apply(yp[0], yp[1], self.stem_bn, 3, 2, 1)
        else:
            x = _MaxPool.apply(self.stem_bn(yp), 3, 2, 1)
        for blk in self.blocks:
            x = self.block_forward(blk, x)
        x = _AvgPool.apply(x)
        return self.fc(x)

    def block_forward(self, blk, x):
        sc = x
        if "cd" in blk:
            sc = blk["bd"](blk["cd"](x), relu=False)
        h = blk["c2"].after_bn(blk["b1"], blk["c1"](x))
        if self.kind == "basic":
            return blk["b2"](h, relu=True, res=sc)
        h = blk["c3"].after_bn(blk["b2"], h)
        return blk["b3"](h, relu=True, res=sc)

    def loss(self, x, labels):
        logits = self.forward(x)
        loss, correct = _SoftmaxXent.apply(logits, labels)
        return loss, correct

    @torch.no_grad()
    def evaluate(self, x, labels):
        """Inference-mode pass (BN with the running statistics, no dropout of state): returns the
        (sum of per-example losses, number correct) of the batch as floats -- the reference's accuracy
        op (/root/reference/mnist_python_m.py:206-207,309-320) for this model family."""
        ops = _ops()

        def bn(y, L, relu, res=None):
            if res is None:
                return ops.bn_infer(y, L.gamma(), L.beta(), L.rmean, L.rvar, L.eps, relu)
            z = ops.bn_infer(y, L.gamma(), L.beta(), L.rmean, L.rvar, L.eps, False).float() + res.float()
            return (z.relu_() if relu else z).to(torch.bfloat16)

        def conv(h, L):
            return ops.conv2d_fwd(h, L.w(), L.stride, L.pad)

        h = bn(conv(ops.pad_channels(x, 8), self.stem), self.stem_bn, True)
        h, _ = ops.maxpool2d_fwd(h, 3, 2, 1)
        for blk in self.blocks:
            sc = bn(conv(h, blk["cd"]), blk["bd"], False) if "cd" in blk else h
            t = bn(conv(h, blk["c1"]), blk["b1"], True)
            if self.kind == "basic":
                h = bn(conv(t, blk["c2"]), blk["b2"], True, sc)
            else:
                t = bn(conv(t, blk["c2"]), blk["b2"], True)
                h = bn(conv(t, blk["c3"]), blk["b3"], True, sc)
        logits = ops.linear_fwd(ops.avgpool_fwd(h), self.fc.w(), self.fc.bias())
        loss_rows, correct, _ = ops.softmax_xent(logits.contiguous(), labels)
        return float(loss_rows.float().sum().item()), int(round(float(correct.float().sum().item())))

    def train_step(self, x, labels, lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 1e-4):
        """fwd + bwd (bucketed all-reduce overlapped) + fused flat SGD-momentum. Returns loss tensor."""
        self.reducer.reset()
        # one fill of the flat fp32 grad buffer instead of a memset per split-K weight gradient
        self.fp.grad.zero_()
        self.grads_zeroed = True
        try:
            loss, _ = self.loss(x, labels)
            # backward on THIS thread, not the autograd engine's device thread: the bucket hooks
            # (BucketReducer.mark_ready) record their ready events inside backward, and stream work
            # issued from the engine's thread into a capture owned by this thread broke the host heap
            # once the captured graph was destroyed (profiles/heap_bisect_r5.log; the event record
            # alone still did, about once in 100+ RCCL capture / destroy cycles)
            with torch.autograd.set_multithreading_enabled(BACKWARD_ON_AUTOGRAD_THREADS):  # same speed (profiles/resnet50_backward_thread_ab_r5.log)
                loss.backward()
        finally:
            self.grads_zeroed = False
        self.reducer.finish()
        scale = 1.0 / self.reducer.world
        _ops().momentum_flat(self.fp.master, self.fp.momentum, self.reducer.reduced_grads(), self.fp.shadow, lr,
                             momentum, weight_decay, False, scale)
        return loss.detach()


class ResNetRunner:
    """The Supervisor's view of a ResNet (training/supervisor.py, the reference's Supervisor + Saver at
    /root/reference/mnist_python_m.py:235-253): a global step and TF-named checkpoint tensors in the
    MNIST runners' layout -- ``global_step``, every parameter under its layer name (conv weights HWIO,
    fc [in, out]), its SGD-momentum slot as ``<name>/Momentum``, and each batch norm's running
    statistics as ``<bn>/moving_mean`` / ``<bn>/moving_variance`` (TF's names)."""

    def __init__(self, model: "ResNet"):
        self.m = model
        self._step = 0
        self.ps_client = None

    def global_step(self) -> int:
        return self._step

    def set_global_step(self, s: int) -> None:
        self._step = int(s)

    def params(self) -> torch.Tensor:
        return self.m.fp.master

    def train_step(self, x, labels, lr: float, **kw):
        loss = self.m.train_step(x, labels, lr=lr, **kw)
        self._step += 1
        return loss

    def state_dict_tf(self):
        from collections import OrderedDict

        import numpy as np

        fp = self.m.fp
        if fp.device.type == "cuda":
            torch.cuda.synchronize(fp.device)
        out = OrderedDict()
        out["global_step"] = np.array(self._step, dtype=np.int64)
        master, mom = fp.master.detach().cpu(), fp.momentum.detach().cpu()
        stem = self.m.stem.name
        for s in fp.specs:
            w, mv = fp.view(master, s), fp.view(mom, s)
            if s.name == stem:  # the kernels' [7, 7, 8, K] channel padding is not saved: TF's [7, 7, 3, K]
                w, mv = w[:, :, :3, :], mv[:, :, :3, :]
            out[s.name] = w.numpy().copy()
            out[s.name + "/Momentum"] = mv.numpy().copy()
        for bn in self.m.bns:
            out[bn.name + "/moving_mean"] = bn.rmean.detach().cpu().numpy().copy()
            out[bn.name + "/moving_variance"] = bn.rvar.detach().cpu().numpy().copy()
        return out

    def load_state_dict_tf(self, tensors) -> None:
        import numpy as np

        fp = self.m.fp
        master = torch.zeros(fp.total)
        mom = torch.zeros(fp.total)
        stem = self.m.stem.name

        def put(dst, arr, s):
            t = torch.from_numpy(np.asarray(arr))
            if s.name == stem and t.numel() != dst.numel():  # [7, 7, 3, K] on disk: zero the padded channels
                dst.zero_()
                dst[:, :, :t.shape[2], :].copy_(t.reshape(s.shape[0], s.shape[1], -1, s.shape[3]))
            else:
                dst.copy_(t.reshape(s.shape))

        for s in fp.specs:
            put(fp.view(master, s), tensors[s.name], s)
            if s.name + "/Momentum" in tensors:
                put(fp.view(mom, s), tensors[s.name + "/Momentum"], s)
        fp.master.copy_(master.to(fp.device))
        fp.momentum.copy_(mom.to(fp.device))
        fp.shadow.copy_(fp.master)
        for bn in self.m.bns:
            bn.rmean.copy_(torch.from_numpy(np.asarray(tensors[bn.name + "/moving_mean"])).to(bn.rmean.device))
            bn.rvar.copy_(torch.from_numpy(np.asarray(tensors[bn.name + "/moving_variance"])).to(bn.rvar.device))
        self._step = int(np.asarray(tensors.get("global_step", 0)))
