"""Device runners for the reference MNIST CNN: what ``sess.run(train_step)`` executes.

* :class:`NativeMnistRunner` (GPU): the C++ ``MnistEngine`` (``csrc/runtime/mnist_engine.cpp``) --
  fused HIP/MFMA forward+backward, bucketed RCCL gradient all-reduce overlapped with the conv
  backward, fused flat optimizer, optional hipGraph replay. This is the only GPU path; it fails
  loudly if the native library is missing.
* :class:`TorchMnistRunner` (CPU, the reference's default ``--num_gpus=0`` worker device,
  ``/root/reference/mnist_python_m.py:169-172``): fp32 PyTorch ops + autograd + the same optimizer
  equations (:class:`training.optimizers.FlatApplier`), gradients averaged over Gloo.

Both keep the parameters in the flat layout of ``csrc/mnist_layout.h`` so checkpoints, broadcasts
and the async parameter-server protocol are layout-identical across devices.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from ..training.optimizers import FlatApplier, base_optimizer
from . import mnist_cnn as M


def _labels_to_ids(y) -> torch.Tensor:
    y = torch.as_tensor(np.asarray(y)) if not isinstance(y, torch.Tensor) else y
    if y.dim() == 2:
        y = y.argmax(1)
    return y.to(torch.int32)


def _as_f32(x) -> torch.Tensor:
    x = torch.as_tensor(np.asarray(x)) if not isinstance(x, torch.Tensor) else x
    return x.reshape(x.shape[0], -1).to(torch.float32)


class MnistRunnerBase:
    batch_size: int
    device: torch.device

    # -- state (flat layout) --
    def params(self) -> torch.Tensor: ...
    def global_step(self) -> int: ...

    ps_client = None  # parallel.async_ps.AsyncPSClient when the variables live on PS tasks

    def state_dict_tf(self) -> "dict":
        """TF-named tensors for the checkpoint (mnist_python_m.py:178,185-196 creation order).
        With the variables on parameter servers (async / backup-worker modes) the values AND the
        optimizer slots are pulled from the PS tasks -- what TF's Saver would save."""
        from collections import OrderedDict

        flat = self.params().detach().float().cpu().clone()
        step = self.global_step()
        slot_t = {k: v.detach().float().cpu() for k, v in self.slot_tensors().items()}
        powers = self.powers()
        if self.ps_client is not None:
            got, t, step = self.ps_client.pull_state(flat)
            kind = getattr(getattr(self, "opt", None), "kind", "adam")
            slot_t = {("accum" if kind == "momentum" else k): v for k, v in got.items()}
            o = self.opt
            powers = {"beta1_power": o.beta1 ** t, "beta2_power": o.beta2 ** t} if kind == "adam" else {}
        out = OrderedDict()
        out["global_step"] = np.array(step, dtype=np.int64)
        views = M.dict_from_flat(flat)
        slots = {k: M.dict_from_flat(v) for k, v in slot_t.items()}
        for key, tf_name, _ in M.PARAM_SPECS:
            out[tf_name] = views[key].numpy().copy()
            if "m" in slots:
                out[tf_name + "/Adam"] = slots["m"][key].numpy().copy()
            if "v" in slots:
                out[tf_name + "/Adam_1"] = slots["v"][key].numpy().copy()
            if "accum" in slots:
                out[tf_name + "/Momentum"] = slots["accum"][key].numpy().copy()
        for k, v in powers.items():
            out[k] = np.array(v, dtype=np.float32)
        return out

    def load_state_dict_tf(self, tensors) -> None:
        flat = torch.zeros(M.TOTAL)
        views = M.dict_from_flat(flat)
        slots = {}
        for key, tf_name, _ in M.PARAM_SPECS:
            views[key].copy_(torch.from_numpy(np.asarray(tensors[tf_name])))
            for suffix, slot in (("/Adam", "m"), ("/Adam_1", "v"), ("/Momentum", "accum")):
                if tf_name + suffix in tensors:
                    sflat = slots.setdefault(slot, torch.zeros(M.TOTAL))
                    M.dict_from_flat(sflat)[key].copy_(torch.from_numpy(np.asarray(tensors[tf_name + suffix])))
        step = int(np.asarray(tensors.get("global_step", 0)))
        self.load_flat(flat, slots, step)

    def slot_tensors(self) -> "dict":
        return {}

    def powers(self) -> "dict":
        return {}

    def load_flat(self, flat: torch.Tensor, slots: "dict", step: int) -> None: ...


class TorchMnistRunner(MnistRunnerBase):
    """fp32 PyTorch implementation (CPU workers, the reference's default device)."""

    def __init__(self, batch_size: int, optimizer, keep_prob: float = 0.75, seed: int = 0, rank: int = 0,
                 device: Optional[torch.device] = None):
        self.batch_size = batch_size
        self.device = device or torch.device("cpu")
        self.keep_prob = keep_prob
        self.opt = base_optimizer(optimizer)
        self.flat = torch.zeros(M.TOTAL, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros_like(self.flat)
        self.applier = FlatApplier(self.opt, M.TOTAL, self.device)
        self._step = 0
        self.gen = torch.Generator(device=self.device).manual_seed(seed * 7919 + rank)
        self.comm = None  # DP reducer: callable(flat_grad) -> None (in-place average)

    def params(self) -> torch.Tensor:
        return self.flat

    def global_step(self) -> int:
        return self._step

    def set_global_step(self, s: int) -> None:
        self._step = int(s)

    def load_flat(self, flat, slots, step):
        self.flat.copy_(flat.to(self.device))
        for name, t in slots.items():
            key = {"accum": "m"}.get(name, name)
            dst = getattr(self.applier, key, None)
            if dst is not None:
                dst.copy_(t.to(self.device))
        self.applier.t = int(step)
        self._step = int(step)

    def slot_tensors(self):
        s = self.applier.slots()
        if self.opt.kind == "momentum":
            return {"accum": s["m"]}
        return s

    def powers(self):
        return self.applier.powers()

    def set_params(self, flat: torch.Tensor) -> None:
        self.flat.copy_(flat.to(self.device))

    def _forward(self, x, keep_prob, mask=None):
        p = M.dict_from_flat(self.flat)
        return M.conv_net(x, p, keep_prob, dropout_mask=mask)

    def compute_grads(self, x, y) -> Tuple[torch.Tensor, float]:
        x = _as_f32(x).to(self.device)
        y = _labels_to_ids(y).to(self.device)
        self.flat.requires_grad_(True)
        mask = (torch.rand(x.shape[0], M.HID, generator=self.gen, device=self.device) < self.keep_prob).float() \
            if self.keep_prob < 1.0 else None
        logits = self._forward(x, self.keep_prob, mask)
        loss = F.cross_entropy(logits, y.long())
        g, = torch.autograd.grad(loss, self.flat)
        self.flat.requires_grad_(False)
        self.grad.copy_(g)
        self._last_loss = float(loss.item())
        return self.grad, self._last_loss

    def apply_grads(self, grad: torch.Tensor, scale: float = 1.0) -> None:
        self.applier.apply(self.flat, grad, scale)
        self._step += 1

    def train_step(self, x, y) -> None:
        g, _ = self.compute_grads(x, y)
        if self.comm is not None:
            self.comm(g)
        self.apply_grads(g)

    def last_loss(self) -> float:
        return float(getattr(self, "_last_loss", float("nan")))

    def set_phase_timing(self, on: bool = True) -> None:
        pass

    def sync_state(self) -> None:
        pass  # never sharded

    def phase_times(self) -> dict:
        """CPU path: host time of the last Gloo gradient all-reduce (the only timed phase)."""
        ms = getattr(self.comm, "last_ms", None)
        return {"allreduce_ms": round(ms, 4)} if ms is not None else {}

    @torch.no_grad()
    def evaluate(self, x, y) -> Tuple[float, int]:
        x = _as_f32(x).to(self.device)
        y = _labels_to_ids(y).to(self.device).long()
        logits = self._forward(x, 1.0)
        loss = F.cross_entropy(logits, y, reduction="sum").item()
        return float(loss), int((logits.argmax(1) == y).sum().item())


class NativeMnistRunner(MnistRunnerBase):
    """GPU runner over the native MnistEngine (HIP kernels + RCCL + hipGraph)."""

    def __init__(self, batch_size: int, optimizer, keep_prob: float = 0.75, seed: int = 0, rank: int = 0,
                 device: Optional[torch.device] = None, comm=None, bf16_grads: bool = True, use_graph: bool = True,
                 dtype: str = "bf16"):
        from .. import _native

        _native.require()
        self.batch_size = batch_size
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.keep_prob = keep_prob
        self.opt = base_optimizer(optimizer)
        self.eng = torch.classes.tfd.MnistEngine(batch_size, self.device.index, keep_prob, seed, rank)
        self.eng.set_dtype(dtype)  # "bf16" MFMA operands, or "fp32" (the reference's precision)
        o = self.opt
        if o.kind == "adam":
            self.eng.set_adam(o.learning_rate, o.beta1, o.beta2, o.epsilon)
        elif o.kind == "momentum":
            self.eng.set_momentum(o.learning_rate, o.momentum, o.use_nesterov)
        else:
            self.eng.set_momentum(o.learning_rate, 0.0, False)
        self.comm = comm
        if comm is not None:
            self.eng.set_comm(comm, bf16_grads)
        self.stream = torch.cuda.Stream(self.device)
        self.use_graph = use_graph
        self._graph_ready = False
        self._grads_graph = False
        self._x_stage = torch.empty(batch_size, 784, dtype=torch.float32).pin_memory()
        self._y_stage = torch.empty(batch_size, dtype=torch.int32).pin_memory()
        self.transport = None  # parallel.transport.DPTransport when DP runs over RCCL/IPC
        self._dev_data = None  # device-resident split (set_device_dataset)
        self._hstep = 0        # host mirror of the device global_step (epoch bookkeeping, no sync)
        self._epoch = -1

    # ---- observability ----
    PHASES = ("fwd_ms", "bwd_fc_ms", "bwd_conv_ms", "optim_ms", "allreduce_ms", "comm_wait_ms", "step_ms_gpu")

    def set_phase_timing(self, on: bool = True) -> None:
        """HIP timing events at the step's phase boundaries (recorded inside the captured graph too).
        Takes effect for graphs captured afterwards."""
        self.eng.set_phase_timing(bool(on))
        self._graph_ready = False

    def phase_times(self) -> dict:
        """GPU milliseconds of the last step's phases (all 0 when timing is off)."""
        self.stream.synchronize()
        return {k: round(float(v), 4) for k, v in zip(self.PHASES, self.eng.phase_times().tolist())}

    def last_loss(self) -> float:
        """Mean training loss of the last step's batch (with its dropout mask)."""
        self.stream.synchronize()
        return float(self.eng.loss_rows().mean().item())

    # ---- device-resident input (reference feed: mnist_python_m.py:291-294) ----
    def set_device_dataset(self, images, labels, seed: int = 0) -> None:
        """Upload a training split once; every later ``train_step(None, None)`` gathers its batch on
        the device from ``perm[(global_step * B + b) % n]``. The permutation is redrawn at every
        epoch boundary, which is ``DataSet.next_batch``'s per-epoch reshuffle without a host feed."""
        x = _as_f32(images)
        y = _labels_to_ids(labels)
        n = x.shape[0]
        self._perm_gen = torch.Generator().manual_seed(int(seed))
        with torch.cuda.stream(self.stream):
            self._dev_data = x.to(self.device, non_blocking=False).contiguous()
            self._dev_labels = y.to(self.device).contiguous()
            self._dev_perm = torch.randperm(n, generator=self._perm_gen).to(torch.int32).to(self.device)
            self.eng.set_dataset(self._dev_data, self._dev_labels, self._dev_perm)
            self.eng.set_input_mode(1)
        self.stream.synchronize()
        self._hstep = self.global_step()
        self._epoch = (self._hstep * self.batch_size) // n

    def last_device_batch(self):
        """(x, y) device tensors of the batch the last device-input step trained on."""
        n = self._dev_data.shape[0]
        pos = ((self._hstep - 1) * self.batch_size + torch.arange(self.batch_size, device=self.device)) % n
        with torch.cuda.stream(self.stream):
            rows = self._dev_perm[pos].long()
            out = self._dev_data[rows], self._dev_labels[rows]
        self.stream.synchronize()
        return out

    def _device_batch(self) -> None:
        n = self._dev_data.shape[0]
        ep = (self._hstep * self.batch_size) // n
        if ep != self._epoch:
            self._epoch = ep
            p = torch.randperm(n, generator=self._perm_gen).to(torch.int32)
            with torch.cuda.stream(self.stream):
                self._dev_perm.copy_(p.to(self.device))
                self.eng.invalidate_prefetch()  # rows prefetched from the old permutation

    # ---- state ----
    def params(self) -> torch.Tensor:
        return self.eng.params()

    def global_step(self) -> int:
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        return int(self.eng.step_tensor().item())

    def set_global_step(self, s: int) -> None:
        with torch.cuda.stream(self.stream):
            self.eng.step_tensor().fill_(int(s))
        self._hstep = int(s)

    def load_flat(self, flat, slots, step):
        with torch.cuda.stream(self.stream):
            self.eng.params().copy_(flat.to(self.device))
            self.eng.sync_shadow()
            if "m" in slots or "accum" in slots:
                self.eng.adam_m().copy_(slots.get("m", slots.get("accum")).to(self.device))
            if "v" in slots:
                self.eng.adam_v().copy_(slots["v"].to(self.device))
            self.eng.step_tensor().fill_(int(step))
        self.stream.synchronize()
        self._hstep = int(step)

    def slot_tensors(self):
        self.stream.synchronize()
        if self.opt.kind == "adam":
            return {"m": self.eng.adam_m(), "v": self.eng.adam_v()}
        if self.opt.kind == "momentum":
            return {"accum": self.eng.adam_m()}
        return {}

    def powers(self):
        o = self.opt
        if o.kind != "adam":
            return {}
        t = self.global_step()
        return {"beta1_power": o.beta1 ** t, "beta2_power": o.beta2 ** t}

    def set_params(self, flat: torch.Tensor) -> None:
        with torch.cuda.stream(self.stream):
            self.eng.params().copy_(flat.to(self.device, non_blocking=True))
            self.eng.sync_shadow()

    def broadcast_from(self, root: int = 0) -> None:
        """Chief init -> every worker (reference M6: init_op on PS vars; here an RCCL broadcast)."""
        if self.comm is None:
            return
        with torch.cuda.stream(self.stream):
            self.comm.broadcast(self.eng.params(), root)
            self.comm.broadcast(self.eng.adam_m(), root)
            self.comm.broadcast(self.eng.adam_v(), root)
            self.comm.broadcast(self.eng.step_tensor(), root)
            self.eng.sync_shadow()
        self.stream.synchronize()
        self._hstep = int(self.eng.step_tensor().item())

    # ---- feeds ----
    def _feed(self, x, y) -> None:
        if x is None:
            assert self._dev_data is not None, "train_step(None, None) needs set_device_dataset() first"
            self._device_batch()
            return
        if self._dev_data is not None:
            raise ValueError("host batches fed to a runner in device-input mode")
        x = _as_f32(x)
        y = _labels_to_ids(y)
        assert x.shape[0] == self.batch_size, f"batch {x.shape[0]} != engine batch {self.batch_size}"
        self._x_stage.copy_(x)
        self._y_stage.copy_(y)
        with torch.cuda.stream(self.stream):
            self.eng.feed_x().copy_(self._x_stage, non_blocking=True)
            self.eng.feed_y().copy_(self._y_stage, non_blocking=True)

    # ---- steps ----
    def train_step(self, x, y) -> None:
        self._feed(x, y)
        with torch.cuda.stream(self.stream):
            if self.use_graph:
                if not self._graph_ready:
                    self.eng.train_step()
                    self.eng.capture_train_step("train")
                    self._graph_ready = True
                else:
                    self.eng.replay("train", 1)
            else:
                self.eng.train_step()
        self._hstep += 1
        if x is not None:
            # the pinned staging buffers are reused next step: wait for the H2D copies to land
            self.stream.synchronize()

    def compute_grads(self, x, y, with_loss: bool = True) -> Tuple[torch.Tensor, Optional[float]]:
        """Forward + backward only (no reduction / optimizer). Bumps the engine's local step. With
        ``use_graph`` the three launches replay as one captured graph (``MnistEngine.capture_grads``).
        ``with_loss=False`` skips the loss read-back (no device-to-host transfer)."""
        self._feed(x, y)
        with torch.cuda.stream(self.stream):
            if self.use_graph:
                if not self._grads_graph:
                    self.eng.forward(True)
                    self.eng.backward_a()
                    self.eng.backward_b()
                    self.eng.capture_grads("grads")
                    self._grads_graph = True
                else:
                    self.eng.replay("grads", 1)
            else:
                self.eng.forward(True)
                self.eng.backward_a()
                self.eng.backward_b()
        self.stream.synchronize()
        self._hstep += 1
        return self.eng.grads(), (float(self.eng.loss_rows().mean().item()) if with_loss else None)

    def sync_state(self) -> None:
        """ZeRO-1 (``eng.zero()``): every worker gathers the fc1 shards of the fp32 master and the Adam
        slots, so ``params()`` / ``slot_tensors()`` are whole (a collective: all workers call it)."""
        with torch.cuda.stream(self.stream):
            self.eng.sync_params()
        self.stream.synchronize()

    def sync_shadow(self) -> None:
        """Re-derive the bf16 operand shadow from the fp32 master (after a parameter server wrote the
        fresh values into ``params()``)."""
        with torch.cuda.stream(self.stream):
            self.eng.sync_shadow()

    def reduce_grads(self, weight: float = 1.0) -> None:
        """Sum-all-reduce of (weight * local grads) over the worker communicator."""
        with torch.cuda.stream(self.stream):
            self.eng.reduce_grads(weight)
        self.stream.synchronize()

    def apply_grads(self, grad: Optional[torch.Tensor] = None, scale: float = 1.0) -> None:
        with torch.cuda.stream(self.stream):
            if grad is not None and grad.data_ptr() != self.eng.grads().data_ptr():
                self.eng.grads().copy_(grad.to(self.device))
            self.eng.apply_optimizer(scale)
        self.stream.synchronize()

    def evaluate(self, x, y) -> Tuple[float, int]:
        x = _as_f32(x).to(self.device)
        y = _labels_to_ids(y).to(self.device)
        with torch.cuda.stream(self.stream):
            r = self.eng.evaluate(x, y)
        self.stream.synchronize()
        r = r.cpu()
        return float(r[0]), int(round(float(r[1])))


def make_runner(batch_size: int, optimizer, device: torch.device, keep_prob: float = 0.75, seed: int = 0,
                rank: int = 0, comm=None, bf16_grads: bool = True, use_graph: bool = True,
                dtype: str = "bf16") -> MnistRunnerBase:
    if device.type == "cuda":
        return NativeMnistRunner(batch_size, optimizer, keep_prob, seed, rank, device, comm, bf16_grads, use_graph,
                                 dtype)
    return TorchMnistRunner(batch_size, optimizer, keep_prob, seed, rank, device)
