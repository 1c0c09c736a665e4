"""The reference 2-conv MNIST CNN: parameters, flat layout, and a pure-PyTorch fp32 oracle.

Topology (``/root/reference/mnist_python_m.py:104-128``, ``mnist_single.py:68-88``)::

    x[-1,784] -> reshape [-1,28,28,1] (NHWC)
    conv1: conv2d(5x5, 1->32, SAME) + bias + relu -> maxpool 2x2/2 SAME -> [14,14,32]
    conv2: conv2d(5x5, 32->64, SAME) + bias + relu -> maxpool 2x2/2 SAME -> [7,7,64]
    fc1  : reshape [-1,3136] (h,w,c order) @ wd1[3136,1024] + bd1 -> relu -> dropout(keep_prob)
    out  : @ out[1024,10] + out_b -> logits

Parameters are created in the reference's dict-literal order (weights wc1, wc2, wd1, out, then
biases bc1, bc2, bd1, out) and initialised ``tf.random_normal`` = N(0, 1) **including the biases**
(``mnist_python_m.py:185-196``). TF auto-names them ``Variable``..``Variable_7``,
which is the checkpoint variable naming we keep.

The native engine keeps all parameters in ONE flat fp32 buffer (``csrc/mnist_layout.h``): each
weight is followed by its bias (so a weight-grad GEMM emits the bias grad as an extra row) and
regions are padded to 64 elements.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Optional

import torch
import torch.nn.functional as F

IMG, C1, C2, FEAT, HID, NCLS = 28, 32, 64, 3136, 1024, 10

# (key, tf auto-name, shape) in reference creation order (mnist_python_m.py:185-196)
PARAM_SPECS = [
    ("wc1", "Variable", (5, 5, 1, 32)),
    ("wc2", "Variable_1", (5, 5, 32, 64)),
    ("wd1", "Variable_2", (FEAT, HID)),
    ("out", "Variable_3", (HID, NCLS)),
    ("bc1", "Variable_4", (32,)),
    ("bc2", "Variable_5", (64,)),
    ("bd1", "Variable_6", (HID,)),
    ("out_b", "Variable_7", (NCLS,)),
]
NUM_PARAMS = 3274634

# flat layout (must match csrc/mnist_layout.h)
OFFSETS = OrderedDict([
    ("wc1", 0), ("bc1", 800),
    ("wc2", 832), ("bc2", 832 + 51200),
    ("wd1", 52096), ("bd1", 52096 + FEAT * HID),
    ("out", 3264384), ("out_b", 3264384 + HID * NCLS),
])
TOTAL = 3274688
BUCKET_SPLIT = 52096  # [0, split): conv grads (bucket B); [split, TOTAL): fc grads (bucket A)
SHAPES = {k: s for k, _, s in PARAM_SPECS}
TF_NAMES = {k: n for k, n, _ in PARAM_SPECS}


def _numel(shape):
    n = 1
    for s in shape:
        n *= s
    return n


def init_params(seed: int = 0, dtype=torch.float32) -> Dict[str, torch.Tensor]:
    """N(0,1) init of every parameter in reference creation order (deterministic for a seed)."""
    g = torch.Generator().manual_seed(seed)
    return OrderedDict((k, torch.randn(*s, generator=g, dtype=dtype)) for k, _, s in PARAM_SPECS)


def flat_from_dict(params: Dict[str, torch.Tensor], device=None) -> torch.Tensor:
    flat = torch.zeros(TOTAL, dtype=torch.float32, device=device)
    for k, off in OFFSETS.items():
        t = params[k].detach().reshape(-1).to(torch.float32)
        flat[off:off + t.numel()].copy_(t)
    return flat


def dict_from_flat(flat: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Views of the flat buffer with the reference shapes (HWIO filters, [in,out] dense)."""
    out = OrderedDict()
    for k, _, shape in PARAM_SPECS:
        off = OFFSETS[k]
        out[k] = flat[off:off + _numel(shape)].view(*shape)
    return out


# ------------------------------------------------------------------ reference ops (fp32 oracle)
def conv2d_same_nhwc(x: torch.Tensor, w_hwio: torch.Tensor, b: torch.Tensor, stride: int = 1) -> torch.Tensor:
    """tf.nn.conv2d(x, W, strides=[1,s,s,1], padding='SAME') + bias_add, NHWC in/out."""
    kh, kw = w_hwio.shape[0], w_hwio.shape[1]
    xn = x.permute(0, 3, 1, 2)
    ih, iw = xn.shape[2], xn.shape[3]
    oh, ow = -(-ih // stride), -(-iw // stride)
    ph = max((oh - 1) * stride + kh - ih, 0)
    pw = max((ow - 1) * stride + kw - iw, 0)
    xn = F.pad(xn, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
    y = F.conv2d(xn, w_hwio.permute(3, 2, 0, 1), b, stride=stride)
    return y.permute(0, 2, 3, 1)


def maxpool_same_nhwc(x: torch.Tensor, k: int = 2) -> torch.Tensor:
    """tf.nn.max_pool(ksize=k, strides=k, padding='SAME'), NHWC (pads with -inf)."""
    xn = x.permute(0, 3, 1, 2)
    h, w = xn.shape[2], xn.shape[3]
    oh, ow = -(-h // k), -(-w // k)
    ph, pw = max(oh * k - h, 0), max(ow * k - w, 0)
    if ph or pw:
        xn = F.pad(xn, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=float("-inf"))
    return F.max_pool2d(xn, k, k).permute(0, 2, 3, 1)


def conv_net(x: torch.Tensor, p: Dict[str, torch.Tensor], keep_prob: float = 1.0,
             dropout_mask: Optional[torch.Tensor] = None, emulate_bf16: bool = False,
             bf16_conv1: bool = True) -> torch.Tensor:
    """Reference forward (mnist_python_m.py:104-128). ``dropout_mask`` (0/1, [B,1024]) overrides
    random dropout so the oracle can replay the native kernel's Philox mask. ``emulate_bf16``
    rounds at exactly the points where the native bf16 kernels store/consume bf16 (``bf16_conv1``:
    conv1's operands too -- the fused conv1->conv2 kernel runs conv1 on the bf16 matrix core)."""
    r = (lambda t: t.to(torch.bfloat16).to(torch.float32)) if emulate_bf16 else (lambda t: t)
    r1 = r if bf16_conv1 else (lambda t: t)
    x = x.reshape(-1, IMG, IMG, 1)
    h = torch.relu(conv2d_same_nhwc(r1(x), r1(p["wc1"]), p["bc1"]))
    h = r(maxpool_same_nhwc(h, 2))
    h = torch.relu(conv2d_same_nhwc(h, r(p["wc2"]), p["bc2"]))
    h = r(maxpool_same_nhwc(h, 2))
    h = h.reshape(-1, FEAT)
    h = torch.relu(h @ r(p["wd1"]) + p["bd1"])
    if dropout_mask is not None:
        h = h * dropout_mask / keep_prob
    elif keep_prob < 1.0:
        h = F.dropout(h, p=1.0 - keep_prob, training=True)
    return h @ p["out"] + p["out_b"]


def fc_sufficient_factors(x: torch.Tensor, labels: torch.Tensor, p: Dict[str, torch.Tensor],
                          keep_prob: float = 1.0, dropout_mask: Optional[torch.Tensor] = None):
    """The per-example factors of this rank's fc-layer gradients (what the native DP step
    all-gathers instead of all-reducing the fc gradients, ``mnist_fc_grad_sfb``):
    p2 [B,3136] (fc1 input), hd [B,1024] (fc1 output after relu + dropout), dh [B,1024] (gradient at
    the fc1 pre-activation), dl [B,10] (gradient at the logits, 1/B of the mean folded in)."""
    x = x.reshape(-1, IMG, IMG, 1)
    h = torch.relu(conv2d_same_nhwc(x, p["wc1"], p["bc1"]))
    h = maxpool_same_nhwc(h, 2)
    h = torch.relu(conv2d_same_nhwc(h, p["wc2"], p["bc2"]))
    p2 = maxpool_same_nhwc(h, 2).reshape(-1, FEAT).detach()
    z = (p2 @ p["wd1"] + p["bd1"]).requires_grad_(True)
    hd = torch.relu(z)
    if dropout_mask is not None:
        hd = hd * dropout_mask / keep_prob
    hd_leaf = hd.detach().requires_grad_(True)
    logits = (hd_leaf @ p["out"] + p["out_b"]).detach().requires_grad_(True)
    loss = softmax_xent_mean(logits, labels)
    (dl,) = torch.autograd.grad(loss, [logits])
    dhd = dl @ p["out"].t()
    (dh,) = torch.autograd.grad(hd, [z], dhd)
    return p2, hd.detach(), dh.detach(), dl.detach()


def fc_grads_from_factors(p2: torch.Tensor, hd: torch.Tensor, dh: torch.Tensor, dl: torch.Tensor):
    """Summed fc-layer gradients over every row of the (gathered) factors -- equal to the sum of the
    per-rank gradients because each is a sum of per-example outer products:
    dW_fc1 = p2^T dh, d bd1 = 1^T dh, dW_out = hd^T dl, d out_b = 1^T dl."""
    return {"wd1": p2.t() @ dh, "bd1": dh.sum(0), "out": hd.t() @ dl, "out_b": dl.sum(0)}


def softmax_xent_mean(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """reduce_mean(softmax_cross_entropy_with_logits(logits, onehot)) — labels: int class ids or one-hot."""
    if labels.dim() == 2:
        return torch.mean(-(labels * torch.log_softmax(logits, dim=1)).sum(1))
    return F.cross_entropy(logits, labels.long())


def accuracy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    lab = labels.argmax(1) if labels.dim() == 2 else labels.long()
    return (logits.argmax(1) == lab).float().mean()


# ------------------------------------------------------------------ native dropout mask (host replay)
def _philox4x32_10(c, k0, k1):
    """Philox4x32-10 on uint64 numpy arrays holding 32-bit lanes (csrc/common.h philox4x32_10)."""
    import numpy as np

    m32 = np.uint64(0xFFFFFFFF)
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
    c0, c1, c2, c3 = (x.astype(np.uint64) for x in c)
    k0 = np.uint64(k0) & m32
    k1 = np.uint64(k1) & m32
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & m32
        hi1, lo1 = p1 >> np.uint64(32), p1 & m32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + W0) & m32
        k1 = (k1 + W1) & m32
    return c0, c1, c2, c3


def native_dropout_mask(batch: int, step: int, rank: int, seed: int, keep_prob: float) -> torch.Tensor:
    """The exact 0/1 dropout mask [batch, 1024] the native head kernel draws at global step ``step``
    (counter = row * 256 + thread, (step lo, step hi, rank); key = (seed, 0x5EED1234); unit j of
    thread t is hidden unit 4t + j; kept iff u01 < keep_prob), so the fp32 oracle can replay it."""
    import numpy as np

    rows = np.arange(batch, dtype=np.uint64)[:, None]
    t = np.arange(256, dtype=np.uint64)[None, :]
    c0 = (rows * np.uint64(256) + t) & np.uint64(0xFFFFFFFF)
    shape = c0.shape
    c1 = np.full(shape, step & 0xFFFFFFFF, dtype=np.uint64)
    c2 = np.full(shape, (step >> 32) & 0xFFFFFFFF, dtype=np.uint64)
    c3 = np.full(shape, rank & 0xFFFFFFFF, dtype=np.uint64)
    out = _philox4x32_10((c0, c1, c2, c3), seed & 0xFFFFFFFF, 0x5EED1234)
    u = np.stack([((v >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)) for v in out], axis=-1)
    return torch.from_numpy((u < np.float32(keep_prob)).reshape(batch, HID).astype(np.float32))
