"""Dropout numerics and the learning curve of the native step (VERDICT r1 'weak' item 6).

* The head kernel's Philox mask is replayed on the host (``mnist_cnn.native_dropout_mask``) and fed
  to the fp32 oracle, so the keep_prob = 0.75 training step (K5 dropout fwd, K9 dropout bwd +
  ReluGrad; ``/root/reference/mnist_python_m.py:124,292``) is checked element for element.
* Keep-rate statistics of the mask, per-step / per-rank independence, no dropout in eval.
* The learning curve at the reference configuration (N(0,1) init, Adam lr 0.01, B = 128,
  keep 0.75; ``mnist_python_m.py:71,185-208``) tracks the fp32 oracle replaying the same masks
  and batches over 48 steps.
"""
import pytest
import torch

from tensorflow_distributed_amd.models import mnist_cnn as M

pytestmark = pytest.mark.gpu
SEED = 1234


def _engine(B, dev, keep):
    return torch.classes.tfd.MnistEngine(B, dev.index or 0, keep, SEED, 0)


def _relerr(a, b):
    return (a - b).norm().item() / max(b.norm().item(), 1e-30)


def test_native_dropout_mask_replayed_by_oracle(cuda):
    B, keep, step = 128, 0.75, 7
    torch.manual_seed(0)
    params = {k: v * 0.05 for k, v in M.init_params(7).items()}
    x = torch.rand(B, 784)
    y = torch.randint(0, 10, (B,), dtype=torch.int32)
    eng = _engine(B, cuda, keep)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.params().copy_(M.flat_from_dict(params).to(cuda))
        eng.sync_shadow()
        eng.step_tensor().fill_(step)
        eng.feed_x().copy_(x.to(cuda))
        eng.feed_y().copy_(y.to(cuda))
        eng.forward(True)
        eng.backward_a()
        eng.backward_b()
    torch.cuda.synchronize()
    mask = M.native_dropout_mask(B, step, 0, SEED, keep)
    hd = eng.hidden().float().cpu()
    assert torch.all(hd[mask == 0] == 0), "a dropped unit carried activation"
    p = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    logits = M.conv_net(x, p, keep, dropout_mask=mask, emulate_bf16=True)
    rows = torch.nn.functional.cross_entropy(logits, y.long(), reduction="none")
    rows.mean().backward()
    assert _relerr(eng.loss_rows().cpu(), rows.detach()) < 5e-3
    g = M.dict_from_flat(eng.grads().cpu())
    for k in p:
        e = _relerr(g[k], p[k].grad)
        assert e < 2e-2, f"{k}: relerr {e:.3e}"


def test_dropout_keep_rate_and_independence(cuda):
    B, keep = 128, 0.75
    masks = [M.native_dropout_mask(B, s, r, SEED, keep) for s in range(8) for r in (0, 1)]
    rate = torch.stack(masks).mean().item()
    assert abs(rate - keep) < 3e-3, rate  # 2.1 M Bernoulli draws: std 3e-4
    # different steps and different ranks draw different masks (~ 2 p (1 - p) = 37.5 % differ)
    d_step = (masks[0] != masks[2]).float().mean().item()
    d_rank = (masks[0] != masks[1]).float().mean().item()
    assert 0.35 < d_step < 0.40 and 0.35 < d_rank < 0.40, (d_step, d_rank)
    # the engine: keep_prob 1 (eval semantics) never drops, training drops exactly the replayed units
    eng = _engine(B, cuda, keep)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.params().copy_(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()}).to(cuda))
        eng.sync_shadow()
        eng.feed_x().copy_(torch.rand(B, 784, device=cuda))
        eng.feed_y().copy_(torch.randint(0, 10, (B,), dtype=torch.int32, device=cuda))
        eng.step_tensor().fill_(3)
        eng.set_keep_prob(1.0)  # the head writes hidden() in training mode only
        eng.forward(True)
        h_eval = eng.hidden().float().cpu().clone()
        eng.set_keep_prob(keep)
        eng.forward(True)
        h_train = eng.hidden().float().cpu().clone()
    torch.cuda.synchronize()
    m = M.native_dropout_mask(B, 3, 0, SEED, keep)
    active = h_eval > 0
    assert torch.equal((h_train > 0), active & (m > 0))
    torch.testing.assert_close(h_train[active & (m > 0)], (h_eval[active & (m > 0)] / keep).to(torch.bfloat16).float(),
                               rtol=1e-2, atol=0)


def _learnable(n, seed):
    g = torch.Generator().manual_seed(seed)
    tmpl = torch.rand(10, 784, generator=g)
    y = torch.randint(0, 10, (n,), generator=g)
    x = (0.4 * tmpl[y] + 0.6 * torch.rand(n, 784, generator=g)).clamp(0, 1)
    return x, y.to(torch.int32)


def test_learning_curve_tracks_fp32_oracle_at_reference_config(cuda):
    """48 steps, N(0,1) init, Adam 0.01, B = 128, keep 0.75: the native bf16 step and the fp32
    oracle (same batches, same replayed dropout masks) stay within a band. With N(0,1) init the
    minibatch losses start near 1e5 and fall by orders of magnitude; bf16 rounding makes the two
    trajectories drift apart slowly: every 8-step window mean within 15 % of the oracle's
    (measured: <= 7 %), and held-out accuracy after 48 steps (a noisy 10-template task) within 8
    points of the oracle's, both above 65 % (measured 76.9 / 71.8 %)."""
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer, FlatApplier

    B, keep, steps = 128, 0.75, 48
    x, y = _learnable(B * steps + 2000, 5)
    xv, yv = x[B * steps:], y[B * steps:]
    p0 = M.flat_from_dict(M.init_params(0))
    eng = _engine(B, cuda, keep)
    eng.set_adam(0.01, 0.9, 0.999, 1e-8)
    s = torch.cuda.Stream()
    nat = []
    with torch.cuda.stream(s):
        eng.params().copy_(p0.to(cuda))
        eng.sync_shadow()
        for i in range(steps):
            eng.feed_x().copy_(x[i * B:(i + 1) * B].to(cuda))
            eng.feed_y().copy_(y[i * B:(i + 1) * B].to(cuda))
            eng.train_step()
            nat.append(eng.loss_rows().mean())
        r = eng.evaluate(xv.to(cuda), yv.to(cuda)).cpu()
    torch.cuda.synchronize()
    nat = torch.stack(nat).cpu()
    acc_nat = float(r[1]) / len(xv)
    flat = p0.clone()
    ap = FlatApplier(AdamOptimizer(0.01), M.TOTAL)
    ora = []
    for i in range(steps):
        xb, yb = x[i * B:(i + 1) * B], y[i * B:(i + 1) * B]
        flat.requires_grad_(True)
        logits = M.conv_net(xb, M.dict_from_flat(flat), keep,
                            dropout_mask=M.native_dropout_mask(B, i, 0, SEED, keep))
        loss = torch.nn.functional.cross_entropy(logits, yb.long())
        g, = torch.autograd.grad(loss, flat)
        flat = flat.detach()
        ap.apply(flat, g)
        ora.append(loss.item())
    with torch.no_grad():
        acc_ora = (M.conv_net(xv, M.dict_from_flat(flat), 1.0).argmax(1) == yv.long()).float().mean().item()
    ora = torch.tensor(ora)
    assert nat[-8:].mean() < 1e-2 * nat[:8].mean()  # it learns (N(0,1) init: huge initial loss)
    curves = [(round(nat[w:w + 8].mean().item(), 3), round(ora[w:w + 8].mean().item(), 3)) for w in range(0, steps, 8)]
    print("window means (native, oracle):", curves, "accuracy:", acc_nat, acc_ora)
    for i, (a, b) in enumerate(curves):
        assert abs(a - b) <= 0.15 * b, curves
    assert acc_nat > 0.65 and acc_ora > 0.65 and abs(acc_nat - acc_ora) < 0.08, (acc_nat, acc_ora)
