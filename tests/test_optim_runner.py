"""Optimizer equations (TF1 ApplyAdam / Momentum / GD) and the CPU runner vs the PyTorch oracle."""
import numpy as np
import pytest
import torch

from tensorflow_distributed_amd.models import mnist_cnn as M
from tensorflow_distributed_amd.models.mnist_runner import TorchMnistRunner
from tensorflow_distributed_amd.training.optimizers import (AdamOptimizer, FlatApplier, GradientDescentOptimizer,
                                                            MomentumOptimizer, SyncReplicasOptimizer)


def _adam_ref(p, grads, lr=0.01, b1=0.9, b2=0.999, eps=1e-8):
    p = p.astype(np.float64).copy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    for t, g in enumerate(grads, 1):
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        lr_t = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        p -= lr_t * m / (np.sqrt(v) + eps)
    return p


def test_adam_matches_tf_apply_adam():
    rng = np.random.RandomState(0)
    p0 = rng.randn(1000).astype(np.float32)
    gs = [rng.randn(1000).astype(np.float32) for _ in range(5)]
    p = torch.tensor(p0)
    ap = FlatApplier(AdamOptimizer(0.01), 1000)
    for g in gs:
        ap.apply(p, torch.tensor(g))
    np.testing.assert_allclose(p.numpy(), _adam_ref(p0, gs), rtol=1e-5, atol=1e-6)
    assert ap.powers()["beta1_power"] == pytest.approx(0.9 ** 5)


def test_momentum_and_sgd():
    p = torch.ones(4)
    ap = FlatApplier(MomentumOptimizer(0.1, 0.5), 4)
    ap.apply(p, torch.ones(4))
    ap.apply(p, torch.ones(4))  # accum: 1, then 1.5 -> p = 1 - 0.1 - 0.15
    assert torch.allclose(p, torch.full((4,), 0.75))
    q = torch.ones(3)
    FlatApplier(GradientDescentOptimizer(0.5), 3).apply(q, torch.full((3,), 2.0), scale=0.5)
    assert torch.allclose(q, torch.full((3,), 0.5))


def test_sync_replicas_resolve():
    s = SyncReplicasOptimizer(AdamOptimizer(), None, None).resolve(3)
    assert s.replicas_to_aggregate == 3 and s.total_num_replicas == 3 and not s.has_backup_workers
    s2 = SyncReplicasOptimizer(AdamOptimizer(), 2, 3).resolve(3)
    assert s2.has_backup_workers
    with pytest.raises(ValueError):
        SyncReplicasOptimizer(AdamOptimizer(), 4, 3).resolve(3)


def test_flat_layout_roundtrip():
    p = M.init_params(3)
    flat = M.flat_from_dict(p)
    back = M.dict_from_flat(flat)
    assert sum(v.numel() for v in back.values()) == M.NUM_PARAMS == 3274634
    for k in p:
        assert torch.equal(back[k], p[k])


def test_torch_runner_grads_match_oracle():
    torch.manual_seed(0)
    B = 16
    params = {k: v * 0.05 for k, v in M.init_params(1).items()}
    x = torch.rand(B, 784)
    y = torch.randint(0, 10, (B,))
    r = TorchMnistRunner(B, AdamOptimizer(0.01), keep_prob=1.0)
    r.load_flat(M.flat_from_dict(params), {}, 0)
    g, loss = r.compute_grads(x, y)
    ref = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    lref = M.softmax_xent_mean(M.conv_net(x, ref, 1.0), torch.nn.functional.one_hot(y, 10).float())
    lref.backward()
    assert loss == pytest.approx(lref.item(), rel=1e-5)
    gd = M.dict_from_flat(g)
    for k in ref:
        torch.testing.assert_close(gd[k], ref[k].grad, rtol=1e-4, atol=1e-6)


def test_torch_runner_checkpoint_state_roundtrip(tmp_path):
    from tensorflow_distributed_amd.training.checkpoint import load_bundle, save_bundle

    r = TorchMnistRunner(8, AdamOptimizer(0.01), keep_prob=1.0)
    r.load_flat(M.flat_from_dict(M.init_params(2)), {}, 0)
    x, y = torch.rand(8, 784), torch.randint(0, 10, (8,))
    r.train_step(x, y)
    r.train_step(x, y)
    sd = r.state_dict_tf()
    assert {"global_step", "Variable", "Variable_7", "Variable/Adam", "Variable_7/Adam_1", "beta1_power"} <= set(sd)
    assert int(sd["global_step"]) == 2 and sd["Variable_2"].shape == (3136, 1024)
    save_bundle(str(tmp_path / "ck"), sd)
    r2 = TorchMnistRunner(8, AdamOptimizer(0.01), keep_prob=1.0)
    r2.load_state_dict_tf(load_bundle(str(tmp_path / "ck")))
    assert r2.global_step() == 2 and torch.equal(r2.params(), r.params())
    r.train_step(x, y)
    r2.train_step(x, y)
    assert torch.allclose(r.params(), r2.params())


def test_cpu_training_learns():
    from tensorflow_distributed_amd.utils import input_data as I

    imgs, labels = I.synthetic_mnist(2048, seed=5)
    ds = I.DataSet(imgs, labels, one_hot=True, seed=0)
    r = TorchMnistRunner(64, AdamOptimizer(0.01), keep_prob=0.75)
    r.load_flat(M.flat_from_dict(M.init_params(0)), {}, 0)
    x0, y0 = ds.images[:512], ds.labels[:512]
    _, c0 = r.evaluate(x0, y0)
    for _ in range(60):  # calibrated (MNIST-difficulty) synthetic data: ~75 % after 60 steps
        r.train_step(*ds.next_batch(64))
    _, c1 = r.evaluate(x0, y0)
    assert c1 > c0 + 100 and c1 / 512 > 0.5, (c0, c1)
