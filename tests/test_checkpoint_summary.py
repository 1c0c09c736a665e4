"""TF-V2-bundle checkpoint + event-file codecs."""
import os
import struct
from collections import OrderedDict

import numpy as np
import pytest

from tensorflow_distributed_amd.training import checkpoint as C
from tensorflow_distributed_amd.training import summary as S


def test_crc32c_known_vector_and_mask():
    assert C.crc32c(b"123456789") == 0xE3069283
    assert C.crc32c(b"") == 0
    for v in (0, 1, 0xDEADBEEF, 0xFFFFFFFF):
        assert C.unmask_crc(C.mask_crc(v)) == v


def test_bundle_roundtrip_many_keys(tmp_path):
    rng = np.random.RandomState(0)
    t = OrderedDict([("global_step", np.array(41, np.int64)), ("Variable", rng.randn(5, 5, 1, 32).astype(np.float32)),
                     ("Variable/Adam", rng.randn(5, 5, 1, 32).astype(np.float32)),
                     ("beta1_power", np.array(0.9 ** 3, np.float32))])
    for i in range(400):  # several data blocks + restart points
        t[f"layer{i:04d}/kernel"] = rng.randn(i % 7 + 1).astype(np.float32)
    prefix = str(tmp_path / "model.ckpt-41")
    C.save_bundle(prefix, t)
    r = C.load_bundle(prefix)
    assert list(r) == sorted(t)
    for k, v in t.items():
        assert r[k].dtype == v.dtype and r[k].shape == v.shape and np.array_equal(r[k], v), k
    names = dict(C.list_variables(prefix))
    assert names["Variable"] == [5, 5, 1, 32] and names["global_step"] == []


def test_bundle_table_format(tmp_path):
    prefix = str(tmp_path / "m")
    C.save_bundle(prefix, OrderedDict(a=np.zeros(3, np.float32)))
    raw = open(prefix + ".index", "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == 0xDB4775248B80FB57  # LevelDB table magic
    items = C.read_sstable(prefix + ".index")
    assert items[0][0] == b"" and items[1][0] == b"a"  # header entry first
    assert os.path.getsize(prefix + ".data-00000-of-00001") == 12


def test_bundle_detects_corruption(tmp_path):
    prefix = str(tmp_path / "m")
    C.save_bundle(prefix, OrderedDict(a=np.arange(16, dtype=np.float32)))
    p = prefix + ".data-00000-of-00001"
    b = bytearray(open(p, "rb").read())
    b[5] ^= 0xFF
    open(p, "wb").write(bytes(b))
    with pytest.raises(ValueError):
        C.load_bundle(prefix)


def test_saver_keeps_latest_and_prunes(tmp_path):
    sv = C.Saver(max_to_keep=2)
    for s in (10, 20, 30):
        sv.save(str(tmp_path), OrderedDict(x=np.array([s], np.float32)), s)
    assert C.latest_checkpoint(str(tmp_path)).endswith("model.ckpt-30")
    st = C.read_checkpoint_state(str(tmp_path))
    assert st["all_model_checkpoint_paths"] == ["model.ckpt-20", "model.ckpt-30"]
    assert not os.path.exists(tmp_path / "model.ckpt-10.index")
    assert C.load_bundle(C.latest_checkpoint(str(tmp_path)))["x"][0] == 30


def test_event_file_roundtrip(tmp_path):
    w = S.EventFileWriter(str(tmp_path))
    w.add_scalar("global_step/sec", 3.5, 7)
    w.add_scalars({"loss": 0.25, "accuracy": 0.5}, 8)
    w.close()
    assert os.path.basename(w.path).startswith("events.out.tfevents.")
    assert S.read_scalars(w.path) == [(7, "global_step/sec", 3.5), (8, "loss", 0.25), (8, "accuracy", 0.5)]
    recs = list(S.read_records(w.path))
    assert b"brain.Event:2" in recs[0]


def test_resnet_supervisor_checkpoint_roundtrip(tmp_path):
    """The ResNet mode's Supervisor state (models/resnet.ResNetRunner, dist_main --model resnet*) on CPU:
    params (HWIO convs), SGD-momentum slots, BN running statistics and global_step go through the
    Saver's V2 bundle in the logdir layout and restore into a freshly initialised model bit for bit;
    the chief's prepare_or_wait_for_session finds the checkpoint and resumes from its step."""
    import torch

    from tensorflow_distributed_amd.models.resnet import ResNet, ResNetRunner
    from tensorflow_distributed_amd.training.checkpoint import latest_checkpoint
    from tensorflow_distributed_amd.training.supervisor import Supervisor

    cpu = torch.device("cpu")
    a = ResNetRunner(ResNet(18, num_classes=16, device=cpu, seed=1, width=16))
    g = torch.Generator().manual_seed(5)
    a.m.fp.master.copy_(torch.randn(a.m.fp.total, generator=g))
    a.m.fp.momentum.copy_(torch.randn(a.m.fp.total, generator=g))
    for bn in a.m.bns:
        bn.rmean.copy_(torch.randn(bn.c, generator=g))
        bn.rvar.copy_(torch.rand(bn.c, generator=g) + 0.5)
    stem = a.m.stem.name
    for buf in (a.m.fp.master, a.m.fp.momentum):  # the stem's padded input channels 3..7 carry no state
        a.m.fp.view(buf, a.m.fp.by_name[stem])[:, :, 3:, :].zero_()
    a.set_global_step(17)
    sd = a.state_dict_tf()
    assert sd["layer1.0.conv1"].shape == (3, 3, 16, 16) and sd["fc"].shape == (128, 16)
    assert sd[stem].shape == (7, 7, 3, 16) and sd[stem + "/Momentum"].shape == (7, 7, 3, 16)  # TF's stem layout
    assert "layer1.0.bn1/moving_mean" in sd and "layer1.0.conv1/Momentum" in sd
    sv = Supervisor(is_chief=True, logdir=str(tmp_path), runner=a, init_fn=lambda: None, summary_writer=False)
    path = sv.save(17)
    assert latest_checkpoint(str(tmp_path)) == path and path.endswith("model.ckpt-17")
    b = ResNetRunner(ResNet(18, num_classes=16, device=cpu, seed=2, width=16))
    inits = []
    sv2 = Supervisor(is_chief=True, logdir=str(tmp_path), runner=b, init_fn=lambda: inits.append(1),
                     summary_writer=False, log=lambda *_: None)
    sv2.prepare_or_wait_for_session()
    assert sv2.restored_from == path and not inits and b.global_step() == 17
    fa, fb = a.m.fp, b.m.fp
    for sp in fa.specs:  # (the flat buffers' 64-element slot padding is not state)
        for buf in ("master", "momentum"):
            assert torch.equal(fb.view(getattr(fb, buf), fb.by_name[sp.name]), fa.view(getattr(fa, buf), sp)), sp.name
        assert torch.equal(fb.w(sp.name), fa.p(sp.name).to(torch.bfloat16)), sp.name
    for x, y in zip(a.m.bns, b.m.bns):
        assert torch.equal(x.rmean, y.rmean) and torch.equal(x.rvar, y.rvar)
    sv2.stop(save=False)
