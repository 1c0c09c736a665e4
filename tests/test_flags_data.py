"""Flag system (tf.app.flags semantics) and the MNIST input pipeline (IDX codec, next_batch)."""
import numpy as np
import pytest

from tensorflow_distributed_amd.utils import flags as F
from tensorflow_distributed_amd.utils import input_data as I


def _fv():
    fv = F.FlagValues()
    F.DEFINE_string("data_dir", "/tmp/mnist-data", "", flag_values=fv)
    F.DEFINE_integer("task_index", 0, "", flag_values=fv)
    F.DEFINE_boolean("sync_replicas", True, "", flag_values=fv)
    F.DEFINE_float("learning_rate", 0.01, "", flag_values=fv)
    F.DEFINE_list("hosts", [], "", flag_values=fv)
    F.DEFINE_enum("mode", "a", ["a", "b"], "", flag_values=fv)
    return fv


def test_flag_forms():
    fv = _fv()
    rest = fv.parse(["prog", "--task_index=3", "--data_dir", "/x", "--nosync_replicas", "--learning_rate=1e-3",
                     "--hosts=a:1,b:2", "pos", "--mode=b"])
    assert fv.task_index == 3 and fv.data_dir == "/x" and fv.sync_replicas is False
    assert fv.learning_rate == pytest.approx(1e-3) and fv.hosts == ["a:1", "b:2"] and fv.mode == "b"
    assert rest == ["prog", "pos"]
    fv2 = _fv()
    fv2.parse(["p", "--sync_replicas=False"])
    assert fv2.sync_replicas is False
    fv3 = _fv()
    fv3.parse(["p", "--sync_replicas"])
    assert fv3.sync_replicas is True


def test_flag_errors():
    with pytest.raises(F.FlagError):
        _fv().parse(["p", "--nope=1"])
    with pytest.raises(F.FlagError):
        _fv().parse(["p", "--task_index=abc"])
    with pytest.raises(F.FlagError):
        _fv().parse(["p", "--mode=c"])


def test_reference_flag_defaults():
    """The 14 reference flags keep their names and defaults (mnist_python_m.py:49-87)."""
    from tensorflow_distributed_amd.training import dist_main

    dist_main.define_flags(1, "worker")
    f = F.FLAGS
    want = dict(data_dir="/tmp/mnist-data", download_only=False, task_index=1, num_gpus=0, replicas_to_aggregate=2,
                hidden_units=100, train_steps=4, batch_size=128, learning_rate=0.01, sync_replicas=True,
                existing_servers=False, ps_hosts="10.0.1.3:2222", worker_hosts="10.0.1.6:2223,10.0.1.2:2224",
                job_name="worker")
    for k, v in want.items():
        assert getattr(f, k) == v, k


def test_idx_roundtrip(tmp_path):
    a = (np.arange(3 * 28 * 28) % 256).astype(np.uint8).reshape(3, 28, 28)
    p = I.write_idx(str(tmp_path / "x-idx3-ubyte"), a)
    assert np.array_equal(I.read_idx(p[:-3]), a)
    p2 = I.write_idx(str(tmp_path / "y-idx1-ubyte"), np.array([1, 2, 3], np.uint8), compress=False)
    assert I.read_idx(p2).tolist() == [1, 2, 3]


def test_read_data_sets_splits_and_next_batch(tmp_path):
    I.write_idx_dataset(str(tmp_path), n_train=6000, n_test=1000)
    ds = I.read_data_sets(str(tmp_path), one_hot=True, validation_size=500, seed=0, verbose=False)
    assert ds.train.num_examples == 5500 and ds.validation.num_examples == 500 and ds.test.num_examples == 1000
    x, y = ds.train.next_batch(128)
    assert x.shape == (128, 784) and x.dtype == np.float32 and 0 <= x.min() and x.max() <= 1
    assert y.shape == (128, 10) and np.allclose(y.sum(1), 1)
    # one epoch of 500 in batches of 100 visits every validation example once
    seen = np.concatenate([ds.validation.next_batch(100)[1].argmax(1) for _ in range(5)])
    assert sorted(seen.tolist()) == sorted(ds.validation.label_ids.tolist())


def test_next_batch_epoch_boundary():
    imgs = np.arange(10 * 784, dtype=np.float32).reshape(10, 784) / (10 * 784)
    ds = I.DataSet(imgs, np.arange(10) % 10, one_hot=False, seed=1)
    got = [ds.next_batch(4)[1] for _ in range(3)]  # 4 + 4 + (2 old + 2 new)
    assert ds.epochs_completed == 1
    assert len(set(np.concatenate(got[:2]).tolist() + got[2][:2].tolist())) == 10


def test_synthetic_is_learnable_shape():
    x, y = I.synthetic_mnist(64, seed=3)
    assert x.shape == (64, 28, 28) and x.dtype == np.uint8 and y.max() <= 9
