"""TensorFlow-V2-bundle-compatible checkpoints (reference: the Supervisor's implicit ``Saver``,
``/root/reference/mnist_python_m.py:235-253``).

Files written under ``logdir`` (same names the reference's Supervisor produces):

* ``model.ckpt-<step>.data-00000-of-00001`` -- raw little-endian tensor bytes, concatenated.
* ``model.ckpt-<step>.index`` -- a LevelDB-format SSTable whose keys are tensor names (sorted) and
  whose values are serialized ``BundleEntryProto`` (dtype, shape, shard, offset, size, masked
  crc32c); the empty key holds the ``BundleHeaderProto``.
* ``checkpoint`` -- the text-format ``CheckpointState`` pointing at the latest prefix.

Protos and the table format are encoded by hand (no TensorFlow / protobuf dependency): varint
fields, prefix-compressed data blocks with restart points, per-block ``type + masked crc32c``
trailers, an index block, an empty metaindex block and the 48-byte footer with the table magic.
CRC32-C comes from the native library (SSE4.2) when loaded, else a table-driven fallback.
Parity note: no TensorFlow is installed here, so byte-compatibility with ``tf.train.Saver`` is
"parity unpinned" -- the reader below is the round-trip oracle and the encoder follows the
published LevelDB table / tensor_bundle.proto layouts.
"""
from __future__ import annotations

import os
import re
import struct
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import numpy as np

# ----------------------------------------------------------------------------- crc32c
_TABLE = None


def _crc_table():
    global _TABLE
    if _TABLE is None:
        t = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            t.append(c)
        _TABLE = t
    return _TABLE


def crc32c(data: bytes, init: int = 0) -> int:
    try:
        import torch

        from .. import _native

        if _native.load(build_if_missing=False):
            t = torch.frombuffer(bytearray(data), dtype=torch.uint8) if len(data) else torch.zeros(0, dtype=torch.uint8)
            return int(torch.ops.tfd.crc32c(t, init)) & 0xFFFFFFFF
    except Exception:  # pragma: no cover - fallback when the native lib is unavailable
        pass
    tab = _crc_table()
    c = init ^ 0xFFFFFFFF
    for b in data:
        c = tab[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def mask_crc(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def unmask_crc(m: int) -> int:
    r = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# ----------------------------------------------------------------------------- proto wire format
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, pos: int) -> Tuple[int, int]:
    shift = 0
    v = 0
    while True:
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7


def _field_varint(num: int, v: int) -> bytes:
    return _varint(num << 3 | 0) + _varint(v)


def _field_bytes(num: int, b: bytes) -> bytes:
    return _varint(num << 3 | 2) + _varint(len(b)) + b


def _field_fixed32(num: int, v: int) -> bytes:
    return _varint(num << 3 | 5) + struct.pack("<I", v)


def _parse_fields(buf: bytes) -> List[Tuple[int, int, object]]:
    out = []
    pos = 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            v = buf[pos:pos + n]
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        else:
            raise ValueError(f"unsupported wire type {wt}")
        out.append((num, wt, v))
    return out


# tensorflow/core/framework/types.proto
_DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.uint8): 4,
       np.dtype(np.int16): 5, np.dtype(np.int8): 6, np.dtype(np.int64): 9, np.dtype(np.bool_): 10,
       np.dtype(np.float16): 19}
_DT_INV = {v: k for k, v in _DT.items()}
_DT_BFLOAT16 = 14


def _shape_proto(shape) -> bytes:
    return b"".join(_field_bytes(2, _field_varint(1, int(d))) for d in shape)


def _entry_proto(dtype: int, shape, offset: int, size: int, crc: int) -> bytes:
    b = _field_varint(1, dtype) + _field_bytes(2, _shape_proto(shape))
    # shard_id (3) = 0 is the default and omitted
    if offset:
        b += _field_varint(4, offset)
    b += _field_varint(5, size) + _field_fixed32(6, crc)
    return b


def _header_proto(num_shards: int = 1) -> bytes:
    version = _field_varint(1, 1)  # VersionDef{producer: 1}
    return _field_varint(1, num_shards) + _field_bytes(3, version)  # endianness LITTLE (0) omitted


def _parse_entry(buf: bytes) -> dict:
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": 0}
    for num, _, v in _parse_fields(buf):
        if num == 1:
            e["dtype"] = v
        elif num == 2:
            for n2, _, v2 in _parse_fields(v):
                if n2 == 2:
                    size = 0
                    for n3, _, v3 in _parse_fields(v2):
                        if n3 == 1:
                            size = v3
                    e["shape"].append(size)
        elif num == 3:
            e["shard_id"] = v
        elif num == 4:
            e["offset"] = v
        elif num == 5:
            e["size"] = v
        elif num == 6:
            e["crc32c"] = v
    return e


# ----------------------------------------------------------------------------- LevelDB table
_TABLE_MAGIC = 0xDB4775248B80FB57
_BLOCK_SIZE = 4096
_RESTART_INTERVAL = 16


class _BlockBuilder:
    def __init__(self):
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last_key = b""

    def add(self, key: bytes, value: bytes):
        shared = 0
        if self.counter < _RESTART_INTERVAL:
            m = min(len(key), len(self.last_key))
            while shared < m and key[shared] == self.last_key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        self.buf += _varint(shared) + _varint(len(key) - shared) + _varint(len(value))
        self.buf += key[shared:] + value
        self.last_key = key
        self.counter += 1

    def size(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4

    def empty(self) -> bool:
        return len(self.buf) == 0

    def finish(self) -> bytes:
        return bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts) + struct.pack("<I", len(self.restarts))


def _write_block(f, contents: bytes, offset: int) -> Tuple[bytes, int]:
    trailer = b"\x00" + struct.pack("<I", mask_crc(crc32c(contents + b"\x00")))
    f.write(contents)
    f.write(trailer)
    handle = _varint(offset) + _varint(len(contents))
    return handle, offset + len(contents) + 5


def write_sstable(path: str, items: List[Tuple[bytes, bytes]]) -> None:
    """Write sorted (key, value) pairs as a LevelDB table (no compression)."""
    keys = [k for k, _ in items]
    assert keys == sorted(keys) and len(set(keys)) == len(keys), "keys must be unique and sorted"
    with open(path, "wb") as f:
        off = 0
        index = _BlockBuilder()
        blk = _BlockBuilder()
        last_key = None
        for k, v in items:
            blk.add(k, v)
            last_key = k
            if blk.size() >= _BLOCK_SIZE:
                handle, off = _write_block(f, blk.finish(), off)
                index.add(last_key, handle)
                blk = _BlockBuilder()
        if not blk.empty():
            handle, off = _write_block(f, blk.finish(), off)
            index.add(last_key, handle)
        meta_handle, off = _write_block(f, _BlockBuilder().finish(), off)
        index_handle, off = _write_block(f, index.finish(), off)
        footer = meta_handle + index_handle
        footer += b"\x00" * (40 - len(footer))
        footer += struct.pack("<Q", _TABLE_MAGIC)
        f.write(footer)


def _read_block(data: bytes, handle: bytes, verify: bool = True) -> bytes:
    off, p = _read_varint(handle, 0)
    size, _ = _read_varint(handle, p)
    contents = data[off:off + size]
    typ = data[off + size]
    if typ != 0:
        raise ValueError("compressed table blocks are not supported")
    if verify:
        crc = struct.unpack_from("<I", data, off + size + 1)[0]
        if unmask_crc(crc) != crc32c(contents + bytes([typ])):
            raise ValueError("table block checksum mismatch")
    return contents


def _block_entries(block: bytes) -> List[Tuple[bytes, bytes]]:
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrest
    out = []
    pos = 0
    last = b""
    while pos < end:
        shared, pos = _read_varint(block, pos)
        nonshared, pos = _read_varint(block, pos)
        vlen, pos = _read_varint(block, pos)
        key = last[:shared] + block[pos:pos + nonshared]
        pos += nonshared
        val = block[pos:pos + vlen]
        pos += vlen
        out.append((key, val))
        last = key
    return out


def read_sstable(path: str) -> List[Tuple[bytes, bytes]]:
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 48 or struct.unpack_from("<Q", data, len(data) - 8)[0] != _TABLE_MAGIC:
        raise ValueError(f"{path}: not an SSTable")
    footer = data[len(data) - 48:len(data) - 8]
    _, p = _read_varint(footer, 0)
    _, p = _read_varint(footer, p)  # metaindex handle
    idx_off, q = _read_varint(footer, p)
    idx_size, _ = _read_varint(footer, q)
    index = _read_block(data, _varint(idx_off) + _varint(idx_size))
    items = []
    for _, handle in _block_entries(index):
        items.extend(_block_entries(_read_block(data, handle)))
    return items


# ----------------------------------------------------------------------------- bundle API
def _as_numpy(t) -> np.ndarray:
    try:
        import torch

        if isinstance(t, torch.Tensor):
            t = t.detach().cpu()
            if t.dtype == torch.bfloat16:
                t = t.float()
            return t.numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(t)


def save_bundle(prefix: str, tensors: "OrderedDict[str, object]") -> None:
    """Write ``prefix.index`` + ``prefix.data-00000-of-00001`` holding ``tensors`` (name -> array)."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    data_path = prefix + ".data-00000-of-00001"
    entries = []
    off = 0
    tmp_data = data_path + ".tmp"
    with open(tmp_data, "wb") as f:
        for name in sorted(tensors):
            arr = _as_numpy(tensors[name])
            arr = arr if arr.flags.c_contiguous else arr.copy(order="C")  # (ascontiguousarray makes 0-d 1-d)
            if arr.dtype not in _DT:
                raise TypeError(f"{name}: unsupported dtype {arr.dtype}")
            raw = arr.astype(arr.dtype.newbyteorder("<"), copy=False).tobytes()
            f.write(raw)
            entries.append((name.encode(), _entry_proto(_DT[arr.dtype], arr.shape, off, len(raw),
                                                        mask_crc(crc32c(raw)))))
            off += len(raw)
    items = [(b"", _header_proto())] + entries
    tmp_index = prefix + ".index.tmp"
    write_sstable(tmp_index, items)
    os.replace(tmp_data, data_path)
    os.replace(tmp_index, prefix + ".index")


def load_bundle(prefix: str, verify: bool = True) -> "OrderedDict[str, np.ndarray]":
    items = read_sstable(prefix + ".index")
    header = None
    out = OrderedDict()
    shards = {}
    for key, val in items:
        if key == b"":
            header = dict((n, v) for n, _, v in _parse_fields(val))
            continue
        e = _parse_entry(val)
        sid = e["shard_id"]
        if sid not in shards:
            nsh = header.get(1, 1) if header else 1
            with open(f"{prefix}.data-{sid:05d}-of-{nsh:05d}", "rb") as f:
                shards[sid] = f.read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        if verify and unmask_crc(e["crc32c"]) != crc32c(raw):
            raise ValueError(f"checksum mismatch for tensor {key.decode()}")
        if e["dtype"] == _DT_BFLOAT16:
            u = np.frombuffer(raw, dtype="<u2").astype(np.uint32) << 16
            arr = u.view(np.float32)
        else:
            arr = np.frombuffer(raw, dtype=_DT_INV[e["dtype"]].newbyteorder("<"))
        out[key.decode()] = arr.reshape(e["shape"]).copy()
    return out


def list_variables(prefix: str) -> List[Tuple[str, List[int]]]:
    """``tf.train.list_variables`` analogue."""
    return [(k.decode(), _parse_entry(v)["shape"]) for k, v in read_sstable(prefix + ".index") if k]


# ----------------------------------------------------------------------------- CheckpointState
def write_checkpoint_state(logdir: str, latest: str, all_paths: List[str]) -> None:
    lines = [f'model_checkpoint_path: "{latest}"'] + [f'all_model_checkpoint_paths: "{p}"' for p in all_paths]
    tmp = os.path.join(logdir, "checkpoint.tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(logdir, "checkpoint"))


def read_checkpoint_state(logdir: str) -> Optional[dict]:
    p = os.path.join(logdir, "checkpoint")
    if not os.path.exists(p):
        return None
    st = {"model_checkpoint_path": None, "all_model_checkpoint_paths": []}
    with open(p) as f:
        for line in f:
            m = re.match(r'\s*(\w+)\s*:\s*"(.*)"\s*$', line)
            if not m:
                continue
            if m.group(1) == "model_checkpoint_path":
                st["model_checkpoint_path"] = m.group(2)
            elif m.group(1) == "all_model_checkpoint_paths":
                st["all_model_checkpoint_paths"].append(m.group(2))
    return st


def latest_checkpoint(logdir: str) -> Optional[str]:
    """``tf.train.latest_checkpoint``: absolute prefix of the newest checkpoint, or None."""
    st = read_checkpoint_state(logdir)
    if not st or not st["model_checkpoint_path"]:
        return None
    p = st["model_checkpoint_path"]
    if not os.path.isabs(p):
        p = os.path.join(logdir, p)
    return p if os.path.exists(p + ".index") else None


class Saver:
    """``tf.train.Saver``-style saver over a name -> tensor mapping, keeping ``max_to_keep`` files."""

    def __init__(self, max_to_keep: int = 5, basename: str = "model.ckpt"):
        self.max_to_keep = max_to_keep
        self.basename = basename
        self._kept: List[str] = []

    def save(self, logdir: str, tensors: "OrderedDict[str, object]", global_step: Optional[int] = None) -> str:
        os.makedirs(logdir, exist_ok=True)
        name = self.basename if global_step is None else f"{self.basename}-{int(global_step)}"
        prefix = os.path.join(logdir, name)
        save_bundle(prefix, tensors)
        st = read_checkpoint_state(logdir)
        kept = [p for p in (st["all_model_checkpoint_paths"] if st else []) if p != name] + [name]
        while self.max_to_keep and len(kept) > self.max_to_keep:
            old = kept.pop(0)
            for suffix in (".index", ".data-00000-of-00001", ".meta"):
                q = os.path.join(logdir, old + suffix)
                if os.path.exists(q):
                    os.remove(q)
        write_checkpoint_state(logdir, name, kept)
        return prefix

    def restore(self, prefix: str) -> "OrderedDict[str, np.ndarray]":
        return load_bundle(prefix)
