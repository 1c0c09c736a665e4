"""TensorBoard-compatible event files (the Supervisor's summary / ``global_step/sec`` services,
``/root/reference/mnist_python_m.py:239-253`` [TF1-lib]).

``events.out.tfevents.<time>.<host>`` is a TFRecord stream: per record ``uint64 len``,
``masked crc32c(len)``, the serialized ``Event`` proto, ``masked crc32c(data)``. Events carry
``wall_time`` (1, double), ``step`` (2, int64) and either ``file_version`` (3) or a ``Summary`` (5)
of ``{tag (1), simple_value (2, float)}`` values -- encoded by hand, no TensorFlow dependency.
"""
from __future__ import annotations

import os
import socket
import struct
import threading
import time
from typing import Dict, Iterator, List, Optional, Tuple

from .checkpoint import _field_bytes, _field_varint, _parse_fields, crc32c, mask_crc, unmask_crc


def _event(wall_time: float, step: int, payload: bytes) -> bytes:
    return _varint_key_double(1, wall_time) + _field_varint(2, step) + payload


def _varint_key_double(num: int, v: float) -> bytes:
    return bytes([num << 3 | 1]) + struct.pack("<d", v)


def _summary_value(tag: str, value: float) -> bytes:
    return _field_bytes(1, tag.encode()) + bytes([2 << 3 | 5]) + struct.pack("<f", float(value))


def encode_record(data: bytes) -> bytes:
    ln = struct.pack("<Q", len(data))
    return ln + struct.pack("<I", mask_crc(crc32c(ln))) + data + struct.pack("<I", mask_crc(crc32c(data)))


class EventFileWriter:
    """``tf.summary.FileWriter`` subset: scalar summaries, flushed per write (thread-safe)."""

    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{filename_suffix}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "wb")
        self._lock = threading.Lock()
        self._write(_event(time.time(), 0, _field_bytes(3, b"brain.Event:2")))

    def _write(self, ev: bytes):
        with self._lock:
            if self._f is None:
                return
            self._f.write(encode_record(ev))
            self._f.flush()

    def add_scalars(self, values: Dict[str, float], step: int, wall_time: Optional[float] = None):
        summ = b"".join(_field_bytes(1, _summary_value(k, v)) for k, v in values.items())
        self._write(_event(wall_time or time.time(), int(step), _field_bytes(5, summ)))

    def add_scalar(self, tag: str, value: float, step: int, wall_time: Optional[float] = None):
        self.add_scalars({tag: value}, step, wall_time)

    def close(self):
        with self._lock:
            if self._f is not None:
                self._f.close()
                self._f = None


def read_records(path: str, verify: bool = True) -> Iterator[bytes]:
    with open(path, "rb") as f:
        buf = f.read()
    pos = 0
    while pos + 12 <= len(buf):
        ln = struct.unpack_from("<Q", buf, pos)[0]
        if verify and unmask_crc(struct.unpack_from("<I", buf, pos + 8)[0]) != crc32c(buf[pos:pos + 8]):
            raise ValueError("record length checksum mismatch")
        data = buf[pos + 12:pos + 12 + ln]
        if verify and unmask_crc(struct.unpack_from("<I", buf, pos + 12 + ln)[0]) != crc32c(data):
            raise ValueError("record data checksum mismatch")
        yield data
        pos += 16 + ln


def read_scalars(path: str) -> List[Tuple[int, str, float]]:
    """(step, tag, value) for every scalar summary in an event file."""
    out = []
    for rec in read_records(path):
        step = 0
        summ = None
        for num, wt, v in _parse_fields(rec):
            if num == 2:
                step = v
            elif num == 5:
                summ = v
        if summ is None:
            continue
        for num, _, val in _parse_fields(summ):
            if num != 1:
                continue
            tag, sv = None, None
            for n2, _, v2 in _parse_fields(val):
                if n2 == 1:
                    tag = v2.decode()
                elif n2 == 2:
                    sv = struct.unpack("<f", struct.pack("<I", v2))[0]
            out.append((step, tag, sv))
    return out
