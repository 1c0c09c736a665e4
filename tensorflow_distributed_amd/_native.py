"""Loader for the in-tree native library ``_C.so`` (HIP kernels + RCCL comm + C++ executors).

On a GPU box the native path is mandatory: :func:`require` raises loudly when the extension is
missing or failed to load, so nothing silently falls back to eager PyTorch. On the CPU-only build
container the library still loads (it is host code + gfx950 code objects) and CPU-side ops such
as ``crc32c`` work.
"""
from __future__ import annotations

import os
import threading

import torch

_LIB = os.environ.get("TFD_NATIVE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_C.so")
_lock = threading.Lock()
_loaded = False
_error: Exception | None = None


def lib_path() -> str:
    return _LIB


def load(build_if_missing: bool = True) -> bool:
    """Load ``_C.so`` into the process (registers ``torch.ops.tfd`` / ``torch.classes.tfd``)."""
    global _loaded, _error
    with _lock:
        if _loaded:
            return True
        try:
            if not os.path.exists(_LIB) and build_if_missing and os.environ.get("TFD_NO_AUTOBUILD") != "1":
                from . import _build

                _build.build()
            torch.ops.load_library(_LIB)
            _loaded = True
        except Exception as e:  # pragma: no cover - exercised only when the build is broken
            _error = e
            _loaded = False
        return _loaded


def available() -> bool:
    return load()


def require() -> None:
    """Raise if the native library is not usable. Called by every GPU code path."""
    if not load():
        raise RuntimeError(f"tensorflow_distributed_amd native library failed to load from {_LIB}: {_error!r}. "
                           "Build it with `python -m tensorflow_distributed_amd._build`.")


def gpu_available() -> bool:
    return torch.cuda.is_available()


def ops():
    require()
    return torch.ops.tfd


def classes():
    require()
    return torch.classes.tfd
