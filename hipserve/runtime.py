"""Loader for the native CPU runtime extension (``hipserve/_runtime*.so``).

Built in-tree by ``python -m hipserve._build`` (g++ + pybind11). If the module is
missing it is built on first use — it is host C++ only, so this works on any box
of this image (CPU container or GPU node) in a couple of seconds.
"""
from __future__ import annotations

import importlib
import threading

_mod = None
_lock = threading.Lock()


def native():
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            try:
                _mod = importlib.import_module("hipserve._runtime")
            except ImportError:
                from ._build import build_runtime

                build_runtime(verbose=False)
                importlib.invalidate_caches()
                _mod = importlib.import_module("hipserve._runtime")
    return _mod
