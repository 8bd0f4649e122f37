"""ctypes bindings of ``libfedmx_host.so`` (CSV reader, exact host AUC)."""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

from . import build

_lock = threading.Lock()
_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            path = build.build_host()  # no-op when up to date (g++ only, no GPU toolchain)
            L = ctypes.CDLL(str(path))
            L.fedmx_csv_shape.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
            L.fedmx_csv_shape.restype = ctypes.c_int
            L.fedmx_csv_parse.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
            L.fedmx_csv_parse.restype = ctypes.c_int64
            L.fedmx_roc_auc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
            L.fedmx_roc_auc.restype = ctypes.c_double
            _lib = L
    return _lib


def read_csv(path: str, nthreads: int = 0) -> np.ndarray:
    """Headerless numeric CSV -> float64 [rows, cols]."""
    L = lib()
    r = ctypes.c_int64()
    c = ctypes.c_int64()
    if L.fedmx_csv_shape(path.encode(), ctypes.byref(r), ctypes.byref(c)) != 0:
        raise OSError(f"cannot read {path}")
    out = np.empty((r.value, c.value), dtype=np.float64)
    if r.value == 0:
        return out
    if nthreads <= 0:
        nthreads = max(1, min(8, os.cpu_count() or 1))
    got = L.fedmx_csv_parse(path.encode(), out.ctypes.data, r.value, c.value, nthreads)
    if got != r.value:
        raise ValueError(f"malformed CSV {path} (code {got})")
    return out


def roc_auc(score: np.ndarray, label: np.ndarray) -> float:
    s = np.ascontiguousarray(score, dtype=np.float64)
    y = np.ascontiguousarray(label, dtype=np.int64)
    return float(lib().fedmx_roc_auc(s.ctypes.data, y.ctypes.data, s.shape[0]))
