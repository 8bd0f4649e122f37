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
            L.fedmx_pickle_tracking.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64]
            L.fedmx_pickle_tracking.restype = ctypes.c_int64
            L.fedmx_write_artifacts.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                                ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                                ctypes.c_int32] + [ctypes.c_void_p] * 7 + [ctypes.c_int32,
                                                                                          ctypes.c_void_p,
                                                                                          ctypes.c_int32]
            L.fedmx_writer_create.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                              ctypes.c_void_p, ctypes.c_int64]
            L.fedmx_writer_create.restype = ctypes.c_void_p
            L.fedmx_writer_submit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
            L.fedmx_writer_submit.restype = ctypes.c_int64
            L.fedmx_writer_wait.argtypes = [ctypes.c_void_p, ctypes.c_int64]
            L.fedmx_writer_wait.restype = ctypes.c_int32
            L.fedmx_store_fence.argtypes = []
            L.fedmx_store_fence.restype = None
            L.fedmx_writer_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            L.fedmx_writer_stats.restype = None
            L.fedmx_writer_flush.argtypes = [ctypes.c_void_p]
            L.fedmx_writer_flush.restype = ctypes.c_int32
            L.fedmx_writer_destroy.argtypes = [ctypes.c_void_p]
            L.fedmx_writer_destroy.restype = None
            L.fedmx_map_file.argtypes = [ctypes.c_int32, ctypes.c_int64]
            L.fedmx_map_file.restype = ctypes.c_void_p
            L.fedmx_unmap_file.argtypes = [ctypes.c_void_p, ctypes.c_int64]
            L.fedmx_unmap_file.restype = ctypes.c_int32
            L.fedmx_write_artifacts.restype = ctypes.c_int32
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


def pickle_tracking(tracking) -> bytes:
    """pickle.dumps([(train, valid), ...], protocol=4), rendered natively."""
    t = np.ascontiguousarray(np.asarray(tracking, dtype=np.float64).reshape(-1, 2))
    cap = 16 + 20 * t.shape[0]
    out = np.empty(cap, dtype=np.uint8)
    n = lib().fedmx_pickle_tracking(t.ctypes.data, t.shape[0], out.ctypes.data, cap)
    if n < 0:
        raise ValueError("tracking too long for the native pickler")
    return out[:n].tobytes()


def map_file(fd: int, size: int) -> int:
    """Shared writable mapping of ``fd`` resized to ``size`` bytes (address)."""
    p = lib().fedmx_map_file(fd, size)
    if not p:
        raise OSError(f"cannot map artefact file (fd {fd}, {size} bytes)")
    return int(p)


def unmap_file(addr: int, size: int) -> None:
    lib().fedmx_unmap_file(addr, size)


def write_artifacts(snap: np.ndarray, canon_idx: np.ndarray, tpl: np.ndarray, regions: np.ndarray,
                    rows: np.ndarray, improved: np.ndarray, cpt_dst: np.ndarray, fd_trk: np.ndarray,
                    size_trk: np.ndarray, trk: np.ndarray, trk_len: np.ndarray,
                    n_threads: int = 1) -> np.ndarray:
    """One round's model.cpt + training_tracking.pkl files (see
    csrc/host/fedmx_artifacts.cpp): parameters patched into the mapped
    model.cpt files at ``cpt_dst`` (addresses), tracking pickles written into
    ``fd_trk``.  ``size_trk`` is updated in place; returns the per-job status
    (0 = written)."""
    n = int(rows.shape[0])
    status = np.zeros(n, dtype=np.int32)
    assert snap.dtype == np.float32 and snap.flags.c_contiguous and trk.dtype == np.float64
    assert trk.shape[0] >= n and trk.shape[2] == 2 and trk.flags.c_contiguous
    lib().fedmx_write_artifacts(
        snap.ctypes.data, snap.shape[1], canon_idx.ctypes.data, canon_idx.shape[0],
        tpl.ctypes.data, tpl.shape[0], regions.ctypes.data, regions.shape[0], n,
        rows.ctypes.data, improved.ctypes.data, cpt_dst.ctypes.data, fd_trk.ctypes.data,
        size_trk.ctypes.data, trk.ctypes.data, trk_len.ctypes.data, trk.shape[1],
        status.ctypes.data, n_threads)
    return status
