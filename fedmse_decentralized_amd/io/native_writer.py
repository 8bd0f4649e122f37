"""Native asynchronous checkpoint writer (``ops/csrc/host/fedmx_artifacts.cpp``).

Each round's ``model.cpt`` + ``training_tracking.pkl`` files of the trained
clients (`src/Trainer/client_trainer.py:337-358`) are written by a C++ thread:
``submit`` (main thread) copies the job's small arrays and paths and returns a
ticket at once, with no system call; the C++ thread opens / creates the files
(kept open, ``model.cpt`` kept mapped), patches the parameters into the mapped
``model.cpt`` files and writes the tracking pickles without touching Python,
so it never waits for the GIL and the main thread never waits for the
filesystem (file creation on the GPU hosts' filesystem costs ~1 ms each);
``wait(ticket)`` blocks (GIL released) until that job is on disk — the
snapshot slot it read may then be reused.

The device-resident round protocol (``engine/device_round.py``) uses it: its
snapshots live in a mapped host ring that the GPU fills and the writer reads.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence, Tuple

import numpy as np

from ..models.layout import DEFAULT_DIMS, ModelDims, padded_index
from . import checkpoint as ckpt
from .files import ArtifactFiles, reserve_fd_table

_MAX_NATIVE_EPOCHS = 1000   # the native pickler's single-batch limit


class NativeCheckpointWriter:
    def __init__(self, dims: ModelDims = DEFAULT_DIMS):
        from ..ops import _host

        self._lib = _host.lib()
        reserve_fd_table()   # the writer thread keeps every client's files open
        self.dims = dims
        self.tpl = ckpt._template(dims)
        self.cidx = np.ascontiguousarray(padded_index(dims)[0].numpy(), dtype=np.int32)
        blob = np.frombuffer(self.tpl.blob_bytes, dtype=np.uint8)
        self.h = self._lib.fedmx_writer_create(self.cidx.ctypes.data, self.cidx.shape[0],
                                               self.tpl.np_regions.ctypes.data, self.tpl.np_regions.shape[0],
                                               blob.ctypes.data, blob.shape[0])
        self._paths = {}
        self.last = 0

    def submit(self, save_dirs: Sequence[str], snap: np.ndarray, rows: Sequence[int], improved: Sequence[bool],
               tracking: Sequence[Sequence[Tuple[float, float]]]) -> int:
        """Queue one round's files; ``snap`` (float32 [rows, P_PAD]) must stay
        valid until ``wait`` of the returned ticket."""
        n = len(save_dirs)
        if n == 0:
            return self.last
        if any(len(t) > _MAX_NATIVE_EPOCHS for t in tracking):
            self.flush()
            files = ArtifactFiles()
            try:
                ckpt.write_round_artifacts(files, save_dirs, snap, rows, improved, tracking, self.cidx, self.dims)
            finally:
                files.close()
            return self.last
        paths = b"".join(self._path_bytes(d) for d in save_dirs)
        lens = np.asarray([len(t) for t in tracking], dtype=np.int32)
        width = max(1, int(lens.max(initial=0)))
        trk = np.zeros((n, width, 2), dtype=np.float64)
        for j, t in enumerate(tracking):
            if len(t):
                trk[j, :len(t)] = np.asarray(t, dtype=np.float64).reshape(-1, 2)
        snap = np.asarray(snap)
        assert snap.dtype == np.float32 and snap.flags.c_contiguous
        rows_a = np.asarray(rows, dtype=np.int32)
        imp_a = np.asarray(improved, dtype=np.int32)
        t = int(self._lib.fedmx_writer_submit(
            self.h, snap.ctypes.data, snap.shape[1], n, rows_a.ctypes.data, imp_a.ctypes.data, paths, len(paths),
            trk.ctypes.data, lens.ctypes.data, width))
        if t < 0:
            raise ValueError("native checkpoint writer: malformed path list")
        self.last = t
        return t

    def _path_bytes(self, save_dir: str) -> bytes:
        b = self._paths.get(save_dir)
        if b is None:
            pc, pt = ckpt._artifact_paths(save_dir)
            b = self._paths[save_dir] = os.fsencode(pc) + b"\0" + os.fsencode(pt) + b"\0"
        return b

    def stats(self) -> dict:
        """The writer thread's own clock (ms) per phase, jobs and files opened."""
        out = np.zeros(6, dtype=np.float64)
        if self.h:
            self._lib.fedmx_writer_stats(self.h, out.ctypes.data)
        return {"open_ms": round(out[0], 3), "first_map_ms": round(out[1], 3), "patch_ms": round(out[2], 3),
                "tracking_ms": round(out[3], 3), "jobs": int(out[4]), "files_opened": int(out[5])}

    def wait(self, ticket: int) -> None:
        rc = self._lib.fedmx_writer_wait(self.h, ticket)
        if rc:
            raise OSError(-rc if rc < 0 else rc, "native checkpoint writer failed")

    def flush(self) -> None:
        """Every queued job written; the writer thread's descriptors and
        mappings released."""
        rc = self._lib.fedmx_writer_flush(self.h)
        if rc:
            raise OSError(-rc if rc < 0 else rc, "native checkpoint writer failed")

    def close(self) -> None:
        if self.h:
            self.flush()
            self._lib.fedmx_writer_destroy(ctypes.c_void_p(self.h))
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
