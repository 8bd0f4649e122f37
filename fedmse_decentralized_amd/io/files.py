"""Open-file cache for the per-round artefacts.

Every round rewrites each trained client's ``model.cpt`` and
``training_tracking.pkl`` and appends one line to each JSONL report.  On the
overlay / ext4 filesystems of the GPU hosts, ``open(path, "wb")`` — a
truncate followed by re-allocating the blocks — costs ~130 us per file, which
made the background writer the slowest stage of a ~1.1 ms round.  Here files
stay open: a rewrite is one ``pwrite`` at offset 0 (plus ``ftruncate`` only
when the content got shorter — ``model.cpt`` has a fixed size for fixed
model dims), an append one ``write`` on an ``O_APPEND`` descriptor (~3 us
each).  The bytes on disk are exactly what ``open(..., "wb"/"a")`` would
leave.  Not thread-safe: owned by the single writer thread.

(The artefacts themselves are the reference's: ``model.cpt`` from
``save_model``, src/Trainer/client_trainer.py:340-345, and
``training_tracking.pkl``, :405-419, which the reference re-creates with
``open(..., "wb")`` on every write.)
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Dict, Tuple

FD_TABLE = 4096
_fd_table = 0


def reserve_fd_table(n: int = FD_TABLE) -> int:
    """Grow this process's descriptor table to ``n`` slots now (raising the
    soft RLIMIT_NOFILE towards the hard limit if needed); returns the slots
    available.

    Linux grows a process's descriptor table by doubling when an open needs
    a slot past its end, and in a multi-threaded process each growth waits
    for an RCU grace period.  In a process holding the GPU (many runtime
    threads) that wait measured 3.7 ms per open averaged over the 32 opens
    crossing a doubling and 124 ms at worst on the GPU hosts
    (``scripts/open_probe.py --gpu --hold``): the artefact writer's
    first-round file creations of a 64-client federation hit it at fds 64,
    128 and 256.  Growing the table once at import / setup (free while the
    process is single-threaded, one grace period otherwise) keeps every later
    open at ~6 us.  The table never shrinks."""
    global _fd_table
    if n <= _fd_table:
        return _fd_table
    try:
        import resource

        soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
        if soft != resource.RLIM_INFINITY and soft < n:
            lim = n if hard == resource.RLIM_INFINITY else min(n, hard)
            resource.setrlimit(resource.RLIMIT_NOFILE, (lim, hard))
            soft = lim
        top = n if soft == resource.RLIM_INFINITY else min(n, soft)
        fd = os.open(os.devnull, os.O_RDONLY)
        try:
            os.dup2(fd, top - 1)
            os.close(top - 1)
        finally:
            os.close(fd)
        _fd_table = top
    except (OSError, ValueError, ImportError):
        pass
    return _fd_table


class ArtifactFiles:
    def __init__(self, max_open: int = 512):
        reserve_fd_table()
        self.max_open = max_open
        self._fds: "OrderedDict[Tuple[str, str], int]" = OrderedDict()
        self._size: Dict[str, int] = {}
        self._maps: Dict[str, Tuple[int, int]] = {}   # path -> (address, size) of mapped files

    def _fd(self, path: str, mode: str) -> int:
        key = (path, mode)
        fd = self._fds.get(key)
        if fd is not None:
            self._fds.move_to_end(key)
            return fd
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if mode == "w":
            fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)   # read access: shared mappings
            self._size[path] = os.fstat(fd).st_size
        else:
            fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
        self._fds[key] = fd
        while len(self._fds) > self.max_open:
            (p, m), old = self._fds.popitem(last=False)
            os.close(old)
        return fd

    def overwrite(self, path: str, data: bytes) -> None:
        """File content becomes exactly ``data``."""
        fd = self._fd(path, "w")
        n = len(data)
        view = memoryview(data)
        off = 0
        while off < n:
            off += os.pwrite(fd, view[off:], off)
        if self._size.get(path, 0) > n:
            os.ftruncate(fd, n)
        self._size[path] = n

    def open_overwrite(self, path: str, reserve: int = 0) -> int:
        """Cached descriptor for in-place rewrites of ``path`` (for a native
        writer); ``reserve`` keeps that many descriptors from being evicted by
        the opens of one batch."""
        if reserve > self.max_open - 16:
            self.max_open = reserve + 16
        return self._fd(path, "w")

    def mapped(self, path: str, content: bytes) -> int:
        """Address of a shared writable mapping of ``path`` (a fixed-size file
        rewritten every round, e.g. model.cpt).  The first call for a path
        resizes the file to ``len(content)`` and writes ``content`` through the
        mapping; later calls return the same mapping, whose bytes the caller
        patches in place."""
        m = self._maps.get(path)
        if m is not None and m[1] == len(content):
            return m[0]
        from ..ops import _host

        if m is not None:
            _host.unmap_file(*m)
        fd = self._fd(path, "w")
        addr = _host.map_file(fd, len(content))
        import ctypes

        ctypes.memmove(addr, content, len(content))
        # the mapping keeps the file referenced: release the descriptor
        os.close(self._fds.pop((path, "w")))
        self._maps[path] = (addr, len(content))
        self._size[path] = len(content)
        return addr

    def size_of(self, path: str) -> int:
        return self._size.get(path, 0)

    def set_size(self, path: str, n: int) -> None:
        self._size[path] = int(n)

    def append(self, path: str, data: bytes) -> None:
        fd = self._fd(path, "a")
        view = memoryview(data)
        off = 0
        while off < len(data):
            off += os.write(fd, view[off:])

    def close(self) -> None:
        if self._maps:
            from ..ops import _host

            for addr, size in self._maps.values():
                _host.unmap_file(addr, size)
            self._maps.clear()
        for fd in self._fds.values():
            os.close(fd)
        self._fds.clear()
        self._size.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
