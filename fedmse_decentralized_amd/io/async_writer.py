"""Background artefact writer.

The reference writes ``model.cpt`` on every validation improvement and the
tracking pickle every epoch from inside the training loop, and appends the
JSONL reports synchronously (`src/Trainer/client_trainer.py:408-419`,
`src/main.py:313-355`).  Here file I/O never sits on the round's critical
path: device snapshots are copied to pinned host memory asynchronously, and a
single writer thread (which preserves per-file append order) waits on the
copy's event and writes the file while the next round already runs.
``flush()`` is called at the end of every sweep combination.
"""
from __future__ import annotations

import queue
import threading
import time
import traceback
from typing import Callable, Optional

import torch

from .files import ArtifactFiles


class AsyncWriter:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled
        self.q: "queue.Queue" = queue.Queue()
        self.errors = []
        self.files = ArtifactFiles()   # used only from the job context (writer thread)
        self.busy_s = 0.0   # time spent running jobs (telemetry)
        self.jobs = 0
        self.t: Optional[threading.Thread] = None
        if enabled:
            self.t = threading.Thread(target=self._run, name="fedmx-writer", daemon=True)
            self.t.start()

    def _run(self):
        while True:
            job = self.q.get()
            if job is None:
                self.q.task_done()
                return
            event, fn = job
            try:
                if event is not None:
                    event.synchronize()
                t0 = time.perf_counter()
                fn()
                self.busy_s += time.perf_counter() - t0
                self.jobs += 1
            except Exception:  # pragma: no cover - surfaced by flush()
                self.errors.append(traceback.format_exc())
            finally:
                self.q.task_done()

    def submit(self, fn: Callable[[], None], event: Optional["torch.cuda.Event"] = None):
        if not self.enabled:
            if event is not None:
                event.synchronize()
            fn()
            return
        self.q.put((event, fn))

    def flush(self):
        if self.enabled:
            self.q.join()
        # the queue is drained (no job running): release the cached
        # descriptors, so files deleted or replaced between sweeps are reopened
        self.files.close()
        if self.errors:
            errs, self.errors = self.errors, []
            raise RuntimeError("artefact writer failed:\n" + "\n".join(errs))

    def close(self):
        if self.enabled and self.t is not None:
            self.flush()
            self.q.put(None)
            self.t.join()
            self.t = None
        self.files.close()


def snapshot_to_host(t: torch.Tensor):
    """Async device->pinned copy; returns (host tensor, event or None)."""
    if t.device.type == "cpu":
        return t.detach().clone(), None
    host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)   # caching host allocator
    host.copy_(t, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    return host, ev
