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

import os
import queue
import sys
import threading
import time
import traceback
from typing import Callable, Optional

import torch

from .files import ArtifactFiles


SWITCH_INTERVAL_S = 1e-4


class AsyncWriter:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled
        self.q: "queue.Queue" = queue.Queue()
        self.errors = []
        self.files = ArtifactFiles()   # used only from the job context (writer thread)
        self.busy_s = 0.0   # time spent running jobs (telemetry)
        self._busy_mark = 0.0
        self._prev_switch = None
        # FEDMX_WRITER_STATS=1: per job kind (count, seconds), printed by close()
        self.stats = {} if os.environ.get("FEDMX_WRITER_STATS") == "1" else None
        self.jobs = 0
        self.t: Optional[threading.Thread] = None
        self.native = None   # NativeCheckpointWriter (device-round checkpoints), created on first use
        if enabled:
            # The writer's jobs release the GIL inside native calls and must
            # take it back afterwards from a main thread that runs Python
            # (enqueueing rounds) almost without pause: at CPython's default
            # 5 ms switch interval every such hand-back cost up to 5 ms, which
            # made the writer — not the GPU — bound large federations (64
            # clients: 4.3 ms writer time per round for ~0.2 ms of work).
            # (restored by close())
            if sys.getswitchinterval() > SWITCH_INTERVAL_S:
                self._prev_switch = sys.getswitchinterval()
                sys.setswitchinterval(SWITCH_INTERVAL_S)
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
                dt = time.perf_counter() - t0
                self.busy_s += dt
                self.jobs += 1
                if self.stats is not None:
                    k = getattr(fn, "__qualname__", type(fn).__name__)
                    n, tot = self.stats.get(k, (0, 0.0))
                    self.stats[k] = (n + 1, tot + dt)
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

    def mark(self) -> None:
        """Start of a timed region: ``busy_s_timed`` counts job time from here."""
        self._busy_mark = self.busy_s

    @property
    def busy_s_timed(self) -> float:
        return self.busy_s - self._busy_mark

    def native_ckpt(self, dims):
        """The process's native checkpoint writer (io.native_writer)."""
        if self.native is None:
            from .native_writer import NativeCheckpointWriter

            self.native = NativeCheckpointWriter(dims)
        return self.native

    def flush(self):
        if self.native is not None:
            self.native.flush()
        if self.enabled:
            self.q.join()
        # the queue is drained (no job running): release the cached
        # descriptors, so files deleted or replaced between sweeps are reopened
        self.files.close()
        if self.errors:
            errs, self.errors = self.errors, []
            raise RuntimeError("artefact writer failed:\n" + "\n".join(errs))

    def report_stats(self):
        """FEDMX_WRITER_STATS=1: per job kind count / total / mean time on stderr."""
        if self.stats:
            print("writer job stats (count, total ms, us/job):", file=sys.stderr)
            for k, (n, tot) in sorted(self.stats.items(), key=lambda kv: -kv[1][1]):
                print(f"  {k}: {n} {1e3 * tot:.1f} {1e6 * tot / n:.1f}", file=sys.stderr)
            from .checkpoint import WRITE_STATS
            if WRITE_STATS:
                print(f"  write_round_artifacts: {WRITE_STATS}", file=sys.stderr)
            if self.native is not None:
                print(f"  native writer thread: {self.native.stats()}", file=sys.stderr)

    def close(self):
        if self.enabled and self.t is not None:
            self.flush()
            self.q.put(None)
            self.t.join()
            self.t = None
            self.enabled = False   # a closed writer runs later jobs inline
            if self._prev_switch is not None:
                sys.setswitchinterval(self._prev_switch)
                self._prev_switch = None
        if self.native is not None:
            self.native.close()
            self.native = None
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
