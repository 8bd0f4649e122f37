"""Per-phase timers, JSONL trace and roctx ranges.

The reference has no instrumentation beyond log timestamps.
Each federated round here is split into phases (select / train / vote /
aggregate / comm / verify / eval / io); ``Telemetry.phase(name)`` times a
phase on the host (optionally synchronising the device first so GPU time is
attributed to the right phase), pushes a roctx range so the phases show up
in ``rocprofv3 --marker-trace`` timelines, and accumulates per-round
totals that are appended to a JSONL trace file.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import time
from collections import defaultdict
from typing import Dict, Optional

_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx or None
    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            return lib
        except OSError:
            continue
    _roctx = False
    return None


class Telemetry:
    def __init__(self, trace_file: Optional[str] = None, sync_fn=None, roctx: bool = True, rank: int = 0):
        self.trace_file = trace_file
        self.sync_fn = sync_fn
        self.rank = rank
        self.roctx = _load_roctx() if roctx else None
        self.round_times: Dict[str, float] = defaultdict(float)
        self.total: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)
        self.sync = bool(trace_file)
        self._stack = []

    @contextlib.contextmanager
    def phase(self, name: str):
        """Time a phase.  Phases nest (e.g. ``wait_writer`` inside ``eval``);
        each is charged its *exclusive* time — a nested phase's time is taken
        out of its parent's — so the per-phase totals never overlap and sum to
        at most the wall time they cover."""
        if self.roctx is not None:
            self.roctx.roctxRangePushA(name.encode())
        frame = [0.0]            # time spent in nested phases
        self._stack.append(frame)
        t0 = time.perf_counter()
        try:
            yield
        finally:
            try:
                if self.sync and self.sync_fn is not None:
                    self.sync_fn()   # may raise (a device error surfacing under --trace)
            finally:
                # the frame and the roctx range are closed whatever the sync did,
                # so later phases never charge a dead parent
                dt = time.perf_counter() - t0
                self._stack.pop()
                if self._stack:
                    self._stack[-1][0] += dt
                if self.roctx is not None:
                    self.roctx.roctxRangePop()
            ex = dt - frame[0]
            self.round_times[name] += ex
            self.total[name] += ex
            self.counts[name] += 1

    def end_round(self, **extra):
        rec = {"rank": self.rank, **{f"{k}_ms": v * 1e3 for k, v in self.round_times.items()}, **extra}
        if self.trace_file:
            os.makedirs(os.path.dirname(os.path.abspath(self.trace_file)), exist_ok=True)
            with open(self.trace_file, "a") as f:
                f.write(json.dumps(rec) + "\n")
        self.round_times = defaultdict(float)
        return rec

    def summary(self) -> Dict[str, float]:
        return {k: v * 1e3 for k, v in self.total.items()}

    def reset_totals(self) -> None:
        """Start the accumulated per-phase totals afresh (e.g. after warm-up
        rounds, so a benchmark's totals cover only its timed rounds)."""
        self.total = defaultdict(float)
        self.counts = defaultdict(int)
