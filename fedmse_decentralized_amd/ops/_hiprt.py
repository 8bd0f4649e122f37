"""Minimal HIP runtime binding for the host-side hot path.

Per-round protocol traffic is tiny (descriptor arrays of a few hundred bytes
down, a few scores up), so its cost is API overhead, not bandwidth.  Instead
of staging copies through torch (dispatcher + hipMemcpyAsync + events, tens
of microseconds each), the framework keeps two rings of *mapped, coherent*
pinned host memory:

* ``DescRing`` – the host writes descriptor arrays with a plain numpy copy and
  passes the ring's *device* address to the kernel (zero copy, no API call).
  The ring lives in fine-grained *device* memory that the host writes through
  the PCIe BAR (write-combined stores, ~0.4 us per KB, then a store fence):
  a kernel on the round's critical path then reads its descriptors from HBM
  instead of paying ~1.2 us per dependent read of mapped host memory
  (``scripts/probes/mapped_latency.hip``; host rewrites between launches are
  always seen, ``scripts/probes/finegrained_host_write.hip``).
  ``FEDMX_DESC_RING=host`` keeps it in mapped pinned host memory;
* ``OutRing``  – kernels write host-visible results (scores, drifts, AUCs,
  training tracking) straight into it; the host reads them after the single
  ``hipStreamSynchronize`` that ends each protocol phase.

A ring region is reused only after a stream synchronisation that follows its
last use (``generation`` bookkeeping), so the host never overwrites bytes a
queued kernel has yet to read.
"""
from __future__ import annotations

import ctypes
import threading
from typing import List, Optional, Sequence

import numpy as np

hipHostMallocMapped = 0x2
hipHostMallocCoherent = 0x40000000
hipDeviceMallocFinegrained = 0x1

_lib = None
_lock = threading.Lock()


def rt():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                L = None
                for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
                    try:
                        L = ctypes.CDLL(name)
                        break
                    except OSError:
                        continue
                if L is None:
                    raise OSError("libamdhip64.so not found")
                vp = ctypes.c_void_p
                L.hipHostMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
                L.hipHostMalloc.restype = ctypes.c_int
                L.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_uint]
                L.hipHostGetDevicePointer.restype = ctypes.c_int
                L.hipStreamSynchronize.argtypes = [vp]
                L.hipStreamSynchronize.restype = ctypes.c_int
                L.hipHostFree.argtypes = [vp]
                L.hipHostFree.restype = ctypes.c_int
                L.hipDeviceSynchronize.argtypes = []
                L.hipDeviceSynchronize.restype = ctypes.c_int
                L.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
                L.hipExtMallocWithFlags.restype = ctypes.c_int
                L.hipFree.argtypes = [vp]
                L.hipFree.restype = ctypes.c_int
                L.hipMemcpy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int]
                L.hipMemcpy.restype = ctypes.c_int
                L.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
                L.hipEventCreateWithFlags.restype = ctypes.c_int
                L.hipEventRecord.argtypes = [vp, vp]
                L.hipEventRecord.restype = ctypes.c_int
                L.hipStreamWaitEvent.argtypes = [vp, vp, ctypes.c_uint]
                L.hipStreamWaitEvent.restype = ctypes.c_int
                L.hipEventDestroy.argtypes = [vp]
                L.hipEventDestroy.restype = ctypes.c_int
                _lib = L
    return _lib


def stream_sync(stream: int) -> None:
    rc = rt().hipStreamSynchronize(ctypes.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"hipStreamSynchronize failed ({rc})")
    SyncClock.tick(stream)


def device_sync() -> None:
    rc = rt().hipDeviceSynchronize()
    if rc != 0:
        raise RuntimeError(f"hipDeviceSynchronize failed ({rc})")
    SyncClock.tick()


hipEventDisableTiming = 0x2
hipEventDisableSystemFence = 0x20000000


class DeviceEvent:
    """A stream-order dependency between two streams of ONE device whose
    consumers are kernels only.  Created with hipEventDisableSystemFence:
    recording it skips the system-scope release (the L2 write-back that makes
    device memory visible to the host and to other devices,
    hip_runtime_api.h), which a kernel-to-kernel dependency on one device does
    not need -- each kernel dispatch carries its own agent-scope release and
    acquire, which is what orders two kernels of one stream across XCDs.  The
    event is re-recorded every use (a wait enqueued after a record waits for
    that record).  Never wait for it on the host, nor read mapped host memory
    behind it: use a torch event for those."""

    def __init__(self):
        L = rt()
        e = ctypes.c_void_p()
        rc = L.hipEventCreateWithFlags(ctypes.byref(e), hipEventDisableTiming | hipEventDisableSystemFence)
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags failed ({rc})")
        self.handle = e

    def record(self, stream: int) -> None:
        rc = rt().hipEventRecord(self.handle, ctypes.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed ({rc})")

    def wait(self, stream: int) -> None:
        """Make ``stream`` wait (on the device) for the last record."""
        rc = rt().hipStreamWaitEvent(ctypes.c_void_p(stream), self.handle, 0)
        if rc != 0:
            raise RuntimeError(f"hipStreamWaitEvent failed ({rc})")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and _lib is not None:
            try:
                _lib.hipEventDestroy(h)
            except Exception:   # interpreter shutdown
                pass


class SyncClock:
    """Counts completed synchronisations (ring-reuse generations): a stream
    synchronisation covers the rings of that stream only, a device
    synchronisation every ring (several runtimes may share the process)."""

    gen = 0                      # device-wide synchronisations
    _stream_gen: dict = {}       # stream -> synchronisations of that stream

    @classmethod
    def tick(cls, stream: Optional[int] = None):
        if stream is None:
            cls.gen += 1
        else:
            cls._stream_gen[stream] = cls._stream_gen.get(stream, 0) + 1

    @classmethod
    def of(cls, stream: int) -> int:
        """Monotone count of the synchronisations that cover ``stream``."""
        return cls.gen + cls._stream_gen.get(stream, 0)


class MappedBuffer:
    def __init__(self, nbytes: int):
        L = rt()
        hp = ctypes.c_void_p()
        # (at least 64 bytes: a rank hosting no client asks for empty rings,
        # and a zero-byte mapping has no device pointer)
        rc = L.hipHostMalloc(ctypes.byref(hp), max(int(nbytes), 64), hipHostMallocMapped | hipHostMallocCoherent)
        if rc != 0:
            raise RuntimeError(f"hipHostMalloc({nbytes}) failed ({rc})")
        dp = ctypes.c_void_p()
        rc = L.hipHostGetDevicePointer(ctypes.byref(dp), hp, 0)
        if rc != 0:
            raise RuntimeError(f"hipHostGetDevicePointer failed ({rc})")
        self.host_ptr = hp.value
        self.dev_ptr = dp.value
        self.nbytes = nbytes
        self.np = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.host_ptr))

    def view(self, off: int, dtype, count: int) -> np.ndarray:
        return self.np[off:off + count * np.dtype(dtype).itemsize].view(dtype)

    def __del__(self):
        try:
            if self.host_ptr:
                # queued kernels may still target this memory: drain first
                if _lib is not None:
                    _lib.hipDeviceSynchronize()
                    _lib.hipHostFree(ctypes.c_void_p(self.host_ptr))
                self.host_ptr = None
        except Exception:
            pass


class DeviceWriteBuffer:
    """Fine-grained device memory the host writes directly (large BAR): the
    same address on both sides.  Host reads of it are slow (uncached PCIe
    reads) — write-only from the host."""

    def __init__(self, nbytes: int):
        L = rt()
        p = ctypes.c_void_p()
        rc = L.hipExtMallocWithFlags(ctypes.byref(p), nbytes, hipDeviceMallocFinegrained)
        if rc != 0 or not p.value:
            raise RuntimeError(f"hipExtMallocWithFlags({nbytes}, fine-grained) failed ({rc})")
        self.host_ptr = p.value
        self.dev_ptr = p.value
        self.nbytes = nbytes
        # without a CPU mapping of the allocation (no large-BAR access) the
        # first host store would fault: check the process's page mappings first
        if not _cpu_mapped_rw(self.host_ptr, nbytes):
            L.hipFree(ctypes.c_void_p(self.host_ptr))
            self.host_ptr = None
            raise RuntimeError("fine-grained device memory is not mapped for host access (no large BAR)")
        self.np = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.host_ptr))
        # the host's stores must reach the device copy: write a pattern, read
        # it back through the runtime (device -> host copy), else refuse
        pat = (np.arange(64, dtype=np.uint8) * 37 + 11).astype(np.uint8)
        self.np[:64] = pat
        _store_fence()()
        back = np.zeros(64, dtype=np.uint8)
        rc = L.hipMemcpy(back.ctypes.data, ctypes.c_void_p(self.dev_ptr), 64, 2)   # hipMemcpyDeviceToHost
        if rc != 0 or not np.array_equal(back, pat):
            L.hipFree(ctypes.c_void_p(self.host_ptr))
            self.host_ptr = None
            raise RuntimeError("host writes to fine-grained device memory are not visible to the device")

    def __del__(self):
        try:
            if self.host_ptr and _lib is not None:
                _lib.hipDeviceSynchronize()
                _lib.hipFree(ctypes.c_void_p(self.host_ptr))
            self.host_ptr = None
        except Exception:
            pass


def _cpu_mapped_rw(addr: int, nbytes: int, maps_path: str = "/proc/self/maps") -> bool:
    """True when [addr, addr + nbytes) lies inside readable + writable
    mappings of this process (contiguous entries may together cover it)."""
    try:
        with open(maps_path) as f:
            lines = f.readlines()
    except OSError:
        return False
    need, end = addr, addr + nbytes
    spans = []
    for ln in lines:
        parts = ln.split()
        if len(parts) < 2 or not parts[1].startswith("rw"):
            continue
        a, b = (int(x, 16) for x in parts[0].split("-"))
        if b > addr and a < end:
            spans.append((a, b))
    for a, b in sorted(spans):
        if a > need:
            return False
        need = max(need, b)
        if need >= end:
            return True
    return False


def _store_fence():
    from . import _host

    return _host.lib().fedmx_store_fence


class _Ring:
    buffer_type = MappedBuffer

    def __init__(self, nbytes: int, stream: int):
        self.buf = self.buffer_type(nbytes)
        self._retired = []   # replaced buffers stay alive (host views may still point into them)
        self.stream = stream
        self.off = 0
        self.wrap_gen = -1   # generation at which the current pass started

    def _alloc(self, nbytes: int) -> int:
        nbytes = (nbytes + 63) & ~63
        if nbytes > self.buf.nbytes:
            # grow (rare: very large federations): drain every queued user of
            # the old ring, then replace it with one twice the request
            device_sync()
            self._retired.append(self.buf)
            self.buf = self.buffer_type(2 * nbytes)
            self.off = 0
            self.wrap_gen = SyncClock.of(self.stream)
        if self.off + nbytes > self.buf.nbytes:
            # wrapping: earlier regions may still be read/written by queued kernels
            # unless a stream synchronisation happened since this pass began
            if SyncClock.of(self.stream) <= self.wrap_gen:
                device_sync()   # kernels on any stream may still read the ring
            self.off = 0
            self.wrap_gen = SyncClock.of(self.stream)
        o = self.off
        self.off += nbytes
        return o


class DescRing(_Ring):
    def __init__(self, nbytes: int, stream: int, device_memory: Optional[bool] = None):
        import os

        if device_memory is None:
            device_memory = os.environ.get("FEDMX_DESC_RING", "device") != "host"
        self.fence = None
        if device_memory:
            self.buffer_type = DeviceWriteBuffer
            # the host's write-combined stores must be visible before the
            # launch that reads them is submitted
            self.fence = _store_fence()
            try:
                super().__init__(nbytes, stream)
                return
            except RuntimeError as e:   # no host-writable device memory here: mapped host ring
                import logging

                logging.getLogger(__name__).warning("descriptor ring in mapped host memory (%s)", e)
                self.buffer_type = MappedBuffer
                self.fence = None
        super().__init__(nbytes, stream)

    def put(self, *arrays: np.ndarray) -> List[int]:
        blobs = [np.ascontiguousarray(a).view(np.uint8).reshape(-1) for a in arrays]
        sizes = [(b.nbytes + 63) & ~63 for b in blobs]
        o = self._alloc(sum(sizes))
        ptrs = []
        for b, s in zip(blobs, sizes):
            self.buf.np[o:o + b.nbytes] = b
            ptrs.append(self.buf.dev_ptr + o)
            o += s
        if self.fence is not None:
            self.fence()
        return ptrs


class OutRing(_Ring):
    def take(self, dtype, count: int):
        """Reserve ``count`` elements; returns (device address, host numpy view)."""
        nb = int(count) * np.dtype(dtype).itemsize
        o = self._alloc(max(nb, 1))
        return self.buf.dev_ptr + o, self.buf.view(o, dtype, int(count))
