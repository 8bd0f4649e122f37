"""Probe: what does recording an event between two kernels cost the GPU?

The round's main stream records one event after the verification kernel
(the side stream's evaluation waits on it), and the kernel trace shows a
~7 us gap before the next round's training kernel at exactly that point,
where every other kernel-to-kernel transition of the round has none.  A
default HIP event performs a system-scope fence when it is recorded (L2
write-back and invalidation, hip_runtime_api.h: hipEventDisableSystemFence);
``hipEventReleaseToDevice`` asks for a device-scope release instead.

Each mode runs a loop of GPU-bound copies (~25 us each, the host stays ahead)
with the named event traffic between them and reports the microseconds per
iteration; the difference to ``none`` is what the event costs on the GPU
(``side-indep``: the side stream's kernel with no dependency at all, the
floor of any cross-stream hand-off that needs no packet on the main stream).

    python scripts/probes/event_gap.py [--iters 400]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import time

import torch

hipEventDisableTiming = 0x2
hipEventDisableSystemFence = 0x20000000
hipEventReleaseToDevice = 0x40000000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--mb", type=int, default=64, help="bytes copied per kernel (MiB)")
    args = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    hip.hipEventRecord.argtypes = [vp, vp]
    hip.hipStreamWaitEvent.argtypes = [vp, vp, ctypes.c_uint]
    dev = torch.device("cuda", 0)
    n = args.mb * (1 << 20) // 4
    x = torch.ones(n, device=dev)
    y = torch.empty_like(x)
    small = torch.zeros(1024, device=dev)
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)

    def hip_event(flags):
        e = vp()
        assert hip.hipEventCreateWithFlags(ctypes.byref(e), flags) == 0
        return e

    def run(mode):
        hev = None
        if mode.startswith("hip"):
            flags = hipEventDisableTiming
            if "device" in mode:
                flags |= hipEventReleaseToDevice
            if "nofence" in mode:
                flags |= hipEventDisableSystemFence
            hev = hip_event(flags)
        cross = mode.endswith("+side")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            y.copy_(x)
            if mode == "none":
                continue
            if mode == "side-indep":   # side-stream work with no dependency on the main stream
                with torch.cuda.stream(side):
                    small.add_(1.0)
                continue
            if mode.startswith("torch"):
                e = torch.cuda.Event()
                e.record(main_s)
                if cross:
                    side.wait_event(e)
            else:
                assert hip.hipEventRecord(hev, vp(main_s.cuda_stream)) == 0
                if cross:
                    assert hip.hipStreamWaitEvent(vp(side.cuda_stream), hev, 0) == 0
            if cross:
                with torch.cuda.stream(side):
                    small.add_(1.0)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.iters * 1e6

    modes = ["none", "side-indep", "torch", "torch+side", "hip", "hip-device", "hip-nofence", "hip-device+side",
             "hip-nofence+side"]
    for m in modes:   # warm-up pass
        run(m)
    out = {}
    for rep in range(3):
        for m in modes:
            out.setdefault(m, []).append(round(run(m), 2))
    base = min(out["none"])
    print(json.dumps({"us_per_iter": out, "event_cost_us": {m: round(min(v) - base, 2) for m, v in out.items()}}))


if __name__ == "__main__":
    main()
