"""Transport probe of a multi-rank job, before any rank touches the GPU
(VERDICT r4 Next #4: the first 8-GPU run must not come back empty).

The driver launches ``bench.py`` as ``torch.distributed.run ... --nproc-per-node
N``: every rank is a fresh process that has imported torch but not yet
initialised HIP.  Before the real job starts, every rank runs a short probe of
the requested transport in a CHILD process of its own (a separate
rendezvous on a fresh port): process-group bring-up, the collective
self-test (``launch.collective_self_test``) and one exchange of the device
protocol's shape (an all-gather into a ``[world * rows, P]`` buffer and an
in-place float64 all-reduce; with ``ipc`` the peer-memory channels must come
up on every rank).  The ranks agree on the outcome through the launcher's
store; on a failure they try the next transport in ``FALLBACK`` order, so the
job runs on the first transport that works on every rank and its record says
which one and why (``transport_fallback``).  A probe child that hangs is
killed at its time limit; nothing is ever re-executed in a process that has
touched the GPU.

Transports: ``rccl`` = torch.distributed ``nccl`` (RCCL) collectives;
``ipc`` = one-shot peer-memory kernels (``parallel/ipc.py``) with a gloo
control plane; ``gloo`` = host-staged gloo collectives.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Tuple

FALLBACK = ("rccl", "ipc", "gloo")
# environment of each transport for the job and its probe
# (None: removed, so the backend is the device's default -- nccl on GPUs)
TRANSPORT_ENV = {
    "rccl": {"FEDMX_COMM": "rccl", "FEDMX_DIST_BACKEND": None},
    "ipc": {"FEDMX_COMM": "ipc", "FEDMX_DIST_BACKEND": "gloo"},
    "gloo": {"FEDMX_COMM": "rccl", "FEDMX_DIST_BACKEND": "gloo"},
}
PROBE_FLAG = "--probe-comm"


def order_from(requested: str) -> List[str]:
    return list(FALLBACK[FALLBACK.index(requested):]) if requested in FALLBACK else list(FALLBACK)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _store(world: int, timeout_s: float):
    """The launcher's store (torch.distributed.run hosts it at MASTER_ADDR:MASTER_PORT)."""
    import datetime

    import torch.distributed as dist

    base = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]), world,
                         is_master=False, timeout=datetime.timedelta(seconds=timeout_s))
    return dist.PrefixStore("fedmx_probe", base)


def apply_env(env, transport: str) -> None:
    for k, v in TRANSPORT_ENV[transport].items():
        if v is None:
            env.pop(k, None)
        else:
            env[k] = v


def requested_transport(comm_flag: Optional[str]) -> str:
    """--comm, else FEDMX_COMM, else gloo when FEDMX_DIST_BACKEND=gloo (one-GPU
    rehearsals), else rccl."""
    if comm_flag:
        return comm_flag
    if os.environ.get("FEDMX_COMM"):
        return os.environ["FEDMX_COMM"]
    return "gloo" if os.environ.get("FEDMX_DIST_BACKEND") == "gloo" else "rccl"


def run_child(transport: str, script: str, port: int, timeout_s: float) -> Tuple[int, str]:
    """This rank's probe of ``transport`` in a child process: (exit code, tail of its output)."""
    env = dict(os.environ)
    apply_env(env, transport)
    env["MASTER_PORT"] = str(port)
    env["MASTER_ADDR"] = "127.0.0.1"
    # the child's own rendezvous: rank 0's child hosts the store
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    env["FEDMX_COMM_SELFTEST"] = "1"
    try:
        r = subprocess.run([sys.executable, script, PROBE_FLAG, transport], env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True, timeout=timeout_s)
        return r.returncode, (r.stdout or "")[-1500:]
    except subprocess.TimeoutExpired as e:
        out = e.stdout.decode(errors="replace") if isinstance(e.stdout, bytes) else (e.stdout or "")
        return 124, (out[-1200:] + f"\n[probe killed after {timeout_s:.0f} s]")


def choose_transport(script: str, requested: str = "rccl", timeout_s: float = 180.0,
                     order: Optional[List[str]] = None) -> Tuple[str, Optional[Dict]]:
    """Every rank (before touching the GPU): probe transports in order until
    one works on every rank.  Returns (transport, fallback record or None when
    the requested one worked).  Raises when none works."""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    store = _store(world, timeout_s * 2 + 120)
    failures = []
    t0 = time.perf_counter()
    for t in (order or order_from(requested)):
        if rank == 0:
            store.set(f"{t}/port", str(_free_port()))
        port = int(store.get(f"{t}/port"))
        rc, tail = run_child(t, script, port, timeout_s)
        store.set(f"{t}/rc/{rank}", str(rc))
        store.set(f"{t}/tail/{rank}", tail[-600:])
        rcs = [int(store.get(f"{t}/rc/{r}")) for r in range(world)]
        if all(c == 0 for c in rcs):
            if t == requested and not failures:
                return t, None
            return t, {"requested": requested, "used": t, "failures": failures,
                       "probe_s": round(time.perf_counter() - t0, 2)}
        bad = [r for r, c in enumerate(rcs) if c != 0]
        failures.append({"transport": t, "ranks_failed": bad, "rc": rcs[bad[0]],
                         "first_failure_tail": store.get(f"{t}/tail/{bad[0]}").decode(errors="replace")})
    raise RuntimeError(f"no transport works on every rank: {failures}")


def child_main(transport: str) -> int:
    """The probe child: bring-up + self-test + one protocol-shaped exchange."""
    import numpy as np
    import torch

    from ..models.layout import P_PAD
    from .launch import init_comm, shutdown

    fail = [x for x in os.environ.get("FEDMX_PROBE_FAIL", "").split(",") if x]
    if transport in fail:   # tests: a transport that fails on this box
        print(f"probe {transport}: failure injected (FEDMX_PROBE_FAIL)", flush=True)
        return 3
    device = "cuda" if torch.cuda.device_count() > 0 else "cpu"
    if transport == "ipc" and device != "cuda":
        print("probe ipc: peer-memory transport needs GPUs", flush=True)
        return 4
    comm = init_comm(device=device, comm_impl=TRANSPORT_ENV[transport]["FEDMX_COMM"])
    W, r, dev = comm.world_size, comm.rank, comm.device
    rows, n = 3, 64
    if transport == "ipc":
        comm.setup_exchange(rows * P_PAD, 4 * n)   # (words: 2n doubles)
        if not getattr(comm, "active", False):
            print("probe ipc: peer-memory channels did not come up on every rank", flush=True)
            shutdown(comm)
            return 5
    send = torch.full((rows, P_PAD), float(r + 1), dtype=torch.float32, device=dev)
    allg = torch.empty(W * rows, P_PAD, dtype=torch.float32, device=dev)
    vec = torch.zeros(2 * n, dtype=torch.float64, device=dev)
    for _ in range(3):
        vec.zero_()
        vec[r % (2 * n)] = float(r + 1)   # one contributor per entry, as the protocol's vectors
        comm.all_gather_into(allg, send)
        comm.all_reduce_inplace(vec)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if hasattr(comm, "check"):
        comm.check()
    want = np.repeat(np.arange(1, W + 1, dtype=np.float32), rows)
    g = allg.cpu().numpy()
    v = vec.cpu().numpy()
    want_v = np.zeros(2 * n)
    for q in range(W):
        want_v[q % (2 * n)] += q + 1
    ok = bool(np.array_equal(g[:, 0], want)) and bool(np.all(g == g[:, :1])) and bool(np.array_equal(v, want_v))
    shutdown(comm)
    if not ok:
        print(f"probe {transport}: exchange returned wrong rows", flush=True)
        return 6
    if r == 0:
        print(f"probe {transport}: ok ({W} ranks on {dev.type})", flush=True)
    return 0
