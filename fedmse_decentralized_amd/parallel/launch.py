"""Process-group bring-up: one process per GPU (torchrun / torch.distributed.run).

Reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the
environment.  On ROCm the ``nccl`` backend is RCCL; for multi-process CPU
tests use ``gloo``.  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` must be exported for
RCCL's dmabuf IPC on this platform, before the HIP runtime starts
(``parallel/env.py``; the entry points export it before importing torch).
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch

from .comm import Comm, LoopbackComm, TorchDistComm
from .env import export_comm_env


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init_comm(backend: Optional[str] = None, device: Optional[str] = None, timeout_s: int = 300,
              comm_impl: Optional[str] = None) -> Comm:
    """Create the comm for this process.  World size 1 -> LoopbackComm.

    ``comm_impl`` (or ``FEDMX_COMM``): ``rccl`` (default) runs the round's
    collectives through torch.distributed (RCCL on the GPU, gloo on the CPU);
    ``ipc`` runs the device protocol's per-round all-gather / all-reduce as
    one-shot peer-memory kernels (``parallel/ipc.py``), falling back to the
    torch.distributed collectives when bring-up fails on any rank."""
    impl = comm_impl or os.environ.get("FEDMX_COMM") or "rccl"
    if impl not in ("rccl", "ipc"):
        raise ValueError(f"FEDMX_COMM / --comm must be rccl or ipc, not {impl!r}")
    world = env_world()
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    # FEDMX_FORCE_COLLECTIVES=1 with world size 1: a real (one-rank) process
    # group, so the multi-rank path runs its RCCL calls on a one-GPU box
    forced = os.environ.get("FEDMX_FORCE_COLLECTIVES", "0") == "1"
    if world <= 1 and not forced:
        dev = torch.device("cuda", 0) if device == "cuda" else torch.device("cpu")
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        return LoopbackComm(dev)
    import torch.distributed as dist

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # normally already exported by the entry point before HIP started
    # (parallel/env.py); set late, HSA never sees it
    late = export_comm_env()
    if late and device == "cuda" and torch.cuda.is_initialized():
        import sys

        print(f"warning: {', '.join(late)} set after the HIP runtime started; export it before launching "
              "(bench.py / main.py do this before importing torch)", file=sys.stderr)
    if backend is None:
        # FEDMX_DIST_BACKEND=gloo: multi-rank rehearsal on one GPU (RCCL needs distinct GPUs)
        backend = os.environ.get("FEDMX_DIST_BACKEND") or ("nccl" if device == "cuda" else "gloo")
    if device == "cuda":
        # FEDMX_DEVICE_INDEX pins every rank to one GPU (multi-rank tests on a
        # one-GPU box, with the gloo backend; RCCL needs distinct GPUs)
        idx = int(os.environ.get("FEDMX_DEVICE_INDEX", local_rank))
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
    else:
        dev = torch.device("cpu")
    if not dist.is_initialized():
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    if impl == "ipc" and dev.type == "cuda":
        # the round's device collectives over peer-mapped memory (parallel/ipc.py);
        # activated collectively by the device protocol's setup_exchange
        from .ipc import IpcComm

        comm = IpcComm(dev)
    else:
        comm = TorchDistComm(dev)
    if os.environ.get("FEDMX_COMM_SELFTEST", "1") != "0":
        res = collective_self_test(comm)
        if comm.is_root:
            import sys

            print(f"collective self-test ok: {res['world']} rank(s) over {getattr(comm, 'backend', '?')}, "
                  f"devices {'distinct' if res['devices_distinct'] else 'shared'}: {res['devices']}",
                  file=sys.stderr)
    return comm


def _device_identity(dev: torch.device):
    """(host, physical GPU) of this rank: ranks on distinct GPUs exchange over
    xGMI, ranks sharing a GPU (one-box rehearsals) do not."""
    import socket

    if dev.type != "cuda":
        return (socket.gethostname(), "cpu", os.getpid())
    p = torch.cuda.get_device_properties(dev)
    ident = getattr(p, "uuid", None)
    ident = str(ident) if ident is not None else f"{os.environ.get('HIP_VISIBLE_DEVICES', '')}:{dev.index}"
    return (socket.gethostname(), ident)


def collective_self_test(comm: Comm) -> dict:
    """Check the process group right after bring-up, before any federation
    work: an all-gather of rank-patterned rows and a float64 all-reduce on the
    rank's device must return exactly the expected values on every rank.  A
    broken transport (wrong device binding, IPC / dmabuf failure, a rank on
    the wrong communicator) then fails here with a diagnosis instead of as
    garbage aggregates or a hang many rounds later.  Also records which
    ranks share a physical GPU (``comm.devices_distinct``)."""
    W, r, dev = comm.world_size, comm.rank, comm.device
    x = torch.arange(257, dtype=torch.float32, device=dev) + 1000.0 * r
    g = comm.all_gather(x).cpu()
    want = torch.arange(257, dtype=torch.float32)[None] + 1000.0 * torch.arange(W, dtype=torch.float32)[:, None]
    s = comm.all_reduce_sum(torch.full((33,), float(r + 1), dtype=torch.float64, device=dev)).cpu()
    bad_g = (g.shape != want.shape) or not torch.equal(g, want)
    bad_r = not bool(torch.all(s == W * (W + 1) / 2))
    ids = comm.all_gather_object(_device_identity(dev))
    comm.devices_distinct = len(set(ids)) == W
    comm.peer_devices = ids
    if bad_g or bad_r:
        what = []
        if bad_g:
            rows = [i for i in range(min(W, g.shape[0])) if not torch.equal(g[i], want[i])]
            what.append(f"all-gather rows {rows} wrong")
        if bad_r:
            what.append(f"all-reduce gave {float(s[0])} (want {W * (W + 1) / 2})")
        backend = getattr(comm, "backend", "?")
        msg = (f"[rank {r}/{W}] collective self-test FAILED on {dev} over {backend}: {'; '.join(what)}. "
               f"Ranks' devices: {ids}. Check one GPU per rank (LOCAL_RANK / HIP_VISIBLE_DEVICES), "
               "HSA_ENABLE_IPC_MODE_LEGACY=0 for RCCL's dmabuf IPC, and MASTER_ADDR/PORT.")
        raise RuntimeError(msg)
    return {"world": W, "devices_distinct": comm.devices_distinct, "devices": ids}


def shutdown(comm: Comm) -> None:
    if isinstance(comm, TorchDistComm):
        import torch.distributed as dist

        if hasattr(comm, "close"):
            # peer-memory channels: every rank drains its queue before any
            # area is unmapped or freed
            if comm.device.type == "cuda":
                torch.cuda.synchronize(comm.device)
            comm.barrier()
            comm.close()
            comm.barrier()
        if dist.is_initialized():
            dist.destroy_process_group()
