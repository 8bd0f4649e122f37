"""Process-group bring-up: one process per GPU (torchrun / torch.distributed.run).

Reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the
environment.  On ROCm the ``nccl`` backend is RCCL; for multi-process CPU
tests use ``gloo``.  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` must stay exported for
RCCL's dmabuf IPC on this platform.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch

from .comm import Comm, LoopbackComm, TorchDistComm


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
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # the exchange buffers are persistent; without this, ProcessGroupNCCL's
    # recordStream on every collective's tensors leaves events that the caching
    # allocator then polls on each later allocation of the round loop
    os.environ.setdefault("TORCH_NCCL_AVOID_RECORD_STREAMS", "1")
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

        return IpcComm(dev)
    return TorchDistComm(dev)


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
