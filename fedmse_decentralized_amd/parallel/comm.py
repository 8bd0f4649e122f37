"""Communication backends for the decentralised protocol.

The reference has no transport at all: peers are Python objects calling
each other's methods in one interpreter (`src/Trainer/client_trainer.py:136-151`,
`src/main.py:259-264`).  Here every rank hosts a shard of the
clients and the protocol's logical messages become a few collectives per
round:

* vote scores / dev-set MSEs / epochs-run  -> ``all_reduce_sum`` of a small
  float64 vector (each entry has exactly one non-zero contributor, so the sum
  is exact and identical on every rank);
* model exchange (M2/M4)                   -> ``all_gather`` of the packed,
  padded parameter vectors of the locally selected clients
  ([world, slots, 9216] fp32); every rank then runs the same weighted reduce,
  so no separate broadcast of the aggregate is needed;
* AUCs / verification results (M6)         -> ``all_reduce_sum``.

Backends:
* ``LoopbackComm``  – world size 1 (single GPU / CPU runs).
* ``ThreadComm``    – N in-process ranks on threads (protocol tests without
  process spawning).
* ``TorchDistComm`` – ``torch.distributed``; backend ``nccl`` (= RCCL over
  xGMI on MI355X, one process per GPU) or ``gloo`` (CPU tests).
"""
from __future__ import annotations

import os
import threading
from typing import Any, List, Optional

import torch


class Comm:
    rank: int = 0
    world_size: int = 1
    device: torch.device = torch.device("cpu")
    phantom: bool = False   # PhantomComm: collectives stubbed (single-GPU projection)
    force_collectives: bool = False
    devices_distinct: bool = False   # every rank on its own GPU (set by launch.collective_self_test)

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    @property
    def collective(self) -> bool:
        """Take the multi-rank code path (pack, collective, unpack).  True for
        world size > 1, and for a world-size-1 torch.distributed group created
        with ``FEDMX_FORCE_COLLECTIVES=1``: a one-GPU box then runs the real
        RCCL calls and stream ordering of the multi-GPU path (RCCL refuses two
        ranks on one GPU, so this is the only RCCL coverage one GPU allows)."""
        return self.world_size > 1 or self.force_collectives

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Returns [world, *t.shape] on t's device."""
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, src: int) -> torch.Tensor:
        raise NotImplementedError

    def all_gather_into(self, out: torch.Tensor, t: torch.Tensor) -> None:
        """All-gather into a caller-owned buffer of ``world * t.shape[0]`` rows
        (persistent exchange buffers: no allocation per round)."""
        out.copy_(self.all_gather(t).reshape(out.shape))

    def barrier(self) -> None:
        pass

    def all_gather_object(self, obj: Any) -> List[Any]:
        raise NotImplementedError

    def all_reduce_inplace(self, t: torch.Tensor) -> None:
        """In-place sum over ranks, stream-ordered on the tensor's device (no
        host synchronisation with RCCL)."""
        t.copy_(self.all_reduce_sum(t))


def _np_wrap(fn):
    """Let a tensor collective also take / return numpy arrays (host protocol vectors)."""
    import functools

    import numpy as np

    @functools.wraps(fn)
    def w(self, t, *a, **k):
        if isinstance(t, np.ndarray):
            return fn(self, torch.from_numpy(np.ascontiguousarray(t)), *a, **k).numpy()
        return fn(self, t, *a, **k)
    return w


class LoopbackComm(Comm):
    def __init__(self, device: Optional[torch.device] = None):
        self.rank = 0
        self.world_size = 1
        self.device = torch.device(device) if device is not None else torch.device("cpu")

    def all_reduce_sum(self, t):
        return t

    def all_gather(self, t):
        return t[None] if not isinstance(t, torch.Tensor) else t.unsqueeze(0)

    def all_gather_into(self, out, t):
        out.copy_(t.reshape(out.shape))

    def broadcast(self, t, src):
        return t

    def all_gather_object(self, obj):
        return [obj]

    def all_reduce_inplace(self, t):
        pass


class PhantomComm(Comm):
    """Rank 0 of a ``world``-rank job with the collectives stubbed out locally:
    ``all_gather`` repeats this rank's contribution for every rank and the
    all-reduces leave the local values as they are.

    A single-GPU *projection* tool (``bench.py --phantom-ranks W``): the rank
    does exactly the per-rank GPU and host work of a W-GPU weak-scaling job
    (its 10 clients, the W-times larger replicated dev set and vote data, the
    W-rank packing / unpacking of the exchange) without RCCL, so the per-rank
    round time of the 8-GPU job can be measured, and optimised, on one GPU.
    The numbers it produces (AUCs, decisions) are not a federation's."""

    phantom = True

    def __init__(self, world: int, device: Optional[torch.device] = None):
        self.rank = 0
        self.world_size = int(world)
        self.device = torch.device(device) if device is not None else torch.device("cpu")

    @_np_wrap
    def all_reduce_sum(self, t):
        return t

    def all_gather(self, t):
        x = t if isinstance(t, torch.Tensor) else torch.as_tensor(t)
        return x.unsqueeze(0).expand((self.world_size,) + tuple(x.shape)).contiguous()

    def all_gather_into(self, out, t):
        out.view((self.world_size,) + tuple(t.shape)).copy_(t.unsqueeze(0).expand((self.world_size,) + tuple(t.shape)))

    def broadcast(self, t, src):
        return t

    def all_gather_object(self, obj):
        return [obj] * self.world_size

    def all_reduce_inplace(self, t):
        pass


class _ThreadGroup:
    def __init__(self, world: int):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots: List[Any] = [None] * world


class ThreadComm(Comm):
    """In-process fake collective group; create with ``ThreadComm.group(n)``."""

    def __init__(self, group: _ThreadGroup, rank: int):
        self.g = group
        self.rank = rank
        self.world_size = group.world
        self.device = torch.device("cpu")

    @staticmethod
    def group(world: int) -> List["ThreadComm"]:
        g = _ThreadGroup(world)
        return [ThreadComm(g, r) for r in range(world)]

    def _exchange(self, obj):
        self.g.barrier.wait()
        self.g.slots[self.rank] = obj
        self.g.barrier.wait()
        out = list(self.g.slots)
        self.g.barrier.wait()
        return out

    @_np_wrap
    def all_reduce_sum(self, t):
        parts = self._exchange(t.detach().cpu().clone())
        acc = parts[0].clone()
        for p in parts[1:]:
            acc += p
        return acc.to(t.device)

    def all_gather(self, t):
        parts = self._exchange(t.detach().cpu().clone())
        return torch.stack(parts, 0).to(t.device)

    def broadcast(self, t, src):
        parts = self._exchange(t.detach().cpu().clone())
        return parts[src].to(t.device)

    def barrier(self):
        self.g.barrier.wait()

    def all_gather_object(self, obj):
        return self._exchange(obj)


class TorchDistComm(Comm):
    """torch.distributed collectives on the default process group."""

    def __init__(self, device: Optional[torch.device] = None):
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.dist = dist
        self.rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        self.backend = dist.get_backend()
        self.force_collectives = os.environ.get("FEDMX_FORCE_COLLECTIVES", "0") == "1"
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        self.device = torch.device(device)

    def _to(self, t):
        return t if t.device == self.device else t.to(self.device)

    @_np_wrap
    def all_reduce_sum(self, t):
        x = self._to(t).clone()
        self.dist.all_reduce(x, op=self.dist.ReduceOp.SUM)
        return x.to(t.device)

    def all_gather(self, t):
        x = self._to(t).contiguous()
        flat = x.reshape(1, -1) if x.dim() == 0 else x
        # concatenated-along-dim-0 form (supported by both gloo and RCCL)
        out = torch.empty((self.world_size * flat.shape[0],) + tuple(flat.shape[1:]), dtype=x.dtype, device=x.device)
        self.dist.all_gather_into_tensor(out, flat)
        return out.view((self.world_size,) + tuple(x.shape)).to(t.device)

    def all_gather_into(self, out, t):
        if out.device == self.device and t.device == self.device:
            self.dist.all_gather_into_tensor(out, t)
        else:
            out.copy_(self.all_gather(t).reshape(out.shape))

    def broadcast(self, t, src):
        x = self._to(t).clone()
        self.dist.broadcast(x, src)
        return x.to(t.device)

    def all_reduce_inplace(self, t):
        if t.device == self.device:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        else:
            t.copy_(self.all_reduce_sum(t))

    def barrier(self):
        if self.backend == "nccl":
            self.dist.barrier(device_ids=[self.device.index])
        else:
            self.dist.barrier()

    def all_gather_object(self, obj):
        out = [None] * self.world_size
        self.dist.all_gather_object(out, obj)
        return out
