"""Client -> rank placement.

Clients are placed in contiguous blocks (rank r hosts global ids
``[start_r, end_r)``), the first ``N % world`` ranks hosting one extra.  On
one GPU all clients share one set of device buffers and never communicate;
across GPUs only the per-round collectives of ``parallel/comm.py`` cross
xGMI.  Placement never changes results: every reduction runs in global
client order.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Tuple


@dataclass(frozen=True)
class ShardMap:
    num_clients: int
    world_size: int
    # placement tables, built once (the round loop asks for owners and
    # bounds of every selected client: ~400 lookups per round at 80 clients)
    _bounds: Tuple[Tuple[int, int], ...] = field(init=False, repr=False, compare=False)
    _owner: Tuple[int, ...] = field(init=False, repr=False, compare=False)

    def __post_init__(self):
        q, r = divmod(self.num_clients, self.world_size)
        b = []
        for rank in range(self.world_size):
            start = rank * q + min(rank, r)
            b.append((start, start + q + (1 if rank < r else 0)))
        own = [0] * self.num_clients
        for rank, (s, e) in enumerate(b):
            for c in range(s, e):
                own[c] = rank
        object.__setattr__(self, "_bounds", tuple(b))
        object.__setattr__(self, "_owner", tuple(own))

    def bounds(self, rank: int):
        return self._bounds[rank]

    def owner(self, cid: int) -> int:
        if not 0 <= cid < self.num_clients:
            raise IndexError(cid)
        return self._owner[cid]

    def local_ids(self, rank: int) -> List[int]:
        s, e = self.bounds(rank)
        return list(range(s, e))

    def to_local(self, rank: int, cid: int) -> int:
        s, e = self.bounds(rank)
        if not (s <= cid < e):
            raise KeyError(f"client {cid} is not hosted by rank {rank}")
        return cid - s

    def max_local(self) -> int:
        return max(self.bounds(r)[1] - self.bounds(r)[0] for r in range(self.world_size))
