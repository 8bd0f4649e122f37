"""Client -> rank placement.

Clients are placed in contiguous blocks (rank r hosts global ids
``[start_r, end_r)``), the first ``N % world`` ranks hosting one extra.  On
one GPU all clients share one set of device buffers and never communicate;
across GPUs only the per-round collectives of ``parallel/comm.py`` cross
xGMI.  Placement never changes results: every reduction runs in global
client order.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List


@dataclass(frozen=True)
class ShardMap:
    num_clients: int
    world_size: int

    def bounds(self, rank: int):
        q, r = divmod(self.num_clients, self.world_size)
        start = rank * q + min(rank, r)
        end = start + q + (1 if rank < r else 0)
        return start, end

    def owner(self, cid: int) -> int:
        for r in range(self.world_size):
            s, e = self.bounds(r)
            if s <= cid < e:
                return r
        raise IndexError(cid)

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
