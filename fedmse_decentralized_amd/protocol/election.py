"""Client selection and aggregator election.

* Selection: ``k = max(1, int(p * N))`` clients drawn with Python's
  ``random.sample`` (`src/main.py:270-273`), replicated on every rank from the
  same seed.
* Election (`src/Trainer/client_trainer.py:249-285`, driver loop
  `src/main.py:281-288`): the selected clients vote in selection order; a voter
  scores every *other* selected client by its reconstruction MSE on the vote
  data (times the tie-break noise), sorts ascending and votes for the first
  one whose ``aggregation_count`` is below the cap; the first voter that finds
  a candidate decides.  Voter score draws happen in selected-list
  order, one per candidate, so the RNG replay stays in step.

Scores arrive from the engine as the noise-free per-client MSE (identical on
every rank after the score all-reduce); only the noise is drawn here.
"""
from __future__ import annotations

import logging
import random
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

log = logging.getLogger("fedmx")


def select_clients(rng: random.Random, n_clients: int, ratio: float) -> List[int]:
    k = max(1, int(ratio * n_clients))
    return rng.sample(range(n_clients), k)


@dataclass
class ElectionResult:
    aggregator: Optional[int]          # global client id, or None
    voter: Optional[int]
    scores: Dict[int, float]           # noisy scores of the deciding voter


def elect_aggregator(selected: Sequence[int], base_scores: Dict[int, float], agg_counts: Sequence[int],
                     max_aggregation: int, noise, log_enabled: bool = True) -> ElectionResult:
    for voter in selected:
        noisy = []
        for cid in selected:
            if cid == voter:
                continue
            f = 1.0 + (noise.rand() - 0.5) * 0.0002
            s = base_scores[cid] * f
            noisy.append((cid, s))
            if log_enabled:
                log.info(f"[Client {voter}] Client {list(selected).index(cid) + 1} MSE score: {s:.6f}")
        noisy.sort(key=lambda t: t[1])
        for cid, s in noisy:
            if agg_counts[cid] < max_aggregation:
                if log_enabled:
                    log.info(f"[Client {voter}] Voting for Client {list(selected).index(cid) + 1} with MSE score: {s:.6f}")
                return ElectionResult(cid, voter, dict(noisy))
    return ElectionResult(None, None, {})
