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

Variants (``ExperimentConfig.election`` / ``protocol_variant``):

* ``elect_majority`` — the legacy centralised ``GlobalAggregator.select_aggregator``
  (source deleted; behaviour reconstructed from the strings of
  `src/Trainer/__pycache__/global_aggregator.cpython-313.pyc`):
  every selected client votes with the same per-voter rule, votes are
  tallied, the candidate with the most votes wins (ties: earliest in
  selection order).
* ``vote_mse_cap`` (thesis Alg. 4.2, Thesis p.20): candidates whose score
  exceeds the cap are never voted for; ``fallback_rng`` (Thesis p.25
  §4.3.4): if no voter finds a valid candidate, a random eligible selected
  client aggregates.
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


def _ballot(voter: int, selected: Sequence[int], base_scores: Dict[int, float], agg_counts: Sequence[int],
            max_aggregation: int, noise, vote_mse_cap: Optional[float], log_enabled: bool):
    """One voter's noisy scores of every other selected client and its choice
    (``vote_for_aggregator``, `src/Trainer/client_trainer.py:249-285`)."""
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
        if vote_mse_cap is not None and not (s <= vote_mse_cap):
            continue
        if agg_counts[cid] < max_aggregation:
            if log_enabled:
                log.info(f"[Client {voter}] Voting for Client {list(selected).index(cid) + 1} with MSE score: {s:.6f}")
            return cid, noisy
    return None, noisy


def _fallback(selected, agg_counts, max_aggregation, rng) -> Optional[int]:
    """Uniform choice among the eligible selected clients from ONE uniform
    draw ``u = rng.random()``: ``eligible[floor(u * n)]`` (the device
    protocol's election kernel applies the same formula to the same draw)."""
    eligible = [c for c in selected if agg_counts[c] < max_aggregation]
    if not eligible:
        return None
    n = len(eligible)
    return eligible[min(int(rng.random() * n), n - 1)]


class OneDraw:
    """A pre-drawn uniform for :func:`_fallback`: the federation draws one
    value per round whether or not the fallback is needed, so the random
    stream does not depend on the election's outcome (and the device
    protocol, which learns the outcome only on the GPU, consumes it alike)."""

    def __init__(self, u: float):
        self.u = float(u)

    def random(self) -> float:
        return self.u


def elect_aggregator(selected: Sequence[int], base_scores: Dict[int, float], agg_counts: Sequence[int],
                     max_aggregation: int, noise, log_enabled: bool = True, vote_mse_cap: Optional[float] = None,
                     fallback_rng: Optional[random.Random] = None) -> ElectionResult:
    for voter in selected:
        cid, noisy = _ballot(voter, selected, base_scores, agg_counts, max_aggregation, noise, vote_mse_cap,
                             log_enabled)
        if cid is not None:
            return ElectionResult(cid, voter, dict(noisy))
    if fallback_rng is not None:
        cid = _fallback(selected, agg_counts, max_aggregation, fallback_rng)
        if cid is not None:
            log.info(f"No valid aggregator voted; randomly selected Client {cid + 1}")
            return ElectionResult(cid, None, {})
    return ElectionResult(None, None, {})


def elect_majority(selected: Sequence[int], base_scores: Dict[int, float], agg_counts: Sequence[int],
                   max_aggregation: int, noise, log_enabled: bool = True, vote_mse_cap: Optional[float] = None,
                   fallback_rng: Optional[random.Random] = None) -> ElectionResult:
    votes: Dict[int, int] = {}
    last_scores: Dict[int, float] = {}
    for voter in selected:
        if log_enabled:
            log.info(f"Client {voter + 1} is voting...")
        cid, noisy = _ballot(voter, selected, base_scores, agg_counts, max_aggregation, noise, vote_mse_cap,
                             log_enabled)
        if cid is not None:
            votes[cid] = votes.get(cid, 0) + 1
            last_scores = dict(noisy)
            if log_enabled:
                log.info(f"Client {voter + 1} voted for aggregator with MSE score: {dict(noisy)[cid]:.4f}")
    best, best_votes = None, 0
    for cid in selected:                 # ties: earliest in selection order
        v = votes.get(cid, 0)
        if v > best_votes:
            best, best_votes = cid, v
    if best is not None:
        if log_enabled:
            log.info(f"Client {best + 1} received {best_votes} votes and has been aggregator {agg_counts[best]} times")
            log.info(f"Selected aggregator with {best_votes} votes")
        return ElectionResult(best, None, last_scores)
    if fallback_rng is not None:
        cid = _fallback(selected, agg_counts, max_aggregation, fallback_rng)
        if cid is not None:
            return ElectionResult(cid, None, {})
    log.warning("No suitable aggregator found")
    return ElectionResult(None, None, {})
