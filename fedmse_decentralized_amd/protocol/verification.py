"""Receiver-side verification of a broadcast aggregate.

Reference ``ModelVerifier.verify_model`` (`src/Trainer/model_verifier.py:29-77`)
and ``ClientTrainer.update_from_peers`` (`src/Trainer/client_trainer.py:174-206`):

* the first model a client ever receives is accepted unconditionally; its
  performance is recorded as history (Q15);
* afterwards: ``drift = sum_tensors ||theta_prev_received - theta_new||_2``,
  ``perf = 1 / (1 + MSE(V, model(V)))``, ``dperf = perf_new - perf_prev``;
  accept iff ``drift <= 3.0`` and ``dperf >= -0.002``;  the history is
  updated to the new model either way (fixed-mode option ``drift_rel``: the
  limit is ``drift_rel * sum_tensors ||theta_prev_received||_2`` instead);
* accept: adopt the model, refresh the FedProx anchor, reset the rejection
  counter; reject: increment it, and at ``>= 3`` log a possible attack.

Drift and perf are computed on the device by the engine; the decision and the
per-client state machine live here (replicated-decision, local-state: each
rank owns the verifiers of its own clients).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field
from typing import Optional

log = logging.getLogger("fedmx")


@dataclass
class VerifierState:
    history_version: Optional[int] = None   # index of the last received aggregate
    history_perf: float = 0.0
    history_round: int = -1
    rejected_updates: int = 0


@dataclass
class VerifyDecision:
    verified: bool
    perf_change: float
    drift: float


class Verifier:
    def __init__(self, verification_threshold: float = 3.0, performance_threshold: float = 0.002,
                 method: str = "val", max_rejected: int = 3, drift_rel: float = 0.0):
        self.thr = verification_threshold
        # > 0: relative drift limit drift <= drift_rel * ||history|| (config.drift_threshold_rel)
        self.drift_rel = drift_rel
        self.perf_thr = performance_threshold
        self.method = method
        self.max_rejected = max_rejected

    def needs_drift(self, st: VerifierState) -> bool:
        return st.history_version is not None

    def decide(self, client_id: int, st: VerifierState, version: int, perf_new: float, drift: float,
               current_round: int, hist_norm: Optional[float] = None) -> VerifyDecision:
        if st.history_version is None:
            st.history_version, st.history_perf, st.history_round = version, perf_new, current_round
            return VerifyDecision(True, 0.0, 0.0)
        change = perf_new - st.history_perf
        st.history_version, st.history_perf, st.history_round = version, perf_new, current_round
        if log.isEnabledFor(logging.INFO):
            log.info(f"Client {client_id} - Param changes: {drift:.10f}, Performance change: {change:.10f}")
            log.info(f"Using {self.method} dataset for verification")
        limit = self.drift_rel * hist_norm if self.drift_rel > 0 and hist_norm is not None else self.thr
        ok = (drift <= limit) and (change >= -self.perf_thr)
        return VerifyDecision(ok, change, drift)

    def apply(self, client_id: int, st: VerifierState, dec: VerifyDecision) -> None:
        if dec.verified:
            st.rejected_updates = 0
            if log.isEnabledFor(logging.INFO):
                log.info(f"[Client {client_id}] Model verified and updated. Performance change: {dec.perf_change:.10f}")
        else:
            st.rejected_updates += 1
            log.warning("[Client %d] Model update rejected. Performance change: %.10f", client_id, dec.perf_change)
            if st.rejected_updates >= self.max_rejected:
                log.error(f"[Client {client_id}] Too many rejected updates. Possible attack detected.")


class ThesisVerifier(Verifier):
    """The thesis's acceptance rule (Thesis p.20-22 Alg. 4.3, p.26 §4.3.6;
    SURVEY §5.3): accept iff the aggregate's validation loss is finite and
    ``new_loss <= old_loss * (1 + ratio)`` where ``old_loss`` is the
    receiver's own current model on the same data; on reject the receiver
    keeps (restores) its own model.  Rejection counting is unchanged."""

    def __init__(self, ratio: float = 0.1, method: str = "val", max_rejected: int = 3):
        super().__init__(method=method, max_rejected=max_rejected)
        self.ratio = ratio

    def needs_drift(self, st: VerifierState) -> bool:
        return False

    def decide_losses(self, client_id: int, st: VerifierState, version: int, old_loss: float, new_loss: float,
                      current_round: int) -> VerifyDecision:
        import math

        st.history_version, st.history_perf, st.history_round = version, 1.0 / (1.0 + new_loss), current_round
        ok = math.isfinite(new_loss) and new_loss <= old_loss * (1.0 + self.ratio)
        if log.isEnabledFor(logging.INFO):
            log.info(f"Client {client_id} - old loss: {old_loss:.10f}, new loss: {new_loss:.10f}")
        return VerifyDecision(ok, old_loss - new_loss, 0.0)
