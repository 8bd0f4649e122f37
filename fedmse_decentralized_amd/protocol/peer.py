"""Per-client peer API: the reference ``ClientTrainer`` surface as views over
the structure-of-arrays client store.

The reference models every client as a Python object that trains, votes,
aggregates and exchanges ``state_dict`` references with its peers
(`src/Trainer/client_trainer.py:26-419`; messaging `:136-206`, SURVEY C16,
C20-C23, M7).  The federation engine runs the same protocol batched over all
clients (``Federation.run_round``); this module exposes the per-client calls
for users who drive the protocol themselves:

    fed = Federation(cfg, "hybrid", "mse_avg", 0).setup()
    peers = fed.peers()                      # one Peer per hosted client
    for p in peers: p.connect_to_peers([q for q in peers if q is not p])
    a = peers[0]
    a.run()                                  # local training (fused kernel)
    agg = a.aggregate_models(peers[:5])      # weighted reduce on the device
    a.broadcast_model()                      # receive_model() on every peer
    for p in peers[1:]: p.update_from_peers()   # verify + adopt

Models travel as padded parameter vectors on the device (no copies of
``state_dict`` objects); ``receive_model`` stores a reference, exactly like
the reference's inbox.  The calls are local to the rank that hosts the
client (multi-rank runs use ``Federation.run_round``'s collectives).
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .aggregation import make_plan
from .verification import VerifierState

log = logging.getLogger("fedmx")


class Peer:
    def __init__(self, fed, cid: int):
        if not fed._mine(cid):
            raise ValueError(f"client {cid} is not hosted on rank {fed.comm.rank}")
        self.fed = fed
        self.client_id = cid
        self.row = fed._loc(cid)
        self.peers: List["Peer"] = []
        self.received_models: Dict[int, torch.Tensor] = {}
        self.mse_score: Optional[float] = None
        self.votes_received = 0
        self.has_aggregated_this_round = False
        self._vstate = VerifierState()
        self._hist: Optional[torch.Tensor] = None
        self._version = 0

    # -- state ---------------------------------------------------------------
    @property
    def aggregation_count(self) -> int:
        return self.fed.agg_counts[self.client_id]

    @property
    def rejected_updates(self) -> int:
        return self._vstate.rejected_updates

    def params(self) -> torch.Tensor:
        """The client's current padded parameter vector (a device view)."""
        return self.fed.engine.store.params[self.row]

    def state_dict(self) -> Dict[str, torch.Tensor]:
        from ..models.layout import canonical_to_state_dict, padded_to_canonical

        return canonical_to_state_dict(padded_to_canonical(self.params().detach().cpu(), self.fed.dims),
                                       self.fed.dims)

    def __repr__(self):
        return f"Peer({self.client_id})"

    # -- local work ------------------------------------------------------------
    def run(self):
        """Local training (`client_trainer.py:360-419`): returns [(train, valid)] per epoch."""
        res = self.fed.engine.train([self.row], self.fed.hp)
        return [tuple(map(float, t)) for t in res.tracking[0]]

    def calculate_mse_score(self, validation_data, noise: bool = False) -> float:
        """Vote score of this client's model (`client_trainer.py:208-247`):
        re-standardised data, batches of 128, mean of batch MSEs (optional
        tie-break noise)."""
        eng = self.fed.engine
        v = validation_data if isinstance(validation_data, torch.Tensor) else eng.to_device(validation_data)
        out = eng.vote_scores([self.row], v, None, self.fed.cfg.vote_batch_size)
        host = eng.fetch([out])[0]
        s = float(np.asarray(host)[0][0])
        if noise:
            s *= 1.0 + (self.fed.noise.rand() - 0.5) * 0.0002
        self.mse_score = s
        return s

    def vote_for_aggregator(self, selected: Sequence["Peer"], validation_data) -> Optional["Peer"]:
        """Score every other selected peer, vote for the best one below the
        aggregation cap (`client_trainer.py:249-285`)."""
        cap = self.fed.cfg.max_aggregation
        for p in selected:
            p.has_aggregated_this_round = False
        scored = sorted(((p.calculate_mse_score(validation_data, noise=True), i, p)
                         for i, p in enumerate(selected) if p is not self), key=lambda t: (t[0], t[1]))
        for s, _, p in scored:
            if p.aggregation_count < cap:
                p.votes_received += 1
                log.info(f"[Client {self.client_id}] Voting for Client {p.client_id} with MSE score: {s:.6f}")
                return p
        return None

    # -- aggregation -----------------------------------------------------------
    def _aggregate(self, sources: Sequence[torch.Tensor], ids: Sequence[int]) -> torch.Tensor:
        fed = self.fed
        eng = fed.engine
        stack = torch.stack([s.to(eng.store.params.device) for s in sources], 0)
        dev_mse = None
        if fed.update_type == "mse_avg":
            saved = eng.store.params[self.row].clone()
            dev_mse = {}
            for i, cid in zip(range(len(ids)), ids):   # each model's MSE on the shared dev set
                eng.store.params[self.row].copy_(stack[i])
                dev_mse[cid] = float(eng.model_mse([self.row], [fed.dev_set])[0])
            eng.store.params[self.row].copy_(saved)
        sim = fw = None
        if fed.update_type == "fusion_avg":
            if fed._fusion_on_device():
                fw = fed._fusion_weights_t(stack).tolist()
            else:
                sim = fed._fusion_similarity_of(stack, ids)
        plan = make_plan(fed.update_type, list(range(len(ids))), self.client_id,
                         {i: dev_mse[c] for i, c in enumerate(ids)} if dev_mse else None, "fixed",
                         sim={i: sim[c] for i, c in enumerate(ids)} if sim else None, fusion_w=fw)
        return eng.weighted_sum(stack[[i for i, _ in plan]], [w for _, w in plan])

    def aggregate_models(self, selected: Sequence["Peer"]) -> Optional[torch.Tensor]:
        """Aggregate the selected peers' models and load the result
        (`client_trainer.py:287-335`); None when capped or already done."""
        fed = self.fed
        if self.aggregation_count >= fed.cfg.max_aggregation or self.has_aggregated_this_round:
            return None
        agg = self._aggregate([p.params() for p in selected], [p.client_id for p in selected])
        fed.agg_counts[self.client_id] += 1
        self.has_aggregated_this_round = True
        fed.engine.adopt([self.row], agg, anchor=False)
        return agg

    # -- messaging (C22 / M7) ----------------------------------------------------
    def connect_to_peers(self, peers: Sequence["Peer"]) -> None:
        self.peers = list(peers)
        log.info(f"[Client {self.client_id}] Connected to {len(self.peers)} peers")

    def receive_model(self, sender, model: torch.Tensor) -> None:
        key = sender.client_id if isinstance(sender, Peer) else int(sender)
        self.received_models[key] = model
        log.info(f"[Client {self.client_id}] Received model from peer {key}")

    def broadcast_model(self, model: Optional[torch.Tensor] = None) -> None:
        m = self.params().clone() if model is None else model
        for p in self.peers:
            p.receive_model(self, m)
        log.info(f"[Client {self.client_id}] Model broadcasted to all peers")

    def request_aggregation(self) -> Optional[torch.Tensor]:
        """Aggregate the inbox with the client's update rule and return it
        (not loaded), or None when capped / empty (`client_trainer.py:153-172`)."""
        if self.aggregation_count >= self.fed.cfg.max_aggregation or not self.received_models:
            return None
        ids = list(self.received_models)
        agg = self._aggregate([self.received_models[i] for i in ids], ids)
        self.fed.agg_counts[self.client_id] += 1
        self.has_aggregated_this_round = True
        return agg

    def update_from_peers(self) -> Optional[bool]:
        """Verify the first received model and adopt it on success
        (`client_trainer.py:174-206`); clears the inbox."""
        if not self.received_models:
            return None
        fed, eng = self.fed, self.fed.engine
        new = next(iter(self.received_models.values())).to(eng.store.params.device)
        data = fed.dev_set if fed.cfg.verification_method == "dev" else fed.valid_all[self.client_id]
        mse, drift = eng.verify_stats(new, [data], self._hist.unsqueeze(0) if self._hist is not None else None)
        mse_h, drift_h = eng.fetch([mse, drift])
        perf = 1.0 / (1.0 + float(np.asarray(mse_h)[0]))
        dr = float(np.asarray(drift_h)[0]) if self._hist is not None else 0.0
        dec = fed.verifier.decide(self.client_id, self._vstate, self._version, perf, dr, fed.round_idx)
        fed.verifier.apply(self.client_id, self._vstate, dec)
        self._hist = new.clone()
        self._version += 1
        if dec.verified:
            eng.adopt([self.row], new, anchor=True)
        self.received_models.clear()
        return dec.verified
