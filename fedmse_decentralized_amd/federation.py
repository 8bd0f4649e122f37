"""The decentralised federated round loop (one sweep combination).

Reference: the body of the combination loop in `src/main.py:108-379`
(client construction, per-round select -> train -> vote -> aggregate ->
broadcast -> verify -> evaluate -> report -> early stop).

MI355X design:

* every rank (one process per GPU) hosts a contiguous shard of the clients
  in an engine (device-resident data + SoA client state);
* protocol *decisions* (selection, election, aggregation plan, early stop)
  are a replicated state machine: every rank computes them from identical
  inputs, so no decision ever needs to be broadcast;
* the logical peer messages are three tiny collectives per round
  (score all-reduce, parameter all-gather, metric all-reduce) over RCCL;
* all selected clients of a rank train concurrently in one fused kernel
  launch; evaluation of all hosted clients is a few batched launches.
"""
from __future__ import annotations

import logging
import os
import random
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .config import ExperimentConfig, load_device_list
from .data.csv import load_data
from .data.prepare import ClientData, prepare_federation
from .data.synthetic import ClientRaw, SyntheticSpec, generate_client
from .engine import Engine, TrainHParams, make_engine
from .eval.evaluator import evaluate_clients
from .io import checkpoint as ckpt
from .io import reports
from .io.async_writer import AsyncWriter, snapshot_to_host
from .models.layout import P_PAD, ModelDims
from .models.reference import init_client_params
from .parallel.comm import Comm, LoopbackComm
from .parallel.sharding import ShardMap
from .protocol.aggregation import make_plan
from .protocol.early_stop import GlobalEarlyStop
from .protocol.election import OneDraw, elect_aggregator, elect_majority, select_clients
from .protocol.verification import ThesisVerifier, Verifier, VerifierState
from .utils.rng_replay import HostNoise, TorchRngReplay
from .utils.telemetry import Telemetry

log = logging.getLogger("fedmx")

_PREP_CACHE: Dict[tuple, Tuple[List[ClientData], np.ndarray]] = {}


# ----------------------------------------------------------------------------
# data
# ----------------------------------------------------------------------------

def _load_optional(path: str, n_cols: int, name: str) -> np.ndarray:
    """A client's abnormal rows, or none: the shipped N-BaIoT non-IID split
    lacks ``abnormal/`` for clients 6, 9 and 10 (`/root/reference/.MISSING_LARGE_BLOBS:4-6`).
    Such a client trains, votes and verifies as usual; its test set holds
    normal rows only, so its detection AUC is undefined: reported as null and
    left out of every mean / min / max (io/reports.py, metric_stats)."""
    try:
        return load_data(path)
    except FileNotFoundError:
        log.warning(f"{name}: no abnormal data at {path}: AUC undefined for this client (reported as null)")
        return np.zeros((0, n_cols), dtype=np.float64)


def metric_stats(metrics) -> Tuple[float, float, float]:
    """(mean, min, max) over the clients whose metric is defined (a client
    without abnormal test rows has a NaN AUC); NaN when none is."""
    m = np.asarray(metrics, dtype=np.float64)
    m = m[~np.isnan(m)]
    if m.size == 0:
        return float("nan"), float("nan"), float("nan")
    return float(m.mean()), float(m.min()), float(m.max())


def load_federation_data(cfg: ExperimentConfig, py_rng: random.Random) -> Tuple[List[ClientData], np.ndarray]:
    """Device sampling + per-client preparation with the reference RNG order.

    Consumes ``py_rng`` exactly like `src/main.py:126` (``random.sample`` of
    the device list); the numpy RNG is a private ``RandomState(data_seed)``.
    Prepared data is cached per process (identical for every combination).
    """
    if cfg.synthetic:
        spec = SyntheticSpec(kind=cfg.synthetic, n_clients=cfg.network_size, iid=cfg.synthetic_iid,
                             alpha=cfg.synthetic_alpha, seed=cfg.synthetic_seed)
        entries = list(range(cfg.network_size))
        chosen = py_rng.sample(entries, cfg.network_size)
        key = ("synthetic", cfg.synthetic, cfg.network_size, cfg.synthetic_iid, cfg.synthetic_alpha,
               cfg.synthetic_seed, cfg.data_seed, cfg.new_device, cfg.scaler, tuple(chosen))
        if key not in _PREP_CACHE:
            raws = [generate_client(spec, i) for i in chosen]
            _PREP_CACHE[key] = prepare_federation(raws, cfg.data_seed, cfg.new_device, cfg.scaler)
        return _PREP_CACHE[key]
    dl = load_device_list(cfg.config_file)
    if len(dl.devices_list) < cfg.network_size:
        raise ValueError(f"{cfg.config_file} lists {len(dl.devices_list)} devices < network_size {cfg.network_size}")
    chosen = py_rng.sample(dl.devices_list, cfg.network_size)
    key = ("csv", os.path.abspath(cfg.config_file), cfg.network_size, cfg.data_seed, cfg.new_device, cfg.scaler,
           tuple(d.name for d in chosen))
    if key not in _PREP_CACHE:
        raws = []
        for d in chosen:
            log.info("Loading data from {}...".format(d.name))
            normal = load_data(dl.resolve(d.normal_data_path))
            abnormal = _load_optional(dl.resolve(d.abnormal_data_path), normal.shape[1], d.name)
            if cfg.new_device:
                if not d.test_normal_data_path:
                    raise ValueError(f"device {d.name} has no test_normal_data_path (needed with new_device)")
                tn = load_data(dl.resolve(d.test_normal_data_path))
            else:
                tn = np.zeros((0, normal.shape[1]))
            log.info(f"{d.name} has {len(normal)} normal data and {len(abnormal)} abnormal data")
            raws.append(ClientRaw(d.name, normal, abnormal, tn))
        _PREP_CACHE[key] = prepare_federation(raws, cfg.data_seed, cfg.new_device, cfg.scaler)
    return _PREP_CACHE[key]


# ----------------------------------------------------------------------------
# federation
# ----------------------------------------------------------------------------

@dataclass
class RoundResult:
    round: int
    selected: List[int]
    aggregator: Optional[int]
    metrics: np.ndarray
    verification: List[Dict]
    epochs_run: Dict[int, int]
    stop: bool = False
    times_ms: Dict[str, float] = field(default_factory=dict)


class _TableNoise:
    """Noise source replaying a pre-drawn table (fixed-compat election)."""

    def __init__(self, table):
        self.table = table
        self.i = 0

    def rand(self) -> float:
        v = self.table[self.i]
        self.i += 1
        return v


class Federation:
    def __init__(self, cfg: ExperimentConfig, model_type: str, update_type: str, run: int,
                 comm: Optional[Comm] = None, device: Optional[torch.device] = None,
                 early_stop: Optional[GlobalEarlyStop] = None, engine: Optional[Engine] = None,
                 telemetry: Optional[Telemetry] = None, write_reports: bool = True,
                 writer: Optional[AsyncWriter] = None):
        self.cfg = cfg
        self.model_type = model_type
        self.update_type = update_type
        self.run = run
        if comm is None and device is None:
            device = cfg.resolved_device()
        self.comm = comm or LoopbackComm(device)
        self.device = torch.device(device) if device is not None else self.comm.device
        self.dims = ModelDims(cfg.dim_features, cfg.hidden_neus, cfg.latent_dim)
        self.early = early_stop or GlobalEarlyStop(cfg.global_patience, cfg.compat)
        self.engine = engine or make_engine(cfg.backend, self.dims, self.device)
        self.tel = telemetry or Telemetry(cfg.trace_file, sync_fn=self.engine.synchronize, rank=self.comm.rank)
        self.write_reports = write_reports and self.comm.is_root
        self.round_idx = 0
        self.last_metrics: Optional[np.ndarray] = None
        self.latent_log: Dict[int, Dict[str, Tuple[np.ndarray, np.ndarray]]] = {}
        self.writer = writer or _default_writer()
        self.defer_verification = False     # set by the concurrent sweep (main.py)
        self._deferred_vr: List[Tuple[int, List[Dict]]] = []

    # -- setup -------------------------------------------------------------------
    def setup(self):
        cfg = self.cfg
        # set_seeds(run*10000) then random/np re-seeded with data_seed (src/main.py:115-117)
        self.py_rng = random.Random(cfg.data_seed)
        clients, dev = load_federation_data(cfg, self.py_rng)
        self.clients = clients
        N = len(clients)
        self.N = N
        self.shard = ShardMap(N, self.comm.world_size)
        self.local = self.shard.local_ids(self.comm.rank)
        init, rng_state = init_client_params(N, self.run * 10000, self.dims)
        if cfg.resolved_init_mode() == "shared":
            # one global initial model (the RNG state after all N inits is kept,
            # so the reference's draw order downstream is unchanged)
            init = init[:1].expand(N, -1).clone()
        self.noise = TorchRngReplay(rng_state, self.dims) if cfg.compat == "reference" else HostNoise(self.run * 10000 + 17)
        eng = self.engine
        loc = [clients[c] for c in self.local]
        eng.setup([c.train for c in loc], [c.valid for c in loc], [c.test for c in loc],
                  [c.test_label for c in loc], init[self.local[0]:self.local[-1] + 1] if self.local else init[:0])
        # replicated small tensors: every client's validation set (vote data) and the dev set
        self.valid_all = [eng.to_device(c.valid) for c in clients]
        self.dev_set = eng.to_device(dev)
        self.agg_counts = [0] * N
        if cfg.protocol_variant == "thesis":
            self.verifier = ThesisVerifier(cfg.thesis_loss_ratio, cfg.verification_method, cfg.max_rejected_updates)
        else:
            self.verifier = Verifier(cfg.verification_threshold, cfg.performance_threshold,
                                     cfg.verification_method, cfg.max_rejected_updates, cfg.drift_threshold_rel)
        # thesis variant: random aggregator fallback (own stream: the reference RNG order is untouched)
        self.fallback_rng = random.Random(cfg.data_seed + 7919 * (self.run + 1)) \
            if cfg.protocol_variant == "thesis" else None
        self._dev_kde = None
        self._dev_kde_t = None   # (dev-row KDE scores, dev rows, padded -> canonical index) on the engine's device
        self.vstate: Dict[int, VerifierState] = {c: VerifierState() for c in self.local}
        self.versions: Dict[int, torch.Tensor] = {}
        self.last_received: List[Optional[int]] = [None] * N
        self.hp = TrainHParams(
            epochs=cfg.epoch, batch_size=cfg.batch_size, lr=cfg.lr_rate,
            shrink_lambda=float(cfg.shrink_lambda) if self.model_type == "hybrid" else 0.0,
            fedprox_mu=cfg.fedprox_mu if self.update_type == "fedprox" else 0.0,
            patience=cfg.global_patience)
        from .models.layout import padded_index

        self._canon_idx = padded_index(self.dims)[0].numpy()
        self.save_dirs = {c: cfg.client_save_dir(self.run, self.model_type, self.update_type, clients[c].name)
                          for c in self.local}
        if cfg.save_checkpoints:
            for d in self.save_dirs.values():
                os.makedirs(d, exist_ok=True)
        snap = ckpt.load_resume(self._resume_path(cfg.resume)) if cfg.resume else None
        if snap is not None:
            self.restore(snap)
        self._fast = None
        from .engine.device_round import DeviceRound, fast_path_supported

        why = fast_path_supported(self)
        if why is None:
            self._fast = DeviceRound(self)
            if snap is not None and snap.get("device"):
                self._fast.restore(snap["device"])
            elif snap is not None:
                # a host-path snapshot resumed on the device path: the device
                # protocol state starts from the restored host state
                self._fast.seed_from_host()
        else:
            log.debug(f"device protocol off: {why}")
        return self

    def reset_aggregation_counts(self) -> None:
        """New protocol episode: every client may aggregate max_aggregation times again."""
        self.agg_counts = [0] * self.N
        if self._fast is not None:
            self._fast.reset_aggregation_counts()

    def finish(self) -> None:
        """Collect every enqueued device round (reports handed to the writer)."""
        if getattr(self, "_fast", None) is not None:
            self._fast.collect_all()

    def check_replicas(self, rnd: int, selected, aggregator, metrics) -> None:
        """Fail loudly if the replicated protocol state differs between ranks."""
        import hashlib

        h = hashlib.sha256()
        h.update(repr((rnd, list(selected), aggregator, list(self.agg_counts))).encode())
        h.update(np.ascontiguousarray(metrics, dtype=np.float64).tobytes())
        digest = h.hexdigest()
        allh = self.comm.all_gather_object(digest)
        if len(set(allh)) != 1:
            raise RuntimeError(f"replicated protocol state diverged at round {rnd + 1}: {allh}")

    # -- report / artefact submission (background writer) ---------------------------
    def _report_round(self, rnd: int, metrics: np.ndarray) -> None:
        reports.append_round_result(self.cfg, self.run, rnd, metrics, self.model_type, self.update_type,
                                    files=self.writer.files)

    def _report_verification(self, rnd: int, vr: List[Dict]) -> None:
        if self.defer_verification:
            # the run's verification file is shared by every combination
            # (src/main.py:313-326): concurrent combinations hold their lines
            # back and write them at conclude(), in combination order
            self._deferred_vr.append((rnd, vr))
            return
        reports.append_verification(self.cfg, self.run, rnd, vr, files=self.writer.files)

    def _flush_deferred_verification(self) -> None:
        for rnd, vr in self._deferred_vr:
            reports.append_verification(self.cfg, self.run, rnd, vr, files=self.writer.files)
        self._deferred_vr = []

    def _submit_checkpoints(self, res, local_sel: Sequence[int], snap, ev) -> None:
        # one job per round: every trained client's model.cpt + tracking pickle
        # rendered and written by the native batched writer (io.checkpoint)
        dirs = [self.save_dirs[c] for c in local_sel]
        rows = [self._loc(c) for c in local_sel]
        improved = [bool(res.best_epoch[i] >= 0) for i in range(len(local_sel))]
        trks = [list(res.tracking[i]) for i in range(len(local_sel))]
        dims, cidx = self.dims, self._canon_idx

        def job(files=self.writer.files):
            ckpt.write_round_artifacts(files, dirs, snap.numpy(), rows, improved, trks, cidx, dims)
        self.writer.submit(job, ev)

    def _resume_path(self, base: str) -> str:
        return base if self.comm.world_size == 1 else f"{base}.rank{self.comm.rank}"

    # -- helpers -------------------------------------------------------------------
    def _loc(self, cid: int) -> int:
        return self.shard.to_local(self.comm.rank, cid)

    def _mine(self, cid: int) -> bool:
        s, e = self.shard.bounds(self.comm.rank)
        return s <= cid < e

    def _gather_params(self, sources: Sequence[int], selected: Sequence[int]) -> torch.Tensor:
        """Stack [len(sources), P] of the given clients' params (identical on all ranks).

        World size 1: a device gather from the local store.  Otherwise every
        rank packs its selected clients (selected order) into fixed slots and
        one RCCL all-gather over xGMI delivers every rank's slots
        ([world, slots, 9216] fp32) — the reference's "collect all selected
        state_dicts" (`src/Trainer/client_trainer.py:306-315`) without a
        single aggregator sink.
        """
        st = self.engine.store
        if not self.comm.collective:
            rows = [self._loc(c) for c in sources]
            if rows == list(range(rows[0], rows[0] + len(rows))) if rows else False:
                return st.params[rows[0]:rows[0] + len(rows)]
            return torch.stack([st.params[r] for r in rows], 0)
        per_rank: Dict[int, List[int]] = {}
        for c in selected:
            per_rank.setdefault(self.shard.owner(c), []).append(c)
        slots = max(len(v) for v in per_rank.values())
        mine = per_rank.get(self.comm.rank, [])
        send = torch.zeros(slots, P_PAD, dtype=torch.float32, device=st.params.device)
        for i, c in enumerate(mine):
            send[i].copy_(st.params[self._loc(c)])
        allg = self.comm.all_gather(send)        # [world, slots, P]
        return torch.stack([allg[self.shard.owner(c), per_rank[self.shard.owner(c)].index(c)] for c in sources], 0)

    def _write_checkpoints(self, res, local_sel: Sequence[int]) -> None:
        """model.cpt (best-validation snapshot of this round's training) and
        training_tracking.pkl per trained client, written by the background
        writer from an asynchronous device->pinned copy."""
        snap, ev = snapshot_to_host(self.engine.store.best)
        self._submit_checkpoints(res, local_sel, snap, ev)

    # -- one round ---------------------------------------------------------------
    def run_round(self) -> RoundResult:
        cfg, eng, st = self.cfg, self.engine, self.engine.store
        rnd = self.round_idx
        N = self.N
        info = log.isEnabledFor(logging.INFO)
        if info:
            log.info(f"Starting round {rnd + 1}/{cfg.num_rounds}")

        with self.tel.phase("select"):
            selected = select_clients(self.py_rng, N, cfg.num_participants)
            if cfg.dropped_clients:   # fault injection: offline clients neither train, vote nor aggregate
                selected = [c for c in selected if c not in cfg.dropped_clients]
        if self._fast is not None:
            return self._fast.enqueue(selected)
        # aggregation_mode "local": local-training-only ablation (same
        # selections, training and evaluation; no election, no aggregate)
        local_only = cfg.aggregation_mode == "local"
        with self.tel.phase("select"):
            local_sel = [c for c in selected if self._mine(c)]
            local_rows = [self._loc(c) for c in local_sel]

        # ---------------- local training of all local selected clients: one launch
        with self.tel.phase("train"):
            if info:
                for c in local_sel:
                    log.info(f"Training client {c + 1}...")
            handle = eng.train_launch(local_rows, self.hp) if local_sel else None
            if local_sel and cfg.malicious_clients:
                for c in local_sel:
                    if c in cfg.malicious_clients:   # fault injection: poisoned update
                        st.params[self._loc(c)].mul_(cfg.malicious_scale)

        # ---------------- vote scores (+ FedMSE dev MSE) of the local selected clients
        with self.tel.phase("vote"):
            need_dev = self.update_type == "mse_avg"
            vote_data = self.valid_all[selected[0]] if selected else self.dev_set
            scores_dev = eng.vote_scores(local_rows, vote_data,
                                         self.dev_set if need_dev else None, cfg.vote_batch_size)
            # first host sync of the round: training results + scores
            host = eng.fetch((handle.tensors if handle is not None else []) + [scores_dev])
            scores_np = host[-1]
            res = eng.train_collect(handle, host[:-1] if handle.tensors else None) if handle is not None else None
        epochs_local: Dict[int, int] = {}
        if res is not None:
            for i, c in enumerate(local_sel):
                epochs_local[c] = int(res.epochs_run[i])
                if info:
                    for e, (tl, vl) in enumerate(res.tracking[i]):
                        log.info(f"[Client {c}] Epoch {e + 1} - Training loss: {tl} - Validating loss: {vl}")
                    log.info(f"Client {c + 1} training done!")
            if cfg.save_checkpoints:
                with self.tel.phase("io"):
                    self._write_checkpoints(res, local_sel)
        log.info("Starting voting for aggregator...")
        vec = np.zeros((N, 3), dtype=np.float64)
        if local_sel:
            ls = np.asarray(local_sel)
            vec[ls, 0] = scores_np[:, 0]
            vec[ls, 1] = scores_np[:, 1] if need_dev else 0.0
            vec[ls, 2] = [epochs_local.get(c, 0) for c in local_sel]
        with self.tel.phase("comm"):
            vec = self.comm.all_reduce_sum(vec)
        with self.tel.phase("vote"):
            base_scores = {c: float(vec[c, 0]) for c in selected}
            dev_mse = {c: float(vec[c, 1]) for c in selected}
            epochs_all = {c: int(vec[c, 2]) for c in selected}
            # torch-RNG replay (compat): one iterator per train and per valid epoch loop
            self.noise.iterators(2 * sum(epochs_all.values()))
            elect = elect_majority if cfg.election == "majority" else elect_aggregator
            cap = cfg.thesis_vote_mse_cap if cfg.protocol_variant == "thesis" else None
            noise = self.noise
            if cfg.compat == "fixed":
                # one k x (k-1) table per round, drawn whatever the outcome (the
                # device protocol draws the same table)
                k = len(selected)
                noise = _TableNoise([float(u) for u in self.noise.rand_n(k * (k - 1))])
            fb = OneDraw(self.fallback_rng.random()) if self.fallback_rng is not None else None
            if local_only:
                aggregator = None   # ablation: nobody aggregates, nobody adopts
            else:
                el = elect(selected, base_scores, self.agg_counts, cfg.max_aggregation, noise,
                           log_enabled=info, vote_mse_cap=cap, fallback_rng=fb)
                aggregator = el.aggregator

        verification_results: List[Dict] = []
        if aggregator is not None:
            if info:
                log.info(f"Client {aggregator + 1} selected as aggregator")
            with self.tel.phase("aggregate"):
                if self.update_type == "mse_avg" and cfg.compat == "reference":
                    for _ in selected:          # calculate_mse_score per client (weights unused, Q3)
                        self.noise.rand()
                sim = fw = None
                if self.update_type == "fusion_avg":
                    if self._fusion_on_device():
                        fw = self._fusion_weights_t(self._gather_params(list(selected), selected)).tolist()
                    else:
                        sim = self._fusion_similarity(selected)
                ns = {c: self.clients[c].train.shape[0] for c in selected} if cfg.fedavg_sample_weighted else None
                plan = make_plan(self.update_type, selected, aggregator, dev_mse, cfg.compat, sim=sim,
                                 num_samples=ns, fusion_w=fw)
            with self.tel.phase("comm"):
                stack = self._gather_params([c for c, _ in plan], selected)
            with self.tel.phase("aggregate"):
                agg = eng.weighted_sum(stack, [w for _, w in plan])
                self.agg_counts[aggregator] += 1
                if self._mine(aggregator):
                    eng.adopt([self._loc(aggregator)], agg, anchor=False)
                version = rnd
                self.versions[version] = agg
            if cfg.aggregation_mode == "centralized":
                # server push (legacy GlobalAggregator.update): every hosted client
                # loads the aggregate and re-anchors FedProx; nothing is verified
                with self.tel.phase("aggregate"):
                    others = [self._loc(c) for c in self.local if c != aggregator]
                    eng.adopt(others, agg, anchor=True)
                    if self._mine(aggregator):
                        eng.adopt([self._loc(aggregator)], agg, anchor=True)
                    self.versions.pop(version, None)
            else:
                with self.tel.phase("verify"):
                    verification_results = self._verify_all(agg, version, aggregator, rnd)
            if self.write_reports and cfg.aggregation_mode != "centralized":
                if info:
                    log.info("Verification results for this round:")
                    for r_ in verification_results:
                        log.info(f"Client {r_['client_id']}: {'Verified' if r_['is_verified'] else 'Rejected'} "
                                 f"(Rejected updates: {r_['rejected_updates']})")
                vr = verification_results
                self.writer.submit(lambda vr=vr, rnd=rnd: self._report_verification(rnd, vr))
        elif not local_only:
            log.warning("No aggregator selected for this round")

        # ---------------- evaluation of every hosted client (batched launches)
        log.info("Calculating metrics for all models...")
        with self.tel.phase("eval"):
            er = eng.evaluate(self.model_type, cfg.metric, keep_latents=cfg.save_latents)
            vec = np.zeros(N, dtype=np.float64)
            if self.local:   # a rank may host no client (fewer clients than ranks)
                vec[self.local[0]:self.local[-1] + 1] = er.metrics
        with self.tel.phase("comm"):
            vec = self.comm.all_reduce_sum(vec)
        metrics = np.array(vec, dtype=np.float64)
        self.noise.iterators(N * (2 if self.model_type == "hybrid" else 1))
        if info:
            for i in range(N):
                log.info(f"Client {i + 1} {cfg.metric} score: {metrics[i]}")
        if cfg.save_latents and er.latents is not None:
            names = [self.clients[c].name for c in self.local]
            self.latent_log[rnd] = {n: l for n, l in zip(names, er.latents)}
        if self.write_reports:
            m_ = metrics.copy()
            self.writer.submit(lambda m_=m_, rnd=rnd: self._report_round(rnd, m_))
        self.last_metrics = metrics
        if cfg.debug_replica_check:
            self.check_replicas(rnd, selected, aggregator, metrics)
        stop = False
        if cfg.global_early_stop:
            stop = self.early.update(metric_stats(metrics)[1])
        self.round_idx += 1
        times = self.tel.end_round(round=rnd + 1, selected=len(selected), aggregator=aggregator)
        return RoundResult(rnd, list(selected), aggregator, metrics, verification_results, epochs_all, stop, times)

    def _verify_all(self, agg: torch.Tensor, version: int, aggregator: int, rnd: int) -> List[Dict]:
        """Every receiver verifies the broadcast aggregate (all N clients but the
        aggregator, Q14): one batched forward for the verification MSEs, one
        drift launch, one host sync, then the accepted receivers adopt the
        aggregate (and refresh their FedProx anchor) in one launch."""
        cfg, eng = self.cfg, self.engine
        N = self.N
        receivers = [c for c in self.local if c != aggregator]
        if cfg.verification_method == "dev":
            key_of = {c: "dev" for c in receivers}
            data_of = {"dev": self.dev_set}
        elif cfg.compat == "reference":
            # every client verifies on the last-constructed client's validation set (Q4)
            key_of = {c: "vlast" for c in receivers}
            data_of = {"vlast": self.valid_all[N - 1]}
        else:
            key_of = {c: f"v{c}" for c in receivers}
            data_of = {f"v{c}": self.valid_all[c] for c in receivers}
        keys = sorted(set(key_of.values()))
        need = sorted({self.vstate[c].history_version for c in receivers if self.vstate[c].history_version is not None})
        hist = torch.stack([self.versions[v] for v in need], 0) if need else None
        thesis = isinstance(self.verifier, ThesisVerifier)
        if thesis:
            hist = None
        mse_t, drift_t = eng.verify_stats(agg, [data_of[k] for k in keys], hist)
        mse_np, drift_np = eng.fetch([mse_t, drift_t])
        perf = {k: 1.0 / (1.0 + float(m)) for k, m in zip(keys, mse_np)}   # 1 / (1 + MSE)
        new_loss = {k: float(m) for k, m in zip(keys, mse_np)}
        old_loss = {}
        if thesis and receivers:   # each receiver's own current model on the same data
            own = eng.model_mse([self._loc(c) for c in receivers], [data_of[key_of[c]] for c in receivers])
            old_loss = {c: float(x) for c, x in zip(receivers, own)}
        drift = {v: float(x) for v, x in zip(need, drift_np)}
        hnorm = {}
        if need and cfg.drift_threshold_rel > 0 and not thesis:
            # relative drift limit: sum_tensors ||history||_2 of each history version
            hn = eng.fetch([eng.param_drift(hist, torch.zeros_like(agg))])[0]
            hnorm = {v: float(x) for v, x in zip(need, hn)}
        accept = []
        vec = np.zeros((N, 2), dtype=np.float64)
        for c in receivers:
            vs_ = self.vstate[c]
            if thesis:
                dec = self.verifier.decide_losses(c, vs_, version, old_loss[c], new_loss[key_of[c]], rnd)
            else:
                dr = drift.get(vs_.history_version, 0.0) if vs_.history_version is not None else 0.0
                dec = self.verifier.decide(c, vs_, version, perf[key_of[c]], dr, rnd,
                                           hist_norm=hnorm.get(vs_.history_version))
            self.verifier.apply(c, vs_, dec)
            if dec.verified:
                accept.append(c)
            vec[c, 0] = vs_.rejected_updates
            vec[c, 1] = 1.0
        if accept:
            eng.adopt([self._loc(c) for c in accept], agg, anchor=True)  # previous_global_model = deepcopy(model)
        self.noise.model_inits(N - 1)                # verifier builds a fresh model per call (Q16)
        # replicated bookkeeping: every non-aggregator received this version;
        # drop aggregate versions no client references any more
        for c in range(N):
            if c != aggregator:
                self.last_received[c] = version
        live = {v for v in self.last_received if v is not None}
        for v in list(self.versions):
            if v not in live:
                del self.versions[v]
        vec = self.comm.all_reduce_sum(vec)
        out = []
        for c in range(N):
            if c == aggregator:
                continue
            rej = int(vec[c, 0])
            out.append({"client_id": c, "rejected_updates": rej, "is_verified": rej == 0})
        return out

    def _fusion_similarity(self, selected: Sequence[int]) -> Dict[int, float]:
        """fusion_avg: JS distance between the KDE density of the dev set and
        that of each selected model's reconstruction of it (host, subsampled
        to ``fusion_max_rows`` dev rows; identical on every rank)."""
        return self._fusion_similarity_of(self._gather_params(list(selected), selected), selected)

    def _fusion_on_device(self) -> bool:
        """The HIP engine forms the fusion weights on the GPU (torch, float64:
        the same computation for the host-decision path and the device round)."""
        return self.engine.name == "hip"

    def _fusion_weights_t(self, stack: torch.Tensor) -> torch.Tensor:
        """[k] float64 fusion_avg weights of the stacked models, on the stack's
        device with no host round trip: each model's reconstruction of the
        first ``fusion_max_rows`` dev rows, the JS distance of its KDE to the
        dev set's, w ~ 1 / distance (utils.similarity ``*_t``)."""
        from .models.layout import padded_index
        from .models.reference import functional_forward, unflatten
        from .utils.similarity import fusion_weights_t, js_distance_t, kde_log_density_t

        dv = stack.device
        if self._dev_kde_t is None or self._dev_kde_t[0].device != dv:
            D = self.dims.d_in
            rows = self.dev_set[: self.cfg.fusion_max_rows, :D].detach().to(dv, torch.float32).contiguous()
            idx = padded_index(self.dims)[0].to(dv)   # once: a per-round host -> device copy would synchronise
            self._dev_kde_t = (kde_log_density_t(rows), rows, idx)
        kde, rows, idx = self._dev_kde_t
        out = []
        with torch.no_grad():
            for i in range(stack.shape[0]):
                t = unflatten(stack[i].float().index_select(-1, idx), self.dims)
                _, y = functional_forward(t, rows)
                out.append(js_distance_t(kde, kde_log_density_t(y)))
            return fusion_weights_t(torch.stack(out))

    def _fusion_similarity_of(self, stack: torch.Tensor, ids: Sequence[int]) -> Dict[int, float]:
        from .models.layout import padded_to_canonical
        from .models.reference import functional_forward, unflatten
        from .utils.similarity import kde_log_density, similarity_score

        D = self.dims.d_in
        dev = self.dev_set[: self.cfg.fusion_max_rows, :D].detach().float().cpu()
        if self._dev_kde is None:
            self._dev_kde = kde_log_density(dev.numpy())
        stack = stack.detach().float().cpu()
        out = {}
        with torch.no_grad():
            for i, c in enumerate(ids):
                t = unflatten(padded_to_canonical(stack[i], self.dims), self.dims)
                _, y = functional_forward(t, dev)
                out[c] = similarity_score(self._dev_kde, y.numpy())
        return out

    # -- per-client peer API (reference ClientTrainer surface) ----------------------
    def peer(self, cid: int):
        from .protocol.peer import Peer

        return Peer(self, cid)

    def peers(self):
        return [self.peer(c) for c in self.local]

    # -- whole combination -------------------------------------------------------
    def run_all(self) -> float:
        """Run ``num_rounds`` rounds (or until global early stop); returns the
        combination's best metric (max over clients of the final models,
        `src/main.py:367-374`)."""
        while not self.step():
            pass
        return self.conclude()

    def step(self) -> bool:
        """One round of ``run_all`` (with its snapshot); True when the
        combination is done (round limit reached or global early stop)."""
        return self.end_step(self.begin_step())

    def begin_step(self):
        """Issue the next round (on the device path: enqueue it, results
        collected lazily); None when the round limit is reached."""
        if self.round_idx >= self.cfg.num_rounds:
            return None
        return self.run_round()

    def end_step(self, r) -> bool:
        """Finish a round from ``begin_step``: snapshot, early-stop decision
        (which reads the round's metrics); True when the combination is done."""
        cfg = self.cfg
        if r is None:
            return True
        if cfg.snapshot_every and self.round_idx % cfg.snapshot_every == 0:
            self.save_snapshot()
        if cfg.global_early_stop and r.stop:
            return True
        return self.round_idx >= cfg.num_rounds

    def conclude(self) -> float:
        """End of the combination: collect every round, flush the artefacts,
        latent pickles; the combination's best metric."""
        cfg = self.cfg
        self.finish()
        if self.defer_verification and self.write_reports:
            # after every round's report job (the writer runs jobs in order)
            self.writer.submit(self._flush_deferred_verification)
        if self.last_metrics is None:
            er = self.engine.evaluate(self.model_type, cfg.metric)
            vec = torch.zeros(self.N, dtype=torch.float64)
            for i, c in enumerate(self.local):
                vec[c] = float(er.metrics[i])
            self.last_metrics = self.comm.all_reduce_sum(vec).numpy()
        self.writer.flush()
        if cfg.save_latents and self.latent_log:
            parts = self.comm.all_gather_object(self.latent_log)
            if self.comm.is_root:
                merged: Dict[int, Dict] = {}
                for p in parts:
                    for r, d in p.items():
                        merged.setdefault(r, {}).update(d)
                path = os.path.join(cfg.output_root, f"Checkpoint/LatentData/{cfg.network_size}/{cfg.experiment_name}/"
                                    f"Run_{self.run}/latent_{self.model_type}_{self.update_type}.pkl")
                ckpt.save_latents(path, merged)
        return metric_stats(self.last_metrics)[2]

    # -- resume ---------------------------------------------------------------------
    def snapshot(self) -> Dict:
        # device-resident rounds still in flight are collected first, so the
        # host-side state (metrics, early stop, counters) is the round's own
        self.finish()
        st = self.engine.store
        vers = sorted(self.versions)
        return {
            "host_noise": self.noise.get_state() if isinstance(self.noise, HostNoise) else [],
            "device": self._fast.snapshot() if getattr(self, "_fast", None) is not None else {},
            "round_idx": self.round_idx,
            "params": st.params.cpu(), "adam_m": st.adam_m.cpu(), "adam_v": st.adam_v.cpu(),
            "adam_step": st.adam_step.cpu(), "anchor": st.anchor.cpu(), "best": st.best.cpu(),
            "agg_counts": torch.tensor(self.agg_counts, dtype=torch.int64),
            "last_received": torch.tensor([-1 if v is None else v for v in self.last_received], dtype=torch.int64),
            "vstate": {int(c): [(-1 if s.history_version is None else int(s.history_version)), float(s.history_perf),
                                int(s.history_round), int(s.rejected_updates)] for c, s in self.vstate.items()},
            "versions": {int(v): self.versions[v].cpu() for v in vers},
            "py_rng": _py_state_to_list(self.py_rng.getstate()),
            "fallback_rng": _py_state_to_list(self.fallback_rng.getstate()) if self.fallback_rng is not None else [],
            "noise_state": self.noise.state.clone() if isinstance(self.noise, TorchRngReplay) else torch.zeros(0),
            "early": [float(self.early.best), int(self.early.worse)],
            "last_metrics": torch.from_numpy(self.last_metrics) if self.last_metrics is not None else torch.zeros(0),
        }

    def save_snapshot(self, path: Optional[str] = None) -> str:
        base = path or os.path.join(self.cfg.output_root, "Checkpoint", "resume",
                                    f"{self.cfg.experiment_name}_{self.model_type}_{self.update_type}_run{self.run}.pt")
        return ckpt.save_resume(self._resume_path(base), self.snapshot())

    def restore(self, s: Dict) -> None:
        st = self.engine.store
        self.round_idx = int(s["round_idx"])
        for k in ("params", "adam_m", "adam_v", "anchor", "best"):
            getattr(st, k).copy_(s[k].to(st.params.device))
        st.adam_step.copy_(s["adam_step"].to(st.adam_step.device))
        self.agg_counts = [int(x) for x in s["agg_counts"].tolist()]
        self.last_received = [None if v < 0 else int(v) for v in s["last_received"].tolist()]
        for c, (hv, hp, hr, rej) in s["vstate"].items():
            self.vstate[int(c)] = VerifierState(None if hv < 0 else hv, hp, hr, rej)
        self.versions = {int(v): t.to(st.params.device) for v, t in s["versions"].items()}
        self.py_rng.setstate(_py_state_from_list(s["py_rng"]))
        if self.fallback_rng is not None and s.get("fallback_rng"):
            self.fallback_rng.setstate(_py_state_from_list(s["fallback_rng"]))
        if isinstance(self.noise, TorchRngReplay) and s["noise_state"].numel():
            self.noise.state = s["noise_state"].clone()
        self.early.best, self.early.worse = float(s["early"][0]), int(s["early"][1])
        if s["last_metrics"].numel():
            self.last_metrics = s["last_metrics"].numpy()
        if isinstance(self.noise, HostNoise) and s.get("host_noise"):
            self.noise.set_state(s["host_noise"])


_WRITER: Optional[AsyncWriter] = None


def _default_writer() -> AsyncWriter:
    global _WRITER
    if _WRITER is None:
        _WRITER = AsyncWriter(enabled=True)
    return _WRITER


def _py_state_to_list(state):
    version, internal, gauss = state
    return [int(version), list(internal), gauss]


def _py_state_from_list(lst):
    version, internal, gauss = lst
    return (int(version), tuple(int(x) for x in internal), gauss)
