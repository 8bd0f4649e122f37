"""Device-resident decentralised round (the fixed-compat fast path).

The host path (``Federation.run_round``) takes the protocol decisions on the
host and therefore synchronises with the GPU three times per round (after
training + voting, after verification, after evaluation).  With
``compat="fixed"`` every decision input is either on the device or drawn from
a host RNG whose consumption does not depend on results, so the whole round
can be *enqueued* instead:

    train (fused kernel, all local selected clients)
    forward + score_reduce -> vec[N,4] (vote score, dev MSE)
                            [with collectives: records straight into the send
                            buffer's row 0, the pack of the selected models in
                            extra workgroups of the same launch]
    [ONE all-gather (RCCL, or --comm ipc): the selected models + their vote records]
    elect_wsum_kernel       aggregator (first voter / majority, thesis cap and
                            fallback), FedAvg / FedMSE / sample weights, aggregate
    verify_decide_kernel    fused: forward(agg, every hosted client's verification
                            data) [+ own model: thesis], MSE + drift reductions,
                            ModelVerifier / thesis rule (or centralised push),
                            adoption, history, aggregation-cap count, evaluation
                            snapshot; artefact snapshot in extra workgroups
    side stream: best models -> mapped host snapshot slot, evaluation (fwd + CEN + AUC)
                 [one all-reduce: AUCs + rejected counts] -> mapped per-round
                 report slot; record the round event
                 (overlaps the next round's training; the next round's
                 verification waits for it before reusing the buffers)

and the host moves on to the next round.  Results are *collected* later
(at most ``max_pending`` rounds behind, or when a caller reads a round's
fields): the mapped slots are read after the round's event, logs are
emitted, and reports / checkpoints are handed to the background writer.
A round therefore costs its GPU time only; the host work of round r+1
overlaps the GPU work of round r.

Decisions, aggregates and metrics are identical to the host path in fixed
mode (tested on the GPU, and over 60 bench-shaped rounds:
scripts/device_vs_host_long.py); the host-side RNG draws one k x (k-1) noise
table per round in both paths (and, in the thesis variant, one fallback
uniform).  Resume snapshots (``snapshot`` / ``restore``), latent logging,
fault injection and the non-AUC metrics run on this path too.
"""
from __future__ import annotations

import logging
import os
import weakref
from collections import deque
from typing import Dict, List, Optional

import numpy as np
import torch

from ..models.layout import P_PAD
from ..ops import _hip

# fence-less device events for the kernel-to-kernel stream dependencies
# ("0": torch events, which record with a system-scope fence)
_DEVICE_EVENTS = os.environ.get("FEDMX_DEVICE_EVENTS", "1") != "0"
_SIDE_FLAG_KEEPALIVE: list = []   # (hand-off word, status buffer) of every DeviceRound (a few bytes each)

log = logging.getLogger("fedmx")


# A/B timing only: pack the multi-rank send buffer with its own copy_rows
# launch instead of inside the score-reduction launch
_PACK_SEPARATE = os.environ.get("FEDMX_PACK_SEPARATE", "0") == "1"


def _thesis_fused_ok(fed) -> bool:
    """The thesis rule runs in the fused verification kernel only (it forwards
    each receiver's rows through the aggregate and its own model in LDS)."""
    if fed.cfg.verification_method == "dev":
        rows = int(fed.dev_set.shape[0])
    else:
        rows = max((int(fed.valid_all[c].shape[0]) for c in fed.local), default=0)
    return rows <= _hip.VERIFY_MAX_ROWS


def fast_path_supported(fed) -> Optional[str]:
    """None when the device round can run this federation, else the reason it cannot."""
    cfg = fed.cfg
    if fed.engine.name != "hip":
        return "engine is not the HIP engine"
    checks = [
        (cfg.compat == "fixed", "compat mode is not 'fixed'"),
        (cfg.election in ("first_voter", "majority"), f"election {cfg.election}"),
        (cfg.aggregation_mode in ("decentralized", "centralized"), f"aggregation mode {cfg.aggregation_mode}"),
        (cfg.protocol_variant == "code" or _thesis_fused_ok(fed),
         "thesis variant with verification rows beyond the fused kernel's LDS buffer"),
        (fed.update_type in ("avg", "fedprox", "mse_avg", "fusion_avg"), f"update type {fed.update_type}"),
        (cfg.metric in ("AUC", "classification", "time"), f"metric {cfg.metric}"),
        # dropped clients leave at least one selection per round (k >= 1: the
        # election kernel needs a voter); larger drop sets take the host path
        (len({c for c in cfg.dropped_clients if 0 <= c < fed.N}) < max(1, int(cfg.num_participants * fed.N)),
         "fault injection could drop every selected client"),
        (cfg.device_protocol, "device protocol disabled"),
    ]
    for ok, why in checks:
        if not ok:
            return why
    return None


class LazyRoundResult:
    """A round whose device results are read on first access."""

    def __init__(self, dr: "DeviceRound", rec: dict):
        self._dr = dr
        self._rec = rec
        self.round = rec["round"]
        self.selected = rec["selected"]
        self.times_ms = rec.get("times_ms", {})

    def _get(self, k):
        if not self._rec["done"]:
            self._dr.collect_until(self._rec["round"])
        return self._rec[k]

    aggregator = property(lambda self: self._get("aggregator"))
    metrics = property(lambda self: self._get("metrics"))
    verification = property(lambda self: self._get("verification"))
    epochs_run = property(lambda self: self._get("epochs_run"))
    stop = property(lambda self: self._get("stop"))


class DeviceRound:
    def __init__(self, fed, max_pending: int = 2):
        self.fed = fed
        eng = fed.engine
        st = eng.store
        dev = eng.device
        self.dev = dev
        N = fed.N
        self.N = N
        self.start = fed.local[0] if fed.local else 0
        self.n_local = len(fed.local)
        self.max_pending = max_pending
        f64, i32, f32 = torch.float64, torch.int32, torch.float32
        # vote records [N,4]: every entry the election reads is rewritten each round
        self.vec = torch.zeros(N, 4, dtype=f64, device=dev)
        # evaluation runs on a side stream and overlaps the next round's
        # training: it reads a snapshot of the parameters taken right after
        # the adoption step, into its own metrics buffer
        self.side = torch.cuda.Stream(device=dev)
        # [AUCs | rejected counts]; only hosted receivers' counts are ever
        # written, so other ranks' entries stay zero for the report all-reduce
        # The buffers the verification writes and the side stream reads
        # (evaluation params, best-model stage, [AUCs | rejected]) rotate over
        # NSIDE slots: round r reuses round r-NSIDE's, whose side work the host
        # has normally collected already, so the main stream only waits (a
        # cross-stream barrier packet, ~6 us on the chain) when it is not done.
        NSIDE = 3
        self.side_slots = [dict(rep=torch.zeros(2 * N, dtype=f64, device=dev),
                                params=torch.empty_like(st.params), best=torch.empty_like(st.best), ev=None)
                           for _ in range(NSIDE)]
        # standardised vote data (src/Trainer/client_trainer.py:220-223: the
        # voter's validation set, re-standardised with its own ddof=1 column
        # stats at every vote).  Each client's validation set is fixed for the
        # whole run, so its standardised copy is computed once here for every
        # client that can vote: the round then reads it with no standardisation
        # launch and no cross-stream wait (that wait, a barrier packet on the
        # main stream even when the side stream is long done, cost ~6 us per
        # round between training and the vote forward).  Federations whose
        # copies would not fit FEDMX_VOTE_CACHE_MB fall back to standardising
        # per round on the side stream (by round parity: round r+2's
        # standardisation is queued behind the side stream's wait for round
        # r+1's decisions, recorded after round r's vote forward read it).
        self.vs_bufs = [None, None]
        self.vs_cache = None
        cache_mb = float(os.environ.get("FEDMX_VOTE_CACHE_MB", "2048"))
        rows = sum(int(v.shape[0]) for v in fed.valid_all)
        if fed.local and rows * int(fed.valid_all[0].shape[1]) * 4 <= cache_mb * (1 << 20):
            self.vs_cache = [_hip.standardize_ddof1(v.contiguous(), fed.dims.d_in) for v in fed.valid_all]
        # best-model snapshots for the artefact writer: a ring of mapped host
        # slots filled by a device copy kernel (no torch pinned allocation or
        # blocking copy on the enqueue path); a slot is reused once the writer
        # has finished the checkpoint jobs that read it
        self.n_snap = 4
        numel = st.best.numel()
        self.snap_buf = _hip._hiprt.MappedBuffer(self.n_snap * numel * 4)
        C = st.best.shape[0]
        self.snap_views = [torch.from_numpy(self.snap_buf.view(i * numel * 4, np.float32, numel).reshape(C, P_PAD))
                           for i in range(self.n_snap)]
        # native checkpoint writer ticket of the job reading each slot (0: free)
        self.snap_ticket = [0] * self.n_snap
        self.ckpt = fed.writer.native_ckpt(fed.dims) if fed.cfg.save_checkpoints and fed.local else None
        if self.ckpt is not None:
            # queued writes read snap_buf: drain them before it can be freed
            weakref.finalize(self, self.ckpt.wait, 0)
        self.snap_i = 0
        self.agg_counts = torch.zeros(N, dtype=i32, device=dev)
        self.weights = torch.zeros(max(N, 1), dtype=f32, device=dev)
        self.state = torch.full((4,), -1, dtype=i32, device=dev)
        self.agg = torch.zeros(P_PAD, dtype=f32, device=dev)
        n = max(self.n_local, 1)
        self.hist = torch.zeros(n, P_PAD, dtype=f32, device=dev)
        self.has_hist = torch.zeros(n, dtype=i32, device=dev)
        self.hist_perf = torch.zeros(n, dtype=f64, device=dev)
        self.rejected = torch.zeros(n, dtype=i32, device=dev)
        self.rt = _hip.runtime(dev)
        cfg = fed.cfg
        if fed.comm.collective:
            # persistent exchange buffers: [1 row of vote records | up to xslots models] per rank
            self.xslots = fed.shard.max_local()
            self.xsend = torch.zeros(self.xslots + 1, P_PAD, dtype=f32, device=dev)
            self.xallg = torch.zeros(fed.comm.world_size * (self.xslots + 1), P_PAD, dtype=f32, device=dev)
            if hasattr(fed.comm, "setup_exchange"):
                # peer-memory channels (parallel/ipc.py): the gather of the
                # exchange rows and the [AUCs | rejected] reduce; collective
                fed.comm.setup_exchange((self.xslots + 1) * P_PAD, 4 * N)
        # verification: the aggregate on every hosted client's verification data (fixed mode: own V)
        if cfg.verification_method == "dev":
            vdata = [fed.dev_set for _ in fed.local]
        else:
            vdata = [fed.valid_all[c] for c in fed.local]
        self.vplan = _hip.FwdPlan(self.agg.unsqueeze(0), [(0, d) for d in vdata], fed.dims,
                                  want_sse=True, want_latent=False) if fed.local else None
        if fed.local:
            self.vsse_off = torch.from_numpy(self.vplan.offs.astype(np.int32)).to(dev)
            self.vsse_n = torch.from_numpy(self.vplan.sizes.astype(np.int32)).to(dev)
            # fused verification (one launch: forward + decide/adopt + snapshots)
            # when every receiver's verification rows fit the kernel's LDS buffer
            self._vdata = vdata
            self.vx = torch.tensor([d.data_ptr() for d in vdata], dtype=torch.int64, device=dev)
        self.fused_verify = bool(fed.local) and max(int(d.shape[0]) for d in vdata) <= _hip.VERIFY_MAX_ROWS
        # split verification (fedmx_protocol.hip verify_split_kernel): each
        # receiver's forward over ceil(tiles / 8) workgroups -- at most one
        # 16-row tile per wave -- plus a drift workgroup; the thesis rule keeps
        # the fused kernel (it forwards two models)
        self.vsplit = None
        if self.fused_verify and _hip.VERIFY_SPLIT and cfg.protocol_variant != "thesis":
            tiles = max((int(d.shape[0]) + 15) // 16 for d in vdata)
            self.vsplit_scratch = (torch.empty(self.n_local, _hip.VERIFY_MAX_ROWS, dtype=f32, device=dev),
                                   torch.zeros(self.n_local, dtype=torch.int64, device=dev),
                                   torch.zeros(self.n_local, dtype=i32, device=dev))
            sse, drift, count = self.vsplit_scratch
            self.vsplit = _hip.VerifySplitArgs(sse=sse.data_ptr(), drift=drift.data_ptr(), count=count.data_ptr(),
                                               splits=max(1, min(64, -(-tiles // 8))), pad=0)
        # side-stream hand-off (fedmx_protocol.hip vs_depart / side_wait_kernel):
        # with split verification the round's evaluation waits on the
        # verification kernel's own hand-off word, so the main stream carries
        # no event between the verification and the next training launch
        self.side_flag = None
        if self.vsplit is not None and _hip.SIDE_FLAG:
            khz = _hip.lib().fedmx_ipc_wall_khz()
            status = _hip._hiprt.MappedBuffer(64)
            view = status.view(0, np.int32, 1)
            view[0] = 0
            timeout_s = float(os.environ.get("FEDMX_SIDE_WAIT_TIMEOUT_S", "120"))
            self.side_flag = dict(done=torch.zeros(2, dtype=i32, device=dev), status=status, view=view, seq=0,
                                  ticks=int(timeout_s * 1e3 * (khz if khz > 0 else 100_000)))
            self.vsplit.done = self.side_flag["done"].data_ptr()
            # both streams use these through raw pointers (the verification
            # kernel on the main stream writes the word, the side stream's
            # wait reads it and may write the status): never released, so no
            # later allocation can reuse them under a wait still in flight
            _SIDE_FLAG_KEEPALIVE.append((self.side_flag["done"], status))
        # the two per-round stream dependencies whose consumers are kernels only
        # (side -> main: the standardised vote data; main -> side: the round's
        # decisions and snapshots for the evaluation): fence-less device events
        # (_hiprt.DeviceEvent), torch events with FEDMX_DEVICE_EVENTS=0
        self.dev_ev = (_hip._hiprt.DeviceEvent(), _hip._hiprt.DeviceEvent()) if _DEVICE_EVENTS else None
        # aggregation weights: 1 = FedMSE 1/MSE (device), 0 = plain mean,
        # 2 = sample-weighted FedAvg (host-computed: they depend on the selection only)
        # fusion_avg: weights formed on the device each round (rule 2 reads them
        # from self.fw; Federation._fusion_weights_t, the host path's computation)
        self.fusion = fed.update_type == "fusion_avg"
        self.rule = 1 if fed.update_type == "mse_avg" else (2 if cfg.fedavg_sample_weighted or self.fusion else 0)
        if self.fusion:
            self.fstack = torch.zeros(max(N, 1), P_PAD, dtype=f32, device=dev)
            self.fw = torch.zeros(max(N, 1), dtype=f32, device=dev)
        self.n_train = {c: fed.clients[c].train.shape[0] for c in range(N)}
        # protocol variants the kernels implement: majority election (every
        # selected client votes) and the centralised push (no verification)
        self.thesis = cfg.protocol_variant == "thesis"
        self.elect_mode = (1 if cfg.election == "majority" else 0) | (6 if self.thesis else 0)
        self.centralized = cfg.aggregation_mode == "centralized"
        self.drift_rel = cfg.drift_threshold_rel > 0   # kernel mode 3: drift <= rel x ||history||
        # training-failure word (TrainArgs.err): a launch whose bounded flag
        # wait ran out sets it; the election kernel reads it and skips the
        # round's aggregation and adoption (report ELECT_TRAIN_FAILED).  With
        # collectives it is the last word of this rank's exchange records row,
        # so it rides the all-gather and every rank sees every rank's failure.
        self.err = torch.zeros(1, dtype=i32, device=dev)
        self.err_ptr = self.err.data_ptr()
        self.err_n, self.err_stride = 1, 0
        if fed.comm.collective:
            if 8 * self.xslots <= P_PAD - 4:   # the records (4 doubles per slot) end before it
                self.err_ptr = self.xsend.data_ptr() + 4 * (P_PAD - 1)
                self.xsend[0, P_PAD - 1] = 0.0   # int32 0
            else:
                self.err_n = 0   # (more than 1,150 clients on one rank: the host-side check only)
        self.pending: deque = deque()
        # optional: HIP-event time of every round's training launch (bench.py
        # at N > 1 measures the wait for the slowest rank's largest client)
        self.train_timing = False
        # global early stop reads each round's metrics: collect right after
        # enqueueing (False: the caller reads them later, e.g. after issuing
        # other federations' rounds -- main.py --concurrent-combos)
        self.eager_collect = True
        self.train_ms: Dict[int, float] = {}
        self.all_rounds: Dict[int, dict] = {}
        self.host_agg_counts = [0] * N

    # ------------------------------------------------------------------------------
    def _host_metrics(self, rec: dict) -> np.ndarray:
        """The evaluator's non-AUC metrics (`src/Evaluator/evaluator.py:64-108`,
        eval.evaluator.evaluate_clients) from this round's device evaluation:
        ``classification`` = F1 at score threshold 0.5 of the round's anomaly
        scores (the AUC plan's scores: CEN distances, or per-row MSE for the
        AE); ``time`` = seconds of the evaluation launches (side-stream events).
        Every rank fills its hosted clients; one host all-reduce."""
        fed, eng, N = self.fed, self.fed.engine, self.N
        vec = np.zeros(N, dtype=np.float64)
        if fed.local:
            if fed.cfg.metric == "time":
                e0, e1 = rec["eval_timing"]
                vec[self.start:self.start + self.n_local] = e0.elapsed_time(e1) / 1e3
            else:
                from ..eval.metrics import classification_metrics

                p = eng._plan(fed.model_type, rec["eval_params"])
                D = fed.dims.d_in
                st = eng.store
                for i, sc in enumerate(p["scores"]):
                    s = sc / D if fed.model_type == "autoencoder" else sc
                    vec[self.start + i] = classification_metrics(st.labels(i), s.detach().cpu().numpy())[0]
        return np.asarray(fed.comm.all_reduce_sum(vec), dtype=np.float64)

    def _auc_fallback(self, rec: dict, metrics: np.ndarray) -> np.ndarray:
        from ..ops import _host

        fed = self.fed
        bad = np.flatnonzero(metrics == -1.0)
        vec = np.zeros(self.N, dtype=np.float64)
        if fed.local:
            p = fed.engine._plan(fed.model_type, rec["eval_params"])
            for c in bad:
                i = int(c) - self.start
                if 0 <= i < self.n_local:
                    s = p["scores"][i].detach().double().cpu().numpy()
                    vec[c] = _host.roc_auc(np.nan_to_num(s), p["labels"][i].cpu().numpy())
        if fed.comm.collective:
            vec = np.asarray(fed.comm.all_reduce_sum(vec), dtype=np.float64)
        out = metrics.copy()
        out[bad] = vec[bad]
        return out

    def snapshot(self) -> dict:
        """The device-resident protocol state a resumed federation needs
        (aggregation caps, every hosted receiver's verifier history and
        rejection count); every enqueued round is collected first.  Per-round
        scratch (vote records, election state, side-stream slots) is rewritten
        by the next round and is not part of it."""
        self.collect_all()
        torch.cuda.synchronize(self.dev)
        return {"agg_counts": self.agg_counts.cpu(), "hist": self.hist.cpu(), "has_hist": self.has_hist.cpu(),
                "hist_perf": self.hist_perf.cpu(), "rejected": self.rejected.cpu(),
                "host_agg_counts": torch.tensor(self.host_agg_counts, dtype=torch.int64)}

    def restore(self, s: dict) -> None:
        for k in ("agg_counts", "hist", "has_hist", "hist_perf", "rejected"):
            t = getattr(self, k)
            if tuple(s[k].shape) != tuple(t.shape):
                raise ValueError(f"resume snapshot: device state {k} has shape {tuple(s[k].shape)}, "
                                 f"this federation needs {tuple(t.shape)}")
            t.copy_(s[k].to(t.device))
        self.host_agg_counts = [int(x) for x in s["host_agg_counts"].tolist()]

    def seed_from_host(self) -> None:
        """Device protocol state from the federation's host-side state (a
        resume snapshot written by the host-decision path has no device
        entry): aggregation caps, and for every hosted receiver its verifier
        history (the last received aggregate, its performance) and rejection
        count — what the host path's Verifier would use next."""
        fed = self.fed
        self.host_agg_counts = [int(x) for x in fed.agg_counts]
        self.agg_counts.copy_(torch.tensor(self.host_agg_counts, dtype=torch.int32))
        for i, c in enumerate(fed.local):
            vs = fed.vstate.get(c)
            if vs is None:
                continue
            self.rejected[i] = int(vs.rejected_updates)
            if vs.history_version is not None and vs.history_version in fed.versions:
                self.hist[i].copy_(fed.versions[vs.history_version])
                self.has_hist[i] = 1
                self.hist_perf[i] = float(vs.history_perf)
            else:
                self.has_hist[i] = 0

    def reset_aggregation_counts(self):
        self.agg_counts.zero_()
        self.host_agg_counts = [0] * self.N

    def _loc(self, c):
        return c - self.start

    def _check_failed(self, rec: dict) -> None:
        if self.side_flag is not None and int(self.side_flag["view"][0]) != 0:
            raise RuntimeError(f"round {rec['round'] + 1}: the evaluation's wait for the verification kernel's "
                               "hand-off ran out (FEDMX_SIDE_WAIT_TIMEOUT_S); rerun with FEDMX_SIDE_FLAG=0")
        if int(rec["report"][0]) == _hip.ELECT_TRAIN_FAILED:
            raise RuntimeError(f"round {rec['round'] + 1}: a training launch failed (a wave's bounded flag wait "
                               "or validator decision wait ran out); the device skipped that round's aggregation "
                               "and adoption")

    def enqueue(self, selected: List[int]) -> LazyRoundResult:
        fed = self.fed
        cfg, eng, st, comm = fed.cfg, fed.engine, fed.engine.store, fed.comm
        # a pending round whose election already reported a failed training
        # launch (mapped report slot, no synchronisation): stop before enqueueing more
        for r in self.pending:
            if "report" in r:
                self._check_failed(r)
        tel = fed.tel
        N, dev = self.N, self.dev
        rnd = fed.round_idx
        k = len(selected)
        local_sel = [c for c in selected if fed._mine(c)]
        local_rows = [self._loc(c) for c in local_sel]
        rec = dict(round=rnd, selected=list(selected), local_sel=local_sel, done=False)

        ev_std = None
        if local_sel and self.vs_cache is not None:
            vs = self.vs_cache[selected[0]]
        elif local_sel:
            # the vote data does not depend on training: standardise it on the
            # side stream (double-buffered by round parity) while training runs
            vdata = fed.valid_all[selected[0]]
            pb = rnd & 1
            if self.vs_bufs[pb] is None or self.vs_bufs[pb].shape[0] < vdata.shape[0]:
                self.vs_bufs[pb] = torch.empty(max(vdata.shape[0], 256), vdata.shape[1], dtype=torch.float32,
                                               device=dev)
            vs = self.vs_bufs[pb][:vdata.shape[0]]
            with _hip.on_stream(self.side):
                _hip.standardize_ddof1(vdata.contiguous(), fed.dims.d_in, out=vs)
                if self.dev_ev is not None:
                    ev_std = self.dev_ev[0]
                    ev_std.record(self.side.cuda_stream)
                else:
                    ev_std = torch.cuda.Event()
                    ev_std.record(self.side)
        with tel.phase("train"):
            tev = None
            if self.train_timing and local_sel:
                tev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                tev[0].record()
            eng.train_err_ptr = self.err_ptr
            handle = eng.train_launch(local_rows, fed.hp) if local_sel else None
            if tev is not None:
                tev[1].record()
                rec["train_ev"] = tev
            rec["handle"] = handle
            for c in local_sel:
                if c in cfg.malicious_clients:   # fault injection: poisoned update (stream-ordered)
                    st.params[self._loc(c)].mul_(cfg.malicious_scale)
        with tel.phase("vote"):
            if local_sel:
                if ev_std is not None:
                    if self.dev_ev is not None:
                        ev_std.wait(torch.cuda.current_stream(dev).cuda_stream)
                    else:
                        torch.cuda.current_stream(dev).wait_event(ev_std)
                need_dev = self.rule == 1
                items = [(r, vs) for r in local_rows]
                # each client's record [vote score, -, dev MSE, dev MSE] (4 doubles):
                # with collectives straight into the exchange buffer's tail row
                # (slot j = j-th local selection, the pack order), else into vec
                if comm.collective:
                    head = self.xsend[0].data_ptr()
                    recp = [head + 32 * j for j in range(len(local_sel))]
                else:
                    recp = [self.vec[c].data_ptr() for c in local_sel]
                outs = list(recp)
                batch = [cfg.vote_batch_size] * len(local_rows)
                if need_dev:
                    items += [(r, fed.dev_set) for r in local_rows]
                    outs += [p + 16 for p in recp]
                    batch += [0] * len(local_rows)
                sse, _ = _hip.forward_rows(st.params, items, fed.dims, True, False)
                # multi-rank: the exchange's pack (row 1 + j of the send buffer =
                # the j-th local selection's parameters) rides the same launch
                copies = [(st.params[self._loc(c)].data_ptr(), self.xsend[1 + j].data_ptr(), P_PAD)
                          for j, c in enumerate(local_sel)] if comm.collective and not _PACK_SEPARATE else ()
                _hip.score_reduce_to(sse, batch, fed.dims.d_in, outs, copies)
        with tel.phase("comm"):
            if not comm.collective:
                base = st.params
                rows = np.asarray([self._loc(c) for c in selected], dtype=np.int64)
            else:
                # ONE collective for models and scores: every rank sends its
                # selected clients' parameter rows plus one extra row carrying
                # their (vote score, dev MSE) records; the all-gather gives
                # every rank the whole selection in a world-size independent
                # order (row strides stay multiples of P for the weighted sum)
                per_rank: Dict[int, List[int]] = {}
                for c in selected:
                    per_rank.setdefault(fed.shard.owner(c), []).append(c)
                # Packing / unpacking index arrays go through the mapped
                # descriptor ring into row-copy kernels: no host -> device
                # copies, which (from pageable memory) would synchronise the
                # host with the training kernel every round.  Rows past a
                # rank's selection are never read, so `send` needs no fill.
                # The exchange buffers are persistent (sized for the largest
                # shard): no allocation or allocator event per round; each
                # round exchanges only the prefix [records row | slots model
                # rows] that its largest per-rank selection needs.
                slots = max(len(v) for v in per_rank.values())
                mine = per_rank.get(comm.rank, [])
                send = self.xsend[:slots + 1]
                allg = self.xallg[:comm.world_size * (slots + 1)]
                if mine:
                    # (the vote records are already in row 0 and the models in
                    # rows 1.. : the score-reduction launch wrote / copied them)
                    if _PACK_SEPARATE:   # A/B: the pack as a launch of its own
                        (loc_ptr,) = self.rt.desc.put(np.asarray([self._loc(c) for c in mine], dtype=np.int32))
                        _hip.copy_rows(send[1].data_ptr(), P_PAD, 0, st.params.data_ptr(), P_PAD, loc_ptr,
                                       len(mine), P_PAD, dev)
                    if comm.phantom and len(mine) < slots:
                        # single-GPU projection (PhantomComm): other ranks' rows are
                        # copies of this rank's, so the spare slots must hold real models
                        n = len(mine)
                        send[1 + n:1 + slots].copy_(send[1:2].expand(slots - n, P_PAD))
                        send[0, 8 * n:8 * slots].copy_(send[0, :8].repeat(slots - n))
                comm.all_gather_into(allg, send)          # [world * (slots+1), P]
                owners = [fed.shard.owner(c) for c in selected]
                # record of client c: row 0 of its owner's block, entry j (4-double
                # units); the election reads the records in place through this table
                rec_idx = np.asarray([(o * (slots + 1) * P_PAD) // 8 + per_rank[o].index(c)
                                      for o, c in zip(owners, selected)], dtype=np.int32)
                base = allg
                rows = np.asarray([o * (slots + 1) + 1 + per_rank[o].index(c) for o, c in zip(owners, selected)],
                                  dtype=np.int64)
        with tel.phase("aggregate"):
            noise = np.asarray(fed.noise.rand_n(k * (k - 1)), dtype=np.float64)
            if comm.collective:
                # every rank's failure word, read in place from the gathered records rows
                err_ptr, err_n, err_stride = base.data_ptr() + 4 * (P_PAD - 1), self.err_n * comm.world_size, \
                    (slots + 1) * P_PAD
            else:
                err_ptr, err_n, err_stride = self.err_ptr, self.err_n, 0
            if comm.collective:
                sel_ptr, noise_ptr, rows_ptr, rec_ptr = self.rt.desc.put(
                    np.asarray(selected, dtype=np.int32), noise if noise.size else np.zeros(1), rows, rec_idx)
                vec_ptr = base.data_ptr()
            else:
                sel_ptr, noise_ptr, rows_ptr = self.rt.desc.put(np.asarray(selected, dtype=np.int32),
                                                                noise if noise.size else np.zeros(1), rows)
                rec_ptr, vec_ptr = 0, self.vec.data_ptr()
            hw_ptr = 0
            if self.fusion:
                # the selected models in selection order (device row gather from
                # the model source the aggregation reads), then their weights
                (sidx,) = self.rt.desc.put(np.asarray(rows, dtype=np.int32))
                _hip.copy_rows(self.fstack.data_ptr(), P_PAD, 0, base.data_ptr(), P_PAD, sidx, k, P_PAD, dev)
                self.fw[:k].copy_(fed._fusion_weights_t(self.fstack[:k]))
                hw_ptr = self.fw.data_ptr()
            elif self.rule == 2:
                from ..protocol.aggregation import plan_mean

                (hw_ptr,) = self.rt.desc.put(np.asarray([w for _, w in plan_mean(selected, self.n_train)],
                                                        dtype=np.float32))
            rep_ptr, rep_view = self.rt.out.take(np.int32, 2)
            rep_view[:] = -2
            a = _hip.ElectArgs(sel=sel_ptr, vec=vec_ptr, noise=noise_ptr,
                               agg_counts=self.agg_counts.data_ptr(), weights=self.weights.data_ptr(),
                               state=self.state.data_ptr(), report=rep_ptr, k=k, cap=cfg.max_aggregation,
                               rule=self.rule, mode=self.elect_mode, rec=rec_ptr, hw=hw_ptr,
                               vote_cap=float(cfg.thesis_vote_mse_cap),
                               # thesis fallback: one uniform per round, drawn whatever the outcome
                               fallback_u=fed.fallback_rng.random() if self.thesis else 0.0,
                               err=err_ptr, err_n=err_n, err_stride=err_stride)
            w = _hip.WsumArgs(base=base.data_ptr(), rows=rows_ptr, weights=self.weights.data_ptr(),
                              state=self.state.data_ptr(), out=self.agg.data_ptr(), k=k, P=P_PAD)
            _hip.elect_wsum(a, w, dev)
            rec["report"] = rep_view
        # the previous round's side work has read the snapshot / report buffers
        side = self.side_slots[rnd % len(self.side_slots)]
        if side["ev"] is not None and not side["ev"].query():
            torch.cuda.current_stream(dev).wait_event(side["ev"])
        side_rep, eval_params, best_stage = side["rep"], side["params"], side["best"]
        with tel.phase("verify"):
            # every hosted receiver: the aggregate's SSE rows on its data, then
            # one kernel reduces MSE + drift, decides, adopts and bumps the cap
            # count; rejected counts go straight into the side stream's report
            # buffer ([AUCs | rejected])
            if self.n_local and not self.fused_verify:
                self.vplan.run()
            d = _hip.DecideArgs(params=st.params.data_ptr(), anchor=st.anchor.data_ptr(),
                                hist=self.hist.data_ptr(), agg=self.agg.data_ptr(), state=self.state.data_ptr(),
                                sse=self.vplan.sse.data_ptr() if self.n_local else 0,
                                sse_off=self.vsse_off.data_ptr() if self.n_local else 0,
                                sse_n=self.vsse_n.data_ptr() if self.n_local else 0,
                                seg=eng._seg.data_ptr(), agg_counts=self.agg_counts.data_ptr(),
                                has_hist=self.has_hist.data_ptr(), hist_perf=self.hist_perf.data_ptr(),
                                rejected=self.rejected.data_ptr(), rej_out=side_rep.data_ptr() + 8 * N,
                                thr=float(cfg.thesis_loss_ratio if self.thesis else
                                          (cfg.drift_threshold_rel if self.drift_rel else cfg.verification_threshold)),
                                pthr=float(cfg.performance_threshold),
                                start=self.start, n_local=self.n_local, P=P_PAD, d_in=fed.dims.d_in,
                                mode=1 if self.centralized else (2 if self.thesis else (3 if self.drift_rel else 0)),
                                pad=0)
            if self.fused_verify:
                # verification forward, decisions, adoption and the evaluation /
                # artefact snapshots in one launch (bit-identical to the
                # separate kernels below)
                v = _hip.VerifyArgs(D=d, vx=self.vx.data_ptr(), vn=self.vsse_n.data_ptr(),
                                    eval_params=eval_params.data_ptr(), best_stage=best_stage.data_ptr(),
                                    best=st.best.data_ptr(), latent=fed.dims.latent, hidden=fed.dims.hidden)
                if self.vsplit is not None:
                    if self.side_flag is not None:
                        self.side_flag["seq"] += 1
                        self.vsplit.seq = self.side_flag["seq"] & 0xFFFFFFFF
                    _hip.verify_split(v, self.vsplit, dev)
                else:
                    _hip.verify_decide(v, dev)
            else:
                _hip.decide_adopt(d, dev)
        slot_ptr, slot = self.rt.out.take(np.float64, 2 * N)
        if not self.fused_verify:
            # snapshot params (for the evaluation) and the best models (for the
            # artefacts) on the main stream: one fused device copy, so the next
            # round's training can start right away
            nd = st.params.numel() // 2
            _hip.copy2_f64(eval_params.data_ptr(), st.params.data_ptr(), nd,
                           best_stage.data_ptr(), st.best.data_ptr(), nd, dev)
        side_flag = self.side_flag if (self.fused_verify and self.vsplit is not None) else None
        if side_flag is not None:
            ev_dec = None   # the verification kernel's hand-off word instead
        elif self.dev_ev is not None:
            ev_dec = self.dev_ev[1]
            ev_dec.record(torch.cuda.current_stream(dev).cuda_stream)
        else:
            ev_dec = torch.cuda.Event()
            ev_dec.record()
        with tel.phase("eval"), _hip.on_stream(self.side):
            if side_flag is not None:
                _hip.side_wait(side_flag["done"].data_ptr() + 4, side_flag["seq"], side_flag["status"].dev_ptr,
                               side_flag["ticks"], self.side.cuda_stream)
            elif self.dev_ev is not None:
                ev_dec.wait(self.side.cuda_stream)
            else:
                self.side.wait_event(ev_dec)
            if local_sel and cfg.save_checkpoints:
                si = self.snap_i
                self.snap_i = (si + 1) % self.n_snap
                with tel.phase("wait_writer"):   # artefact writer backlog (host-bound indicator)
                    if self.snap_ticket[si]:
                        self.ckpt.wait(self.snap_ticket[si])
                        self.snap_ticket[si] = 0
                nd = st.best.numel() // 2
                _hip.copy2_f64(self.snap_buf.dev_ptr + si * st.best.numel() * 4, best_stage.data_ptr(), nd,
                               0, 0, 0, dev)
                rec["snap_slot"] = si
            if cfg.metric == "time":
                t_ev0 = torch.cuda.Event(enable_timing=True)
                t_ev0.record(self.side)
            eng.evaluate_launch(fed.model_type, params=eval_params)
            if cfg.metric == "time":
                t_ev1 = torch.cuda.Event(enable_timing=True)
                t_ev1.record(self.side)
                rec["eval_timing"] = (t_ev0, t_ev1)
            rec["eval_params"] = eval_params   # --save-latents: the plan whose latent buffers hold this round's
            aucs_ptr = eng._plan(fed.model_type, eval_params)["aucs_buf"].dev_ptr
            if not comm.collective:
                _hip.copy2_f64(slot_ptr, aucs_ptr, N, slot_ptr + 8 * N, side_rep.data_ptr() + 8 * N, N, dev)
            else:
                # [AUCs | rejected counts]: one RCCL all-reduce, off the main stream.
                # Every entry this rank does not write must be zero going in: the
                # slot is cleared right after its sum is copied out (so when the
                # slot comes round again, only this round's verification has
                # written it — the hosted receivers' counts)
                if self.n_local:
                    _hip.copy_f64(side_rep.data_ptr() + 8 * self.start, aucs_ptr, self.n_local, dev)
                comm.all_reduce_inplace(side_rep)
                _hip.copy_f64(slot_ptr, side_rep.data_ptr(), 2 * N, dev)
                side_rep.zero_()
            ev = torch.cuda.Event()
            ev.record(self.side)
            side["ev"] = ev
        rec["slot"] = slot
        rec["event"] = ev
        fed.round_idx += 1
        rec["times_ms"] = tel.end_round(round=rnd + 1, selected=k, aggregator=None)
        self.pending.append(rec)
        self.all_rounds[rnd] = rec
        res = LazyRoundResult(self, rec)
        # bounded run-ahead: collect rounds that are max_pending behind (normally already finished)
        while len(self.pending) > self.max_pending:
            with tel.phase("collect"):    # mostly waiting for round r-2 on the GPU
                self._collect(self.pending.popleft())
        if cfg.global_early_stop and self.eager_collect:
            self.collect_until(rnd)
        return res

    # ------------------------------------------------------------------------------
    def collect_until(self, rnd: int):
        while self.pending and self.pending[0]["round"] <= rnd:
            self._collect(self.pending.popleft())

    def collect_all(self):
        while self.pending:
            self._collect(self.pending.popleft())

    def _collect(self, rec: dict):
        fed = self.fed
        cfg, eng = fed.cfg, fed.engine
        rec["event"].synchronize()
        if hasattr(fed.comm, "check"):
            fed.comm.check()   # peer-memory exchange: no wait of this round timed out
        N = self.N
        rnd = rec["round"]
        info = log.isEnabledFor(logging.INFO)
        self._check_failed(rec)
        agg = int(rec["report"][0])
        aggregator = agg if agg >= 0 else None
        slot = rec["slot"]
        metrics = np.array(slot[:N], dtype=np.float64)
        rej = np.array(slot[N:2 * N], dtype=np.float64)
        if cfg.metric != "AUC":
            metrics = self._host_metrics(rec)
        elif bool(np.any(metrics == -1.0)):
            # a class too large for the kernel's LDS sort: exact host AUC of
            # those clients from the round's device scores (the same fallback
            # as HipEngine._auc_fixup); every rank sees the same set
            metrics = self._auc_fallback(rec, metrics)
        handle = rec.get("handle")
        if rec.get("train_ev") is not None:
            self.train_ms[rnd] = rec["train_ev"][0].elapsed_time(rec["train_ev"][1])
        epochs_local: Dict[int, int] = {}
        if handle is not None:
            res = eng.train_collect(handle, [np.array(t) for t in handle.tensors])
            for i, c in enumerate(rec["local_sel"]):
                epochs_local[c] = int(res.epochs_run[i])
                if info:
                    for e, (tl, vl) in enumerate(res.tracking[i]):
                        log.info(f"[Client {c}] Epoch {e + 1} - Training loss: {tl} - Validating loss: {vl}")
            if cfg.save_checkpoints:
                si = rec["snap_slot"]
                # the side stream's event (synchronised above) covers the slot's
                # snapshot copy: the native writer may read it right away
                sel = rec["local_sel"]
                self.snap_ticket[si] = self.ckpt.submit(
                    [fed.save_dirs[c] for c in sel], self.snap_views[si].numpy(), [self._loc(c) for c in sel],
                    [bool(res.best_epoch[i] >= 0) for i in range(len(sel))],
                    [list(res.tracking[i]) for i in range(len(sel))])
        verification = []
        if aggregator is not None and self.centralized:
            # centralised push: every client adopted the aggregate, nothing to report
            self.host_agg_counts[aggregator] += 1
            fed.agg_counts[aggregator] += 1
            if info:
                log.info(f"Client {aggregator + 1} selected as aggregator")
        elif aggregator is not None:
            self.host_agg_counts[aggregator] += 1
            fed.agg_counts[aggregator] += 1
            if info:
                log.info(f"Client {aggregator + 1} selected as aggregator")
            for c in range(N):
                if c != aggregator:
                    r = int(rej[c])
                    verification.append({"client_id": c, "rejected_updates": r, "is_verified": r == 0})
            if fed.write_reports:
                vr = verification
                fed.writer.submit(lambda vr=vr, rnd=rnd: fed._report_verification(rnd, vr))
        else:
            log.warning("No aggregator selected for this round")
        if info:
            for i in range(N):
                log.info(f"Client {i + 1} {cfg.metric} score: {metrics[i]}")
        if fed.write_reports:
            m_ = metrics.copy()
            fed.writer.submit(lambda m_=m_, rnd=rnd: fed._report_round(rnd, m_))
        fed.last_metrics = metrics
        if cfg.save_latents and fed.model_type == "hybrid" and fed.local:
            # LatentData pickles: every hosted client's test-set
            # latents of this round's evaluation.  The side slot's plan is not
            # reused before this round is collected (NSIDE > max_pending).
            p = eng._plan(fed.model_type, rec["eval_params"])
            st = eng.store
            fed.latent_log[rnd] = {fed.clients[c].name: (l.detach().cpu().numpy().astype(np.float32),
                                                         st.labels(i).astype(np.float32))
                                   for i, (c, l) in enumerate(zip(fed.local, p["test_lat"]))}
        if cfg.debug_replica_check:
            fed.check_replicas(rnd, rec["selected"], aggregator, metrics)
        stop = False
        if cfg.global_early_stop:
            from ..federation import metric_stats

            stop = fed.early.update(metric_stats(metrics)[1])
        rec.update(aggregator=aggregator, metrics=metrics, verification=verification, epochs_run=epochs_local,
                   stop=stop, done=True)
        for key in ("handle", "snap_slot", "slot", "report", "_keep", "event", "eval_params", "eval_timing", "train_ev"):
            rec.pop(key, None)
        self.all_rounds.pop(rnd, None)
