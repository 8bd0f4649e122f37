"""The device-resident round (engine/device_round.py) against the host-decision
path on the same GPU: identical aggregators, verification results, metrics,
parameters and report files (fixed compat), single rank and two gloo ranks
sharing one GPU."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

from fedmse_decentralized_amd.config import ExperimentConfig

SHRINK = dict(normal_rows=(150, 170), abnormal_rows=(200, 220), test_normal_rows=30)


def _shrink():
    from fedmse_decentralized_amd.data import synthetic

    if getattr(synthetic.SyntheticSpec, "_fedmx_shrunk", False):
        return
    orig = synthetic.SyntheticSpec.resolved

    def resolved(self):
        s = orig(self)
        s.normal_rows, s.abnormal_rows, s.test_normal_rows = SHRINK["normal_rows"], SHRINK["abnormal_rows"], \
            SHRINK["test_normal_rows"]
        return s
    synthetic.SyntheticSpec.resolved = resolved
    synthetic.SyntheticSpec._fedmx_shrunk = True
    synthetic.SyntheticSpec._fedmx_orig_resolved = orig


class _full_size:
    """Temporarily undo _shrink (tests whose point is the real client sizes)."""

    def __enter__(self):
        from fedmse_decentralized_amd.data import synthetic

        self.cls = synthetic.SyntheticSpec
        self.saved = self.cls.resolved if getattr(self.cls, "_fedmx_shrunk", False) else None
        if self.saved is not None:
            self.cls.resolved = self.cls._fedmx_orig_resolved
        return self

    def __exit__(self, *exc):
        if self.saved is not None:
            self.cls.resolved = self.saved
        return False


def _cfg(out, **kw):
    base = dict(synthetic="nbaiot", network_size=6, num_rounds=6, epoch=2, batch_size=12, output_root=out,
                backend="hip", device="cuda", log_level="WARNING", compat="fixed", global_early_stop=False,
                save_checkpoints=True, model_types=["hybrid"], update_types=["mse_avg"])
    base.update(kw)
    return ExperimentConfig(**base)


def _run(cfg, update_type, rounds, comm=None):
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    federation._PREP_CACHE.clear()
    fed = Federation(cfg, "hybrid", update_type, 0, comm=comm).setup()
    rs = [fed.run_round() for _ in range(rounds)]
    fed.finish()
    fed.writer.flush()
    out = dict(agg=[r.aggregator for r in rs], metrics=[r.metrics.tolist() for r in rs],
               ver=[r.verification for r in rs], sel=[r.selected for r in rs])
    torch.cuda.synchronize()
    return fed, out


@pytest.mark.parametrize("update_type", ["mse_avg", "avg"])
def test_device_round_matches_host_path(tmp_path, update_type):
    _shrink()
    fa, a = _run(_cfg(str(tmp_path / "dev"), device_protocol=True), update_type, 6)
    fb, b = _run(_cfg(str(tmp_path / "host"), device_protocol=False), update_type, 6)
    assert fa._fast is not None and fb._fast is None
    assert a["sel"] == b["sel"]
    assert a["agg"] == b["agg"]
    assert a["ver"] == b["ver"]
    for x, y in zip(a["metrics"], b["metrics"]):
        np.testing.assert_array_equal(np.array(x), np.array(y))
    assert torch.equal(fa.engine.store.params, fb.engine.store.params)
    assert torch.equal(fa.engine.store.anchor, fb.engine.store.anchor)
    assert fa.agg_counts == fb.agg_counts
    # identical report files and checkpoint artefacts (device path: the native
    # writer thread; host path: the Python writer job)
    n_ckpt = 0
    for root_a, _, files in os.walk(str(tmp_path / "dev")):
        for fn in files:
            if fn in ("model.cpt", "training_tracking.pkl"):
                pa = os.path.join(root_a, fn)
                pb = pa.replace(str(tmp_path / "dev"), str(tmp_path / "host"))
                assert open(pa, "rb").read() == open(pb, "rb").read(), pa
                n_ckpt += 1
            if fn.endswith(".json"):
                pa = os.path.join(root_a, fn)
                pb = pa.replace(str(tmp_path / "dev"), str(tmp_path / "host"))
                assert open(pa).read() == open(pb).read(), fn
    assert n_ckpt >= 2 * 3   # every client trained at least once in 6 rounds of 3 selections


def test_device_round_early_stop_and_episode_reset(tmp_path):
    _shrink()
    cfg = _cfg(str(tmp_path), global_early_stop=True, num_rounds=8)
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    federation._PREP_CACHE.clear()
    fed = Federation(cfg, "hybrid", "avg", 0).setup()
    assert fed._fast is not None
    fed.run_all()
    assert 1 <= fed.round_idx <= 8
    fed.reset_aggregation_counts()
    assert int(fed._fast.agg_counts.sum()) == 0


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), FEDMX_DEVICE_INDEX="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    _shrink()
    from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown

    comm = init_comm(backend="gloo", device="cuda")
    fed, res = _run(_cfg(os.path.join(out, f"r{rank}"), save_checkpoints=False, debug_replica_check=True), "mse_avg",
                    4, comm=comm)
    res["fast"] = fed._fast is not None
    res["params"] = fed.engine.store.params.double().sum(1).tolist()
    res["local"] = fed.local
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    shutdown(comm)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_device_round_multi_rank_one_gpu(tmp_path, world):
    """world=4 shards 6 clients unevenly (2/2/1/1) over four gloo ranks."""
    out = str(tmp_path)
    mp.start_processes(_worker, args=(world, _port(), out), nprocs=world, join=True, start_method="spawn")
    _shrink()
    fed, ref = _run(_cfg(os.path.join(out, "single"), save_checkpoints=False), "mse_avg", 4)
    ref_params = fed.engine.store.params.double().sum(1).tolist()
    for r in range(world):
        d = json.load(open(os.path.join(out, f"rank{r}.json")))
        assert d["fast"]
        assert d["agg"] == ref["agg"] and d["sel"] == ref["sel"] and d["ver"] == ref["ver"]
        for x, y in zip(d["metrics"], ref["metrics"]):
            np.testing.assert_array_equal(np.array(x), np.array(y))
        loc = d["local"]
        assert d["params"] == ref_params[loc[0]:loc[-1] + 1]


def _edge_worker(rank, world, port, out, n_clients):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), FEDMX_DEVICE_INDEX="0", HSA_ENABLE_IPC_MODE_LEGACY="0",
                      FEDMX_COMM_SELFTEST="0")
    _shrink()
    from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown

    comm = init_comm(backend="gloo", device="cuda")
    fed, res = _run(_cfg(os.path.join(out, f"r{rank}"), network_size=n_clients, save_checkpoints=False,
                         debug_replica_check=True), "mse_avg", 3, comm=comm)
    res["fast"] = fed._fast is not None
    res["params"] = fed.engine.store.params.double().sum(1).tolist()
    res["local"] = fed.local
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    shutdown(comm)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n_clients", [10, 8, 4],
                         ids=["10-clients-over-8-ranks", "one-client-per-rank", "ranks-without-clients"])
def test_device_round_eight_ranks_edge_shapes(tmp_path, n_clients):
    """The device protocol in the shapes the first 8-GPU run meets (VERDICT r3
    Next #5): 8 gloo ranks sharing GPU 0 run the headline 10-client federation
    (most ranks have no selected client in a round), one client per rank
    (BASELINE config 3) and 4 clients (ranks hosting none).  Every rank must
    match the single-process device round's decisions and AUCs."""
    out = str(tmp_path)
    mp.start_processes(_edge_worker, args=(8, _port(), out, n_clients), nprocs=8, join=True, start_method="spawn")
    _shrink()
    fed, ref = _run(_cfg(os.path.join(out, "single"), network_size=n_clients, save_checkpoints=False), "mse_avg", 3)
    ref_params = fed.engine.store.params.double().sum(1).tolist()
    for r in range(8):
        d = json.load(open(os.path.join(out, f"rank{r}.json")))
        assert d["fast"]
        assert d["agg"] == ref["agg"] and d["sel"] == ref["sel"] and d["ver"] == ref["ver"]
        for x, y in zip(d["metrics"], ref["metrics"]):
            np.testing.assert_array_equal(np.array(x), np.array(y))
        loc = d["local"]
        assert d["params"] == (ref_params[loc[0]:loc[-1] + 1] if loc else [])


def test_device_round_is_deterministic(tmp_path):
    """Run-to-run determinism: two identical device-protocol
    runs give bit-identical parameters, Adam state and metrics."""
    _shrink()
    fa, a = _run(_cfg(str(tmp_path / "a"), save_checkpoints=False), "mse_avg", 4)
    fb, b = _run(_cfg(str(tmp_path / "b"), save_checkpoints=False), "mse_avg", 4)
    assert a == b
    for name in ("params", "adam_m", "adam_v", "anchor", "best"):
        assert torch.equal(getattr(fa.engine.store, name), getattr(fb.engine.store, name)), name


def test_bench_phantom_ranks_projection(tmp_path):
    """bench.py --phantom-ranks: rank 0 of a 4-rank weak-scaling job on one
    GPU (40 clients, collectives stubbed) runs and labels its record."""
    import json

    import bench

    out = tmp_path / "b.json"
    assert bench.main(["--phantom-ranks", "4", "--steps", "3", "--warmup", "1", "--no-artifacts",
                       "--out", str(out)]) == 0
    rec = json.loads(out.read_text())
    assert rec["config"]["clients"] == 40 and rec["config"]["device_protocol"]
    # a projection is never recorded as a multi-GPU measurement
    assert "projection" in rec and rec["value"] is None and rec["n_gpus"] == 1
    assert rec["projected_ranks"] == 4 and rec["projected_value"] > 0
    # only rank 0's own clients are evaluated: their AUCs, not zero-filled ones
    assert rec["detection_auc_min"] > 0.5


def test_rccl_one_rank_forced_collectives_match_loopback(tmp_path):
    """The multi-GPU code path with real RCCL on a one-GPU box: a one-rank
    nccl (= RCCL) process group with FEDMX_FORCE_COLLECTIVES=1 packs, all-gathers
    and all-reduces every round exactly as a rank of the N-GPU job does; its
    results are bit-identical to the loopback (no-collective) run."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(extra_env, name):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **extra_env)
        out = tmp_path / f"{name}.json"
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "6", "--warmup", "2",
                            "--no-artifacts", "--out", str(out)], env=env, cwd=root, capture_output=True,
                           text=True, timeout=150)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(out.read_text())

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    base = run({}, "loopback")
    forced = run({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(port), "FEDMX_FORCE_COLLECTIVES": "1"}, "rccl1")
    assert forced["config"]["device_protocol"] and base["config"]["device_protocol"]
    assert forced["detection_auc_mean"] == base["detection_auc_mean"]
    assert forced["detection_auc_min"] == base["detection_auc_min"]


def test_device_round_matches_host_path_large_selection(tmp_path):
    """24 clients (12 selections per round: the election kernel's
    one-element-per-thread aggregation path, k > 8) against the host path's
    weighted_sum_kernel: identical aggregators, decisions and parameters."""
    _shrink()
    fa, a = _run(_cfg(str(tmp_path / "dev"), device_protocol=True, network_size=24, save_checkpoints=False),
                 "mse_avg", 4)
    fb, b = _run(_cfg(str(tmp_path / "host"), device_protocol=False, network_size=24, save_checkpoints=False),
                 "mse_avg", 4)
    assert fa._fast is not None and fb._fast is None
    assert len(a["sel"][0]) == 12
    assert a["sel"] == b["sel"] and a["agg"] == b["agg"] and a["ver"] == b["ver"]
    assert torch.equal(fa.engine.store.params, fb.engine.store.params)
    assert torch.equal(fa.engine.store.anchor, fb.engine.store.anchor)


def test_device_round_resume_matches_uninterrupted(tmp_path):
    """Checkpoint / resume on the device-resident protocol: a
    federation resumed from a round-3 snapshot (parameters, Adam state,
    aggregation caps, verifier histories, tie-break noise stream) continues
    bit-identically to the uninterrupted run."""
    _shrink()
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    federation._PREP_CACHE.clear()
    a = Federation(_cfg(str(tmp_path / "a"), save_checkpoints=False), "hybrid", "mse_avg", 0).setup()
    assert a._fast is not None
    for _ in range(3):
        a.run_round()
    snap = a.save_snapshot(str(tmp_path / "snap.pt"))
    ra = [a.run_round() for _ in range(3)]
    a.finish()
    ra = [(r.aggregator, r.metrics.tolist(), r.verification) for r in ra]
    federation._PREP_CACHE.clear()
    b = Federation(_cfg(str(tmp_path / "b"), save_checkpoints=False, resume=snap), "hybrid", "mse_avg", 0).setup()
    assert b._fast is not None and b.round_idx == 3
    rb = [b.run_round() for _ in range(3)]
    b.finish()
    rb = [(r.aggregator, r.metrics.tolist(), r.verification) for r in rb]
    assert ra == rb
    for name in ("params", "adam_m", "adam_v", "anchor", "best"):
        assert torch.equal(getattr(a.engine.store, name), getattr(b.engine.store, name)), name
    for name in ("agg_counts", "hist", "has_hist", "hist_perf", "rejected"):
        assert torch.equal(getattr(a._fast, name), getattr(b._fast, name)), name


def test_device_round_auc_with_a_class_beyond_the_lds_sort(tmp_path):
    """Clients whose test classes both exceed the AUC kernel's 8,192-key LDS
    sort (~9,000 benign and ~10,000 attack rows): the device protocol falls back to the exact
    host AUC for them instead of failing, and reports the host
    path's metrics."""
    from fedmse_decentralized_amd.data import synthetic

    cls = synthetic.SyntheticSpec
    saved = cls.resolved
    base = getattr(cls, "_fedmx_orig_resolved", saved)

    def big(self):
        s = base(self)
        # both test classes beyond the sort (the kernel sorts the smaller one)
        s.normal_rows, s.abnormal_rows, s.test_normal_rows = (150, 170), (10000, 10040), 9000
        return s
    cls.resolved = big
    try:
        fa, a = _run(_cfg(str(tmp_path / "dev"), save_checkpoints=False, network_size=4), "mse_avg", 3)
        fb, b = _run(_cfg(str(tmp_path / "host"), save_checkpoints=False, network_size=4, device_protocol=False),
                     "mse_avg", 3)
    finally:
        cls.resolved = saved
    assert fa._fast is not None and fb._fast is None
    lab = fa.engine.store.labels(0)
    assert min(int(lab.sum()), int((lab == 0).sum())) > 8192
    assert a == b
    assert all(0.5 < m <= 1.0 for ms in a["metrics"] for m in ms)


def test_host_snapshot_resumed_on_device_path(tmp_path):
    """A resume snapshot written by the host-decision path (no device entry)
    resumed with the device protocol: the device state is seeded from the
    restored host state (caps, verifier histories, rejection counts), so the
    resumed rounds equal the uninterrupted host-path run's."""
    _shrink()
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    federation._PREP_CACHE.clear()
    a = Federation(_cfg(str(tmp_path / "a"), save_checkpoints=False, device_protocol=False), "hybrid", "mse_avg",
                   0).setup()
    assert a._fast is None
    for _ in range(3):
        a.run_round()
    snap = a.save_snapshot(str(tmp_path / "snap.pt"))
    ra = [a.run_round() for _ in range(3)]
    ra = [(r.aggregator, r.verification) for r in ra]
    federation._PREP_CACHE.clear()
    b = Federation(_cfg(str(tmp_path / "b"), save_checkpoints=False, resume=snap), "hybrid", "mse_avg", 0).setup()
    assert b._fast is not None and b.round_idx == 3
    rb = [b.run_round() for _ in range(3)]
    b.finish()
    rb = [(r.aggregator, r.verification) for r in rb]
    assert ra == rb
    torch.testing.assert_close(a.engine.store.params, b.engine.store.params, rtol=0, atol=0)


def test_device_round_save_latents_matches_host_path(tmp_path):
    """--save-latents (LatentData pickles) on the device-resident
    protocol: the same per-round test-set latents as the host path."""
    _shrink()
    fa, _ = _run(_cfg(str(tmp_path / "dev"), save_checkpoints=False, save_latents=True), "mse_avg", 4)
    fb, _ = _run(_cfg(str(tmp_path / "host"), save_checkpoints=False, save_latents=True, device_protocol=False),
                 "mse_avg", 4)
    assert fa._fast is not None and fb._fast is None
    assert sorted(fa.latent_log) == sorted(fb.latent_log) == [0, 1, 2, 3]
    for r in fa.latent_log:
        assert sorted(fa.latent_log[r]) == sorted(fb.latent_log[r])
        for name, (lat, lab) in fa.latent_log[r].items():
            lat_b, lab_b = fb.latent_log[r][name]
            assert lat.shape[1] == 7
            np.testing.assert_array_equal(lat, lat_b)
            np.testing.assert_array_equal(lab, lab_b)


def test_device_round_fault_injection_matches_host_path(tmp_path):
    """Fault injection on the device-resident protocol: a dropped client
    never trains, votes or aggregates, a malicious client's poisoned update
    is screened by the verifiers — decisions, counts and parameters equal the
    host path's."""
    _shrink()
    kw = dict(save_checkpoints=False, dropped_clients=[1], malicious_clients=[2], malicious_scale=25.0)
    fa, a = _run(_cfg(str(tmp_path / "dev"), **kw), "mse_avg", 6)
    fb, b = _run(_cfg(str(tmp_path / "host"), device_protocol=False, **kw), "mse_avg", 6)
    assert fa._fast is not None and fb._fast is None
    assert all(1 not in s for s in a["sel"])
    assert a["sel"] == b["sel"] and a["agg"] == b["agg"] and a["ver"] == b["ver"]
    for x, y in zip(a["metrics"], b["metrics"]):
        np.testing.assert_array_equal(np.array(x), np.array(y))
    assert torch.equal(fa.engine.store.params, fb.engine.store.params)
    assert fa.agg_counts == fb.agg_counts


def test_device_round_sample_weighted_fedavg_matches_host_path(tmp_path):
    """Sample-weighted FedAvg (weights ∝ training-set size) on the device
    protocol (host-computed weights, rule 2 of the election kernel): the same
    aggregates as the host path's weighted_sum."""
    _shrink()
    fa, a = _run(_cfg(str(tmp_path / "dev"), save_checkpoints=False, fedavg_sample_weighted=True), "avg", 4)
    fb, b = _run(_cfg(str(tmp_path / "host"), save_checkpoints=False, fedavg_sample_weighted=True,
                      device_protocol=False), "avg", 4)
    fc, c = _run(_cfg(str(tmp_path / "mean"), save_checkpoints=False), "avg", 4)
    assert fa._fast is not None and fa._fast.rule == 2 and fb._fast is None
    assert a["sel"] == b["sel"] and a["agg"] == b["agg"] and a["ver"] == b["ver"]
    assert torch.equal(fa.engine.store.params, fb.engine.store.params)
    # and the weighting is not the plain mean's
    assert not torch.equal(fa.engine.store.params, fc.engine.store.params)


@pytest.mark.parametrize("election,mode,n", [("majority", "decentralized", 6), ("first_voter", "centralized", 6),
                                              ("majority", "centralized", 6), ("majority", "decentralized", 132)])
def test_device_round_protocol_variants_match_host_path(tmp_path, election, mode, n):
    """The legacy centralised GlobalAggregator variants on the
    device protocol: majority election (every selected client votes; the
    k > 64 case takes the election kernel's serial path) and the centralised
    push (every client adopts and re-anchors, nothing verified) match the
    host-decision path."""
    _shrink()
    kw = dict(save_checkpoints=False, election=election, aggregation_mode=mode, network_size=n)
    rounds = 4 if n < 100 else 2
    fa, a = _run(_cfg(str(tmp_path / "dev"), **kw), "mse_avg", rounds)
    fb, b = _run(_cfg(str(tmp_path / "host"), device_protocol=False, **kw), "mse_avg", rounds)
    assert fa._fast is not None and fb._fast is None
    assert a["sel"] == b["sel"] and a["agg"] == b["agg"] and a["ver"] == b["ver"]
    for x, y in zip(a["metrics"], b["metrics"]):
        np.testing.assert_array_equal(np.array(x), np.array(y))
    assert torch.equal(fa.engine.store.params, fb.engine.store.params)
    assert torch.equal(fa.engine.store.anchor, fb.engine.store.anchor)
    assert fa.agg_counts == fb.agg_counts
    if mode == "centralized":
        assert all(v == [] for v in a["ver"])


@pytest.mark.parametrize("rel,fused", [(0.05, True), (0.5, True), (0.05, False)])
def test_device_round_relative_drift_threshold_matches_host_path(tmp_path, monkeypatch, rel, fused):
    """drift_threshold_rel (fixed-mode option, profiles/r4_adoption_ablation.md):
    the device kernels' relative drift limit (mode 3: drift <= rel x
    sum_tensors ||history||) reaches the host verifier's decisions, on the
    fused verification kernel and on decide_adopt (fused=False: the fused
    kernel's row limit forced below the data size)."""
    from fedmse_decentralized_amd.ops import _hip

    _shrink()
    if not fused:
        monkeypatch.setattr(_hip, "VERIFY_MAX_ROWS", 1)
    kw = dict(save_checkpoints=False, drift_threshold_rel=rel)
    fa, a = _run(_cfg(str(tmp_path / "dev"), **kw), "mse_avg", 6)
    fb, b = _run(_cfg(str(tmp_path / "host"), device_protocol=False, **kw), "mse_avg", 6)
    assert fa._fast is not None and fb._fast is None
    assert fa._fast.fused_verify == fused
    assert a["sel"] == b["sel"] and a["agg"] == b["agg"] and a["ver"] == b["ver"]
    for x, y in zip(a["metrics"], b["metrics"]):
        np.testing.assert_array_equal(np.array(x), np.array(y))
    assert torch.equal(fa.engine.store.params, fb.engine.store.params)
    rejected = sum(1 for v in a["ver"] for d in v if not d["is_verified"])
    if rel == 0.05:
        assert rejected > 0   # a tight limit does reject


@pytest.mark.parametrize("model_type", ["hybrid", "autoencoder"])
def test_device_round_classification_metric_matches_host_path(tmp_path, model_type):
    """--metric classification (F1 at threshold 0.5, the reference
    Evaluator's alternative metric) on the device protocol: the same per-client
    F1 as the host path's evaluator; --metric time reports positive seconds."""
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    _shrink()

    def go(out, **kw):
        federation._PREP_CACHE.clear()
        fed = Federation(_cfg(out, save_checkpoints=False, **kw), model_type, "avg", 0).setup()
        rs = [fed.run_round() for _ in range(3)]
        fed.finish()
        return fed, [r.metrics.tolist() for r in rs]

    fa, a = go(str(tmp_path / "dev"), metric="classification")
    fb, b = go(str(tmp_path / "host"), metric="classification", device_protocol=False)
    assert fa._fast is not None and fb._fast is None
    assert a == b
    assert all(0.0 <= v <= 1.0 for m in a for v in m)
    ft, t = go(str(tmp_path / "time"), metric="time")
    assert ft._fast is not None
    assert all(v > 0 for m in t for v in m)


@pytest.mark.parametrize("election,vote_cap", [("first_voter", 3.0), ("first_voter", 1e-9), ("majority", 1e-9)])
def test_device_round_thesis_variant_matches_host_path(tmp_path, election, vote_cap):
    """The thesis protocol (Thesis p.20-26: vote-MSE cap, random eligible
    aggregator when nobody is voted for, loss-ratio acceptance against the
    receiver's own model) on the device protocol matches the host path; a
    tiny cap forces the random fallback every round."""
    _shrink()
    kw = dict(save_checkpoints=False, protocol_variant="thesis", election=election, thesis_vote_mse_cap=vote_cap)
    fa, a = _run(_cfg(str(tmp_path / "dev"), **kw), "mse_avg", 5)
    fb, b = _run(_cfg(str(tmp_path / "host"), device_protocol=False, **kw), "mse_avg", 5)
    assert fa._fast is not None and fb._fast is None
    assert a["sel"] == b["sel"] and a["agg"] == b["agg"] and a["ver"] == b["ver"]
    assert all(x is not None for x in a["agg"])
    for x, y in zip(a["metrics"], b["metrics"]):
        np.testing.assert_array_equal(np.array(x), np.array(y))
    assert torch.equal(fa.engine.store.params, fb.engine.store.params)
    assert torch.equal(fa.engine.store.anchor, fb.engine.store.anchor)
    assert fa.agg_counts == fb.agg_counts


def _worker_kw(rank, world, port, out, kw):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), FEDMX_DEVICE_INDEX="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    _shrink()
    from fedmse_decentralized_amd.parallel.launch import init_comm, shutdown

    comm = init_comm(backend="gloo", device="cuda")
    kw = dict(kw)
    ut = kw.pop("_update", "mse_avg")
    fed, res = _run(_cfg(os.path.join(out, f"r{rank}"), save_checkpoints=False, debug_replica_check=True, **kw),
                    ut, 4, comm=comm)
    res["fast"] = fed._fast is not None
    res["params"] = fed.engine.store.params.double().sum(1).tolist()
    res["local"] = fed.local
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    shutdown(comm)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kw", [dict(protocol_variant="thesis", election="majority"),
                                dict(metric="classification", fedavg_sample_weighted=True),
                                dict(aggregation_mode="centralized", dropped_clients=[2]),
                                # poisoned updates: receivers on both ranks reject, and every
                                # side slot is reused (4 rounds > 3 slots) with fresh counts
                                dict(malicious_clients=[1, 4], malicious_scale=25.0),
                                # fusion weights formed on each rank's GPU from the gathered models
                                dict(_update="fusion_avg", fusion_max_rows=256)])
def test_device_round_variants_multi_rank_one_gpu(tmp_path, kw):
    """Protocol variants on the device path with two gloo ranks sharing one
    GPU: every rank reaches the single-process run's decisions, metrics and
    parameters (replicated state checked every round)."""
    out = str(tmp_path)
    mp.start_processes(_worker_kw, args=(2, _port(), out, kw), nprocs=2, join=True, start_method="spawn")
    _shrink()
    kw = dict(kw)
    ut = kw.pop("_update", "mse_avg")
    fed, ref = _run(_cfg(os.path.join(out, "single"), save_checkpoints=False, **kw), ut, 4)
    ref_params = fed.engine.store.params.double().sum(1).tolist()
    for r in range(2):
        d = json.load(open(os.path.join(out, f"rank{r}.json")))
        assert d["fast"]
        assert d["agg"] == ref["agg"] and d["sel"] == ref["sel"] and d["ver"] == ref["ver"]
        for x, y in zip(d["metrics"], ref["metrics"]):
            np.testing.assert_array_equal(np.array(x), np.array(y))
        loc = d["local"]
        assert d["params"] == ref_params[loc[0]:loc[-1] + 1]


def test_device_round_fusion_avg_matches_host_path(tmp_path):
    """fusion_avg on the device round: the KDE / JS weights formed on the GPU
    each round (no host round trip) give the host-decision path's rounds."""
    _shrink()
    kw = dict(save_checkpoints=False, fusion_max_rows=256)
    fa, a = _run(_cfg(str(tmp_path / "dev"), device_protocol=True, update_types=["fusion_avg"], **kw), "fusion_avg", 4)
    fb, b = _run(_cfg(str(tmp_path / "host"), device_protocol=False, update_types=["fusion_avg"], **kw),
                 "fusion_avg", 4)
    assert fa._fast is not None and fb._fast is None
    assert a == b
    assert torch.equal(fa.engine.store.params, fb.engine.store.params)


@pytest.mark.parametrize("rel,network_size", [(0.0, 10), (0.05, 10), (0.0, 40)])
def test_split_verification_matches_fused_kernel(tmp_path, monkeypatch, rel, network_size):
    """VERDICT r5 Next #7: the split verification kernel (each receiver's
    forward over several workgroups plus a drift workgroup, the last arriver
    decides; fedmx_protocol.hip verify_split_kernel) against the fused
    one-workgroup-per-receiver kernel: bit-identical decisions, parameters,
    anchors, histories, per-round metrics and rejection counts, over rounds
    with absolute (mode 0) and relative (mode 3) drift limits, at the
    synthetic clients' real sizes (verification sets of ~100-250 rows: two
    forward workgroups per receiver) and 40 clients (shorter sets)."""
    from fedmse_decentralized_amd.ops import _hip

    kw = dict(save_checkpoints=False, network_size=network_size, num_rounds=5, drift_threshold_rel=rel)
    with _full_size():
        monkeypatch.setattr(_hip, "VERIFY_SPLIT", True)
        fa, a = _run(_cfg(str(tmp_path / "split"), **kw), "mse_avg", 5)
        monkeypatch.setattr(_hip, "VERIFY_SPLIT", False)
        fb, b = _run(_cfg(str(tmp_path / "fused"), **kw), "mse_avg", 5)
    assert fa._fast.vsplit is not None and fb._fast.vsplit is None
    assert fa._fast.vsplit.splits >= 1
    assert a["sel"] == b["sel"] and a["agg"] == b["agg"] and a["ver"] == b["ver"]
    for x, y in zip(a["metrics"], b["metrics"]):
        np.testing.assert_array_equal(np.array(x), np.array(y))
    for name in ("params", "anchor", "best"):
        assert torch.equal(getattr(fa.engine.store, name), getattr(fb.engine.store, name)), name
    for name in ("hist", "has_hist", "hist_perf", "rejected", "agg_counts"):
        assert torch.equal(getattr(fa._fast, name), getattr(fb._fast, name)), name
    # the arrival counters are back at zero after every launch
    assert int(fa._fast.vsplit_scratch[2].abs().sum()) == 0
