"""End-to-end parity (SURVEY §4 tier T4): the same federation run through the
HIP engine on the MI355X and through the plain-PyTorch CPU engine (the
numerical oracle), reference-compat mode (host decisions, the reference's
torch RNG stream replayed).  Selections, elections and verification results
must agree exactly; AUCs and parameters to fp32-trajectory tolerance."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from fedmse_decentralized_amd.config import ExperimentConfig

from test_device_protocol_gpu import _shrink


def _run(out, backend, device, model_type, update_type, rounds=3, batch_size=12):
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    cfg = ExperimentConfig(synthetic="nbaiot", network_size=6, num_rounds=rounds, epoch=2, batch_size=batch_size,
                           output_root=out, backend=backend, device=device, log_level="WARNING",
                           compat="reference", global_early_stop=False, save_checkpoints=False,
                           model_types=[model_type], update_types=[update_type])
    federation._PREP_CACHE.clear()
    fed = Federation(cfg, model_type, update_type, 0).setup()
    assert fed._fast is None          # reference compat: host decisions on both engines
    rs = [fed.run_round() for _ in range(rounds)]
    fed.finish()
    fed.writer.flush()
    if device == "cuda":
        torch.cuda.synchronize()
    return fed, rs


@pytest.mark.parametrize("model_type,update_type", [("hybrid", "mse_avg"), ("autoencoder", "avg"),
                                                    ("hybrid", "fedprox")])
def test_hip_engine_matches_torch_engine(tmp_path, model_type, update_type):
    _shrink()
    fh, rh = _run(str(tmp_path / "hip"), "hip", "cuda", model_type, update_type)
    ft, rt = _run(str(tmp_path / "torch"), "torch", "cpu", model_type, update_type)
    assert fh.engine.name == "hip" and ft.engine.name == "torch"
    for a, b in zip(rh, rt):
        assert a.selected == b.selected
        assert a.aggregator == b.aggregator
        assert a.verification == b.verification
        np.testing.assert_allclose(np.array(a.metrics), np.array(b.metrics), atol=2e-3)
    torch.testing.assert_close(fh.engine.store.params.cpu(), ft.engine.store.params, rtol=2e-2, atol=2e-4)


@pytest.mark.parametrize("update_type", ["mse_avg", "fedprox"])
def test_hip_engine_matches_torch_engine_batch_64(tmp_path, update_type):
    """The thesis's batch-64 configuration end to end: the helper-wave
    kernel's 16-row-chunk path (batches over 12 rows) inside the federation,
    against the CPU oracle."""
    _shrink()
    fh, rh = _run(str(tmp_path / "hip"), "hip", "cuda", "hybrid", update_type, batch_size=64)
    ft, rt = _run(str(tmp_path / "torch"), "torch", "cpu", "hybrid", update_type, batch_size=64)
    for a, b in zip(rh, rt):
        assert a.selected == b.selected
        assert a.aggregator == b.aggregator
        assert a.verification == b.verification
        np.testing.assert_allclose(np.array(a.metrics), np.array(b.metrics), atol=2e-3)
    torch.testing.assert_close(fh.engine.store.params.cpu(), ft.engine.store.params, rtol=2e-2, atol=2e-4)


def test_hip_device_protocol_matches_oracle_at_64_clients(tmp_path):
    """A 64-client federation (32 trained per round), fixed compat: the HIP
    engine's device-resident round against the plain-PyTorch CPU engine's
    host-decision round — same selections and aggregators, AUCs within
    fp32-trajectory tolerance, and no detection collapse."""
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    _shrink()
    runs = {}
    for backend, device in (("hip", "cuda"), ("torch", "cpu")):
        cfg = ExperimentConfig(synthetic="nbaiot", network_size=64, num_rounds=3, epoch=2, batch_size=12,
                               output_root=str(tmp_path / backend), backend=backend, device=device,
                               log_level="WARNING", compat="fixed", global_early_stop=False, save_checkpoints=False,
                               model_types=["hybrid"], update_types=["mse_avg"])
        federation._PREP_CACHE.clear()
        fed = Federation(cfg, "hybrid", "mse_avg", 0).setup()
        assert (fed._fast is not None) == (backend == "hip")
        rs = [fed.run_round() for _ in range(3)]
        fed.finish()
        runs[backend] = [(r.selected, r.aggregator, np.array(r.metrics)) for r in rs]
    for (sh, ah, mh), (st, at, mt) in zip(runs["hip"], runs["torch"]):
        assert sh == st and ah == at
        np.testing.assert_allclose(mh, mt, atol=5e-3)
        assert mh.mean() > 0.95 and mt.mean() > 0.95


def test_hip_256_client_federation_does_not_collapse(tmp_path):
    """256 N-BaIoT-shaped clients at their real sizes, 12 rounds on the HIP
    device protocol: with the shared initial model (init_mode auto under
    compat fixed) every round keeps the mean AUC near the 10-client level;
    with one independent init per client (the reference) it fell to 0.64 by
    round 3 (profiles/r3_network_scale_hip_per_client_init.jsonl)."""
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    from test_device_protocol_gpu import _full_size

    with _full_size():
        cfg = ExperimentConfig(synthetic="nbaiot", network_size=256, num_rounds=12, output_root=str(tmp_path),
                               backend="hip", device="cuda", log_level="WARNING", compat="fixed",
                               global_early_stop=False, save_checkpoints=False,
                               model_types=["hybrid"], update_types=["mse_avg"])
        federation._PREP_CACHE.clear()
        fed = Federation(cfg, "hybrid", "mse_avg", 0).setup()
        assert fed._fast is not None and cfg.resolved_init_mode() == "shared"
        means = [float(np.mean(fed.run_round().metrics)) for _ in range(12)]
        fed.finish()
        federation._PREP_CACHE.clear()
    assert min(means) > 0.96, means


@pytest.mark.timeout(900)
def test_bench_config_20_rounds_matches_oracle(tmp_path):
    """VERDICT r3 Weak #4 (end-to-end horizon): the headline configuration
    (10 N-BaIoT-sized clients, 50 % participation, 5 local epochs, fixed
    compat, shared initial model) for 20 rounds, the HIP engine's
    device-resident round against the plain-PyTorch CPU engine's host round.

    The protocol's discrete outcomes are themselves sensitive at the last
    bit: the oracle re-run with lr x (1 + 2^-23) elects a different
    aggregator from round 5 on (profiles/r5_long_horizon_sensitivity.md: a
    near-tie of two candidates' vote scores).  So the HIP run must agree with
    the oracle in every discrete outcome (selection, aggregator, each
    receiver's verification decision) for at least as many rounds as the
    oracle agrees with that perturbed copy of itself, with per-client AUCs
    within 5e-3 there; and over all 20 rounds its per-round mean AUC must stay
    as close to the oracle's as the perturbed oracle's does (x2, floor 5e-3)."""
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation

    rounds = 20

    def run(backend, device, lr):
        cfg = ExperimentConfig(synthetic="nbaiot", network_size=10, num_rounds=rounds, epoch=5, batch_size=12,
                               lr_rate=lr, output_root=str(tmp_path / f"{backend}{lr}"), backend=backend,
                               device=device, log_level="ERROR", compat="fixed", global_early_stop=False,
                               save_checkpoints=False, model_types=["hybrid"], update_types=["mse_avg"])
        federation._PREP_CACHE.clear()
        fed = Federation(cfg, "hybrid", "mse_avg", 0, write_reports=False).setup()
        assert (fed._fast is not None) == (backend == "hip")
        out = []
        for _ in range(rounds):
            r = fed.run_round()
            ver = [(v["client_id"], v["is_verified"]) for v in (r.verification or [])]
            out.append((r.selected, r.aggregator, ver, np.array(r.metrics)))
        fed.finish()
        return out

    hip = run("hip", "cuda", 1e-3)
    ref = run("torch", "cpu", 1e-3)
    pert = run("torch", "cpu", 1e-3 * (1 + 2.0 ** -23))

    def horizon(a, b):
        for i, (x, y) in enumerate(zip(a, b)):
            if x[:3] != y[:3]:
                return i
        return rounds

    h_oracle = horizon(ref, pert)
    h_hip = horizon(hip, ref)
    worst = max((float(np.abs(hip[i][3] - ref[i][3]).max()) for i in range(h_hip)), default=0.0)
    mean_gap = max(abs(float(hip[i][3].mean() - ref[i][3].mean())) for i in range(rounds))
    mean_gap_oracle = max(abs(float(pert[i][3].mean() - ref[i][3].mean())) for i in range(rounds))
    print(f"bench config, {rounds} rounds: discrete agreement hip/oracle {h_hip} rounds, oracle/perturbed oracle "
          f"{h_oracle}; max |AUC hip - oracle| while agreeing {worst:.2e}; max per-round mean-AUC gap hip "
          f"{mean_gap:.2e}, perturbed oracle {mean_gap_oracle:.2e}")
    # at least as long as the oracle agrees with its own perturbed copy, and
    # never fewer than MIN_AGREE rounds (h_oracle can be 0; round 5
    # measured h_oracle 4 on the CPU, the HIP engine 15)
    MIN_AGREE = 5
    assert h_hip >= max(min(h_oracle, rounds), MIN_AGREE), (h_hip, h_oracle)
    assert worst < 5e-3
    assert mean_gap <= max(5e-3, 2 * mean_gap_oracle)
