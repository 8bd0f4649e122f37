"""A failed training launch is stopped on the device (VERDICT r4 Next #5,
ADVICE r4 medium).

The helper-wave kernel's FedProx instantiation hands W4 from each helper wave
to its main wave through an LDS flag with a bounded wait
(`fedmx_train_hw.hip`, `FEDMX_HW_FLAGS_PROX=1`).  A wait that runs out marks
the launch failed: every wave ORs its failure bit into an LDS word before the
epilogue's last barrier, thread 0 alone then writes `epochs_run = -1000` and
sets the round's error word (`TrainArgs.err`).  The election kernel reads that
word (with collectives: every rank's, riding the model all-gather) and elects
nobody, so nothing is aggregated or adopted, and reports ELECT_TRAIN_FAILED;
the host raises at its next look at the round instead of two rounds later.

The failure is injected with the runtime test bit TRAIN_FLAG_TEST_DROP_W4
(helper 0 never publishes launch step 3's W4), i.e. through the production
library, not a special build.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from fedmse_decentralized_amd.config import ExperimentConfig


def _cfg(out, **kw):
    base = dict(synthetic="nbaiot", network_size=6, num_rounds=3, epoch=1, batch_size=12, output_root=out,
                backend="hip", device="cuda", log_level="WARNING", compat="fixed", global_early_stop=False,
                save_checkpoints=False, model_types=["hybrid"], update_types=["fedprox"])
    base.update(kw)
    return ExperimentConfig(**base)


def _engine(mu):
    from fedmse_decentralized_amd.data.prepare import prepare_federation
    from fedmse_decentralized_amd.data.synthetic import SyntheticSpec, generate_federation
    from fedmse_decentralized_amd.engine.hip_engine import HipEngine
    from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS
    from fedmse_decentralized_amd.models.reference import init_client_params

    raws = generate_federation(SyntheticSpec(kind="nbaiot", n_clients=2, seed=4))
    clients, _ = prepare_federation(raws, 1234)
    init, _ = init_client_params(2, 0)
    eng = HipEngine(DEFAULT_DIMS, torch.device("cuda", 0))
    eng.setup([c.train for c in clients], [c.valid for c in clients], [c.test for c in clients],
              [c.test_label for c in clients], init)
    return eng


def test_engine_raises_on_injected_flag_timeout(monkeypatch):
    """HipEngine: the launch reports -1000 for the client whose wave timed out
    and sets the error word; train_collect raises."""
    from fedmse_decentralized_amd.engine.base import TrainHParams
    from fedmse_decentralized_amd.ops import _hip

    eng = _engine(0.001)
    err = torch.zeros(1, dtype=torch.int32, device=eng.device)
    eng.train_err_ptr = err.data_ptr()
    monkeypatch.setattr(_hip, "TRAIN_TEST_FLAGS", _hip.TRAIN_FLAG_TEST_DROP_W4)
    hp = TrainHParams(epochs=1, batch_size=12, lr=1e-3, shrink_lambda=5.0, fedprox_mu=0.001)
    h = eng.train_launch([0, 1], hp)
    torch.cuda.synchronize()
    er = np.array(h.tensors[1])
    assert er.tolist() == [-1000, -1000], er
    assert int(err.item()) == 1
    with pytest.raises(RuntimeError, match="flag wait"):
        eng.train_collect(h)
    # the same launch without the injection: ok, error word untouched
    monkeypatch.setattr(_hip, "TRAIN_TEST_FLAGS", 0)
    err.zero_()
    res = eng.train_collect(eng.train_launch([0, 1], hp))
    assert res.epochs_run.tolist() == [1, 1]
    assert int(err.item()) == 0


def test_device_round_blocks_adoption_after_failed_launch(tmp_path, monkeypatch):
    """Device protocol: the failed round elects nobody, nothing is aggregated
    or adopted (every client that did not train keeps its parameters), and the
    host raises at the next enqueue once the round's election has run."""
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.ops import _hip

    federation._PREP_CACHE.clear()
    fed = Federation(_cfg(tmp_path), "hybrid", "fedprox", 0).setup()
    dr = fed._fast
    assert dr is not None, "device round expected on the HIP engine in fixed mode"
    st = fed.engine.store
    torch.cuda.synchronize()
    before = st.params.clone()
    monkeypatch.setattr(_hip, "TRAIN_TEST_FLAGS", _hip.TRAIN_FLAG_TEST_DROP_W4)
    r = fed.run_round()
    torch.cuda.synchronize()
    rec = dr.all_rounds[r.round]
    assert int(rec["report"][0]) == _hip.ELECT_TRAIN_FAILED
    assert int(dr.state[0].item()) == -1
    assert int(dr.err.item()) == 1
    sel = set(r.selected)
    for c in range(fed.N):
        if c not in sel:   # no adoption: untouched by this round
            assert torch.equal(st.params[c], before[c]), c
    monkeypatch.setattr(_hip, "TRAIN_TEST_FLAGS", 0)
    with pytest.raises(RuntimeError, match="training launch failed"):
        fed.run_round()


def test_engine_raises_when_a_validator_never_answers(monkeypatch):
    """VERDICT r5 Next #2b: asynchronous validation (plain instantiation) with
    client slot 0's validator workgroup muted (runtime test bit
    TRAIN_FLAG_TEST_MUTE_VALIDATOR; the decision wait is 0.2 s under it).  Its
    trainer's bounded wait runs out: that client reports -1000, the launch's
    error word is set and the host raises; the other client's launch result
    stands."""
    from fedmse_decentralized_amd.engine.base import TrainHParams
    from fedmse_decentralized_amd.ops import _hip

    eng = _engine(0.0)
    err = torch.zeros(1, dtype=torch.int32, device=eng.device)
    eng.train_err_ptr = err.data_ptr()
    monkeypatch.setattr(_hip, "TRAIN_TEST_FLAGS", _hip.TRAIN_FLAG_TEST_MUTE_VALIDATOR)
    hp = TrainHParams(epochs=3, batch_size=12, lr=1e-3, shrink_lambda=5.0, fedprox_mu=0.0, patience=10 ** 6)
    h = eng.train_launch([0, 1], hp)
    torch.cuda.synchronize()
    assert _hip.lib().fedmx_train_hw_last_grid() == 4, "validator workgroups expected"
    er = np.array(h.tensors[1])
    assert er.tolist() == [-1000, 3], er
    assert int(err.item()) == 1
    with pytest.raises(RuntimeError, match="decision wait"):
        eng.train_collect(h)
    monkeypatch.setattr(_hip, "TRAIN_TEST_FLAGS", 0)
    err.zero_()
    res = eng.train_collect(eng.train_launch([0, 1], hp))
    assert res.epochs_run.tolist() == [3, 3]
    assert int(err.item()) == 0


def test_device_round_blocks_adoption_after_muted_validator(tmp_path, monkeypatch):
    """The device protocol after a validator decision wait ran out: nobody is
    elected, nothing aggregated or adopted, and the host raises next round."""
    from fedmse_decentralized_amd import federation
    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.ops import _hip

    federation._PREP_CACHE.clear()
    fed = Federation(_cfg(tmp_path, update_types=["avg"], epoch=3), "hybrid", "avg", 0).setup()
    dr = fed._fast
    assert dr is not None, "device round expected on the HIP engine in fixed mode"
    st = fed.engine.store
    torch.cuda.synchronize()
    before = st.params.clone()
    monkeypatch.setattr(_hip, "TRAIN_TEST_FLAGS", _hip.TRAIN_FLAG_TEST_MUTE_VALIDATOR)
    r = fed.run_round()
    torch.cuda.synchronize()
    rec = dr.all_rounds[r.round]
    assert int(rec["report"][0]) == _hip.ELECT_TRAIN_FAILED
    assert int(dr.err.item()) == 1
    sel = set(r.selected)
    for c in range(fed.N):
        if c not in sel:
            assert torch.equal(st.params[c], before[c]), c
    monkeypatch.setattr(_hip, "TRAIN_TEST_FLAGS", 0)
    with pytest.raises(RuntimeError, match="training launch failed"):
        fed.run_round()
