"""Protocol state machine: selection, election, aggregation plans (incl. the
reference's state-dict aliasing quirk Q2), verification and early stop."""
import random

import numpy as np
import pytest
import torch

from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS, state_dict_to_canonical
from fedmse_decentralized_amd.models.reference import ReferenceSAE
from fedmse_decentralized_amd.protocol.aggregation import make_plan, plan_mean, plan_mse_avg
from fedmse_decentralized_amd.protocol.early_stop import GlobalEarlyStop
from fedmse_decentralized_amd.protocol.election import elect_aggregator, select_clients
from fedmse_decentralized_amd.protocol.verification import Verifier, VerifierState


class _FixedNoise:
    def __init__(self, vals=None):
        self.vals = list(vals or [])

    def rand(self):
        return self.vals.pop(0) if self.vals else 0.5


def test_selection_matches_python_random_sample():
    a = random.Random(1234)
    b = random.Random(1234)
    assert select_clients(a, 10, 0.5) == b.sample(range(10), 5)
    assert len(select_clients(a, 10, 0.01)) == 1   # max(1, int(p*N))


def test_election_excludes_voter_and_respects_cap():
    sel = [4, 1, 7, 2]
    scores = {4: 0.1, 1: 0.5, 7: 0.2, 2: 0.3}
    counts = [0] * 10
    r = elect_aggregator(sel, scores, counts, 3, _FixedNoise())
    assert r.voter == 4 and r.aggregator == 7         # voter 4 cannot pick itself
    counts[7] = 3
    r = elect_aggregator(sel, scores, counts, 3, _FixedNoise())
    assert r.aggregator == 2
    # every candidate of the first voter capped -> the second voter decides
    counts = [0] * 10
    for c in (1, 7, 2):
        counts[c] = 3
    r = elect_aggregator(sel, scores, counts, 3, _FixedNoise())
    assert r.voter == 1 and r.aggregator == 4
    counts[4] = 3
    assert elect_aggregator(sel, scores, counts, 3, _FixedNoise()).aggregator is None


def test_election_noise_breaks_ties():
    sel = [0, 1, 2]
    scores = {0: 1.0, 1: 1.0, 2: 1.0}
    # noise factor 1 + (u-0.5)*2e-4: lower u -> lower score
    r = elect_aggregator(sel, scores, [0, 0, 0], 3, _FixedNoise([0.9, 0.1]))
    assert r.aggregator == 2


def _reference_fed_mse_avg(models, aggregator_index, dev):
    """The reference's aggregate_models + fed_mse_avg with real nn.Modules
    (state_dict() aliasing included, src/Trainer/client_trainer.py:115-130, :306-315)."""
    agg_model = models[aggregator_index]
    local_models = [(m.state_dict(), 1.0) for m in models]
    update_weights = []
    for state, _ in local_models:
        agg_model.load_state_dict(state)
        with torch.no_grad():
            _, gen, _ = agg_model(dev)
            mse = torch.nn.MSELoss(reduction="mean")(dev, gen)
            update_weights.append((state, 1 / mse))
    total = sum(w for _, w in update_weights)
    out = {}
    for key in update_weights[0][0].keys():
        out[key] = sum(w[key] * (wt / total) for w, wt in update_weights)
    return out


@pytest.mark.parametrize("a", [0, 2, 4])
def test_mse_avg_compat_plan_reproduces_aliasing(a):
    torch.manual_seed(0)
    K = 5
    models = [ReferenceSAE(DEFAULT_DIMS, shrink_lambda=0.0) for _ in range(K)]
    thetas = [state_dict_to_canonical(m.state_dict()).clone() for m in models]
    dev = torch.randn(64, 115)
    # true per-model dev MSEs (computed before any aliasing mutation)
    mses = {}
    for k, m in enumerate(models):
        with torch.no_grad():
            _, gen, _ = m(dev)
            mses[k] = float(torch.nn.MSELoss()(dev, gen))
    ref = state_dict_to_canonical(_reference_fed_mse_avg(models, a, dev))
    plan = plan_mse_avg(list(range(K)), a, mses, compat="reference")
    ours = sum(torch.tensor(w, dtype=torch.float32) * thetas[src] for src, w in plan)
    torch.testing.assert_close(ours, ref, rtol=1e-5, atol=1e-6)
    fixed = plan_mse_avg(list(range(K)), a, mses, compat="fixed")
    assert sorted(src for src, _ in fixed) == list(range(K))
    assert abs(sum(w for _, w in fixed) - 1.0) < 1e-12


def test_mean_plan():
    p = make_plan("avg", [3, 1, 2], 1)
    assert [s for s, _ in p] == [3, 1, 2] and all(abs(w - 1 / 3) < 1e-15 for _, w in p)
    assert make_plan("fedprox", [3, 1], 3) == plan_mean([3, 1])
    with pytest.raises(ValueError):
        make_plan("bogus", [1], 1)


def test_verifier_boundaries():
    v = Verifier(3.0, 0.002)
    st = VerifierState()
    d = v.decide(0, st, version=0, perf_new=0.5, drift=99.0, current_round=0)
    assert d.verified and d.perf_change == 0.0       # first receipt always accepted
    d = v.decide(0, st, version=1, perf_new=0.5 - 0.0019, drift=3.0, current_round=1)
    assert d.verified                                # both bounds inclusive
    d = v.decide(0, st, version=2, perf_new=0.4981 - 0.0021, drift=0.1, current_round=2)
    assert not d.verified                            # perf drop
    d = v.decide(0, st, version=3, perf_new=0.9, drift=3.0001, current_round=3)
    assert not d.verified                            # drift too large
    assert st.history_version == 3 and st.history_perf == 0.9   # history updated regardless
    for _ in range(3):
        v.apply(0, st, d)
    assert st.rejected_updates == 3


def test_early_stop_compat_vs_fixed():
    ref = GlobalEarlyStop(1, "reference")
    # AUC compared as a loss: rising AUC counts as "worse"
    assert not ref.update(0.90)
    assert not ref.update(0.95)
    assert ref.update(0.96)
    ref.start_combination()          # NOT reset in compat mode (Q8)
    assert ref.update(0.99)
    fx = GlobalEarlyStop(1, "fixed")
    assert not fx.update(0.90) and not fx.update(0.95) and not fx.update(0.96)
    assert not fx.update(0.95)
    assert fx.update(0.94)
    fx.start_combination()
    assert not fx.update(0.5)


def test_sample_weighted_fedavg_plan():
    from fedmse_decentralized_amd.protocol.aggregation import make_plan

    plan = make_plan("avg", [2, 0, 1], 0, num_samples={0: 100, 1: 300, 2: 600})
    assert plan == [(2, 0.6), (0, 0.1), (1, 0.3)]
    assert make_plan("fedprox", [2, 0], 0) == [(2, 0.5), (0, 0.5)]
