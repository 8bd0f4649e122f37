"""Long-horizon numerical parity of the fused training kernel at the paper's
hyper-parameters (VERDICT r3 Next #3, r4 Next #3).

The paper configuration is 100 local epochs at lr 1e-5 and shrink lambda 10
(`/root/reference/README.md:30-34`); the reference's local loop
(`/root/reference/src/Trainer/client_trainer.py:360-419`) then runs ~5,700
Adam steps per client-round on N-BaIoT-sized clients (~680 training rows,
batch 12; ~1,100 at the thesis's batch 64).  This test runs the whole horizon
in ONE launch of the helper-wave kernel (``fedmx_train_hw.hip``; batch 64 is
its MULTI instantiation: four 16-row chunks per Adam step) and compares it
with the plain-PyTorch oracle (``TorchEngine``: nn-free torch ops with the
reference's op order, itself tested against ``nn.Module`` +
``torch.optim.Adam``), patience disabled so every epoch runs.

Tolerances are the oracle's OWN sensitivity, not fitted numbers.  Client 1 of
this data set is chaotic at these hyper-parameters: its latent codes shrink
to ||z|| ~ 2e-5 on some rows (lambda 10), where the shrink penalty's gradient
lambda z / (B ||z||) keeps unit size but takes its direction from z itself,
i.e. from last-bit noise.  Re-running the oracle from initial parameters
perturbed by 1 ulp moves client 1 by ~6.7e-5 in its final parameters and
~1.5e-4 in its losses, client 0 by ~1e-7 (profiles/r5_long_horizon_sensitivity.md).
So a client that exceeds the fixed floors below is held to ``SENS_FACTOR``
times the divergence the oracle itself shows from a 1-ulp-perturbed copy:
agreement to within the spread any two correct fp32 implementations show.  Identical epochs run / best epoch / Adam step counts
are required exactly.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# floors: per-epoch losses 1e-4 relative; parameters / best snapshot rtol 1e-3
# atol 1e-5; Adam moments rtol 1e-3 atol 1e-6 / 1e-9 (a first moment of a
# near-zero gradient entry is itself tiny)
LOSS_RTOL = 1e-4
TOL = (("params", 1e-3, 1e-5), ("best", 1e-3, 1e-5), ("adam_m", 1e-3, 1e-6), ("adam_v", 1e-3, 1e-9))
SENS_FACTOR = 3.0
# absolute ceilings on the sensitivity-based limits: SENS_FACTOR x
# the largest divergence the CPU oracle showed from its 1-ulp-perturbed copies
# over every perturbation, both clients and all four (mu, batch) cases
# (profiles/r6_long_horizon_sensitivity.json, scripts/long_horizon_sensitivity.py:
# loss 2.06e-4 relative, parameters 1.65e-4, Adam m 2.72e-2, v 7.71e-2 -- the
# chaotic client 1 at FedProx, batch 12), rounded up: a kernel regression of
# chaotic size cannot pass by drawing a wider perturbation
SENS_CEIL = {"loss_rel": 6.5e-4, "params": 5e-4, "best": 5e-4, "adam_m": 8.5e-2, "adam_v": 0.24}


def _clients(seed=3):
    from fedmse_decentralized_amd.data.prepare import prepare_federation
    from fedmse_decentralized_amd.data.synthetic import SyntheticSpec, generate_federation

    raws = generate_federation(SyntheticSpec(kind="nbaiot", n_clients=2, seed=seed))
    clients, _ = prepare_federation(raws, 1234)
    return clients


def _init():
    from fedmse_decentralized_amd.models.reference import init_client_params

    return init_client_params(2, 0)[0]


def _engines(clients, dev, init=None):
    from fedmse_decentralized_amd.engine.hip_engine import HipEngine
    from fedmse_decentralized_amd.engine.torch_engine import TorchEngine
    from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS

    init = _init() if init is None else init
    args = ([c.train for c in clients], [c.valid for c in clients], [c.test for c in clients],
            [c.test_label for c in clients], init)
    ref = TorchEngine(DEFAULT_DIMS, torch.device("cpu"))
    ref.setup(*args)
    hip = None
    if dev is not None:
        hip = HipEngine(DEFAULT_DIMS, dev)
        hip.setup(*args)
    return ref, hip


def _set_anchor(engines, mu):
    if not mu:
        return
    from fedmse_decentralized_amd.models.layout import canonical_to_padded, padded_to_canonical

    base = engines[0].store.params.cpu()
    anchor = base + 0.01 * torch.randn(base.shape, generator=torch.Generator().manual_seed(5))
    anchor = canonical_to_padded(padded_to_canonical(anchor))
    for e in engines:
        e.store.anchor.copy_(anchor.to(e.store.anchor.device))


def _perturbations(hp):
    """1-ulp-scale perturbations of the oracle's run: initial parameters x (1
    +- 2^-23) and x (1 +- 2^-20) under random sign patterns (the divergence
    of a chaotic trajectory is event-like -- a latent row crossing ||z|| = 0 --
    so any one perturbation may or may not set it off; measured on the CPU,
    client 1 either stays within ~1e-6 or moves by the same saturated
    ~6.7e-5 (plain) / ~1.6e-4 (FedProx))."""
    init = _init()
    for mag in (2.0 ** -23, 2.0 ** -20):
        for seed in (1, 2, 3, 4):
            sign = torch.randint(0, 2, init.shape, generator=torch.Generator().manual_seed(seed)) * 2 - 1
            yield init * (1 + sign * mag)


def _diffs(r_a, a, r_b, b):
    """Per client: max relative per-epoch loss difference and the max absolute
    difference of every compared tensor between two runs."""
    out = {}
    for c in range(2):
        x, y = np.array(r_a.tracking[c]), np.array(r_b.tracking[c])
        d = {"loss_rel": float(np.max(np.abs(x - y) / np.abs(x)))}
        for name, _, _ in TOL:
            d[name] = float((getattr(a.store, name)[c].cpu().double() - getattr(b.store, name)[c].cpu().double())
                            .abs().max())
        out[c] = d
    return out


def _violations(r1, ref, r2, hip, sens):
    bad = []
    for c in range(2):
        a, b = np.array(r1.tracking[c]), np.array(r2.tracking[c])
        rel = float(np.max(np.abs(b - a) / np.abs(a)))
        lim = max(LOSS_RTOL, min(SENS_FACTOR * sens[c]["loss_rel"], SENS_CEIL["loss_rel"]))
        if rel > lim:
            bad.append(f"client {c} losses rel {rel:.3g} > {lim:.3g}")
        for name, rtol, atol in TOL:
            x = getattr(hip.store, name)[c].cpu().double()
            y = getattr(ref.store, name)[c].double()
            d = (x - y).abs()
            lim_abs = max(atol, min(SENS_FACTOR * sens[c][name], SENS_CEIL[name]))
            over = d > (lim_abs + rtol * y.abs())
            if bool(over.any()):
                bad.append(f"client {c} {name}: {int(over.sum())} entries beyond atol {lim_abs:.3g} + rtol {rtol} "
                           f"(max abs diff {float(d.max()):.3g})")
    return bad


def _compare(r1, r2, ref, hip, clients, hp, report=None):
    """Kernel (r2, hip) against the oracle (r1, ref): exact epochs / best
    epoch / step counts; losses and tensors within the fixed floors, or, if a
    client exceeds them, within SENS_FACTOR x the largest divergence of the
    oracle from 1-ulp-perturbed copies of itself (every one of
    _perturbations, always the whole set, and recorded), capped by
    SENS_CEIL."""
    stats = {"epochs_run": [list(map(int, r1.epochs_run)), list(map(int, r2.epochs_run))],
             "best_epoch": [list(map(int, r1.best_epoch)), list(map(int, r2.best_epoch))],
             "kernel_vs_oracle": _diffs(r1, ref, r2, hip)}
    zero = {c: {"loss_rel": 0.0, **{name: 0.0 for name, _, _ in TOL}} for c in range(2)}
    sens, tried = zero, 0
    bad = _violations(r1, ref, r2, hip, sens)
    per_pert = []
    if bad:
        for p_init in _perturbations(hp):
            p, _ = _engines(clients, None, p_init)
            _set_anchor([p], hp.fedprox_mu)
            r_p = p.train([0, 1], hp)
            tried += 1
            d = _diffs(r1, ref, r_p, p)
            per_pert.append(d)
            sens = {c: {k: max(sens[c][k], d[c][k]) for k in sens[c]} for c in range(2)}
        bad = _violations(r1, ref, r2, hip, sens)
    stats.update(oracle_sensitivity=sens, perturbations_tried=tried, per_perturbation=per_pert)
    print("long-horizon stats", json.dumps(stats), flush=True)   # on record even when an assertion fails
    if report is not None:
        report.update(stats)
    assert list(r1.epochs_run) == list(r2.epochs_run)
    assert list(r1.best_epoch) == list(r2.best_epoch)
    assert torch.equal(hip.store.adam_step.cpu(), ref.store.adam_step)
    assert not bad, bad
    return stats


def _run_case(dev, mu, batch):
    from fedmse_decentralized_amd.engine.base import TrainHParams

    clients = _clients()
    ref, hip = _engines(clients, dev)
    _set_anchor([ref, hip], mu)
    hp = TrainHParams(epochs=100, batch_size=batch, lr=1e-5, shrink_lambda=10.0, fedprox_mu=mu, patience=10 ** 6)
    r1 = ref.train([0, 1], hp)
    r2 = hip.train([0, 1], hp)
    assert list(r2.epochs_run) == [100, 100]
    n0 = int(ref.store.train_off[1] - ref.store.train_off[0])
    assert int(hip.store.adam_step[0]) == 100 * ((n0 + batch - 1) // batch)
    return _compare(r1, r2, ref, hip, clients, hp)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("batch", [12, 64], ids=["b12", "b64"])
@pytest.mark.parametrize("mu", [0.0, 0.001], ids=["fedmse-sae", "fedprox"])
def test_paper_config_100_epochs_matches_torch_oracle(mu, batch):
    """Batch 12 (the code default, compact one-chunk step) and batch 64 (the
    thesis's GPU runs, SURVEY §5.6: the MULTI instantiation, four 16-row
    chunks per Adam step with the weight gradients accumulated over them)."""
    stats = _run_case(torch.device("cuda", 0), mu, batch)
    print("long-horizon", f"mu={mu} batch={batch}", json.dumps(stats))


_CHILD = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
from test_long_horizon_gpu import _run_case
from fedmse_decentralized_amd.ops import _hip
st = _run_case(torch.device("cuda", 0), 0.0, 12)
st["lib"] = _hip.lib_path()
print(json.dumps(st))
"""


@pytest.mark.timeout(600)
def test_exact_adam_build_matches_torch_oracle():
    """The IEEE-division Adam build (-DFEDMX_EXACT_ADAM=1: torch's rounding
    sequence, unscaled moments; ``libfedmx_hip_exact.so``) over the same
    horizon, in a child process that loads that library, to the same
    sensitivity-derived tolerances as the default build."""
    from fedmse_decentralized_amd.ops import build

    # rebuilt here when its content hash (sources, flags, compiler) is stale,
    # so an edited kernel source is never tested through an old library
    lib = build.build_hip(extra_flags=["-DFEDMX_EXACT_ADAM=1"], target=build.HIP_EXACT_LIB)
    env = dict(os.environ, FEDMX_HIP_LIB=str(lib))
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=env, capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    st = json.loads(r.stdout.strip().splitlines()[-1])
    assert st["lib"].endswith("libfedmx_hip_exact.so")
    print("exact-adam long-horizon", json.dumps(st))
