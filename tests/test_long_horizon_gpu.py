"""Long-horizon numerical parity of the fused training kernel at the paper's
hyper-parameters (VERDICT r3 Next #3).

The paper configuration is 100 local epochs at lr 1e-5 and shrink lambda 10
(`/root/reference/README.md:30-34`); the reference's local loop
(`/root/reference/src/Trainer/client_trainer.py:360-419`) then runs ~5,700
Adam steps per client-round on N-BaIoT-sized clients (~680 training rows,
batch 12).  The short GPU tests stop at 3 epochs; this one runs the whole
horizon in ONE launch of the helper-wave kernel (``fedmx_train_hw.hip``) and
compares it with the plain-PyTorch oracle (``TorchEngine``: nn-free torch
ops with the reference's op order, itself tested against ``nn.Module`` +
``torch.optim.Adam``), patience disabled so every epoch runs.

Agreement required: identical epochs run and best epoch, per-epoch train /
validation losses within 1e-4 relative, final parameters within rtol 1e-3
(atol 1e-5), Adam moments within rtol 1e-3 (atol 1e-6 / 1e-9).  The kernel's default Adam uses the
hardware square root / reciprocal (<= 1 ulp each); the IEEE build
(``-DFEDMX_EXACT_ADAM=1``, torch's rounding sequence with IEEE square root /
division) is exercised by ``test_exact_adam_build_matches_torch_oracle`` in a
child process that loads that library variant; it does NOT end closer to the
oracle: client 1's trajectory at these hyper-parameters is sensitive to the
last bit of the update (the two builds end 3.9e-5 apart in its parameters,
each deterministic run to run), and the default build happens to track the
oracle more closely (3e-8).
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


def _clients(seed=3):
    from fedmse_decentralized_amd.data.prepare import prepare_federation
    from fedmse_decentralized_amd.data.synthetic import SyntheticSpec, generate_federation

    raws = generate_federation(SyntheticSpec(kind="nbaiot", n_clients=2, seed=seed))
    clients, _ = prepare_federation(raws, 1234)
    return clients


def _engines(clients, dev):
    from fedmse_decentralized_amd.engine.hip_engine import HipEngine
    from fedmse_decentralized_amd.engine.torch_engine import TorchEngine
    from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS
    from fedmse_decentralized_amd.models.reference import init_client_params

    init, _ = init_client_params(2, 0)
    args = ([c.train for c in clients], [c.valid for c in clients], [c.test for c in clients],
            [c.test_label for c in clients], init)
    ref = TorchEngine(DEFAULT_DIMS, torch.device("cpu"))
    ref.setup(*args)
    hip = HipEngine(DEFAULT_DIMS, dev)
    hip.setup(*args)
    return ref, hip


# (Adam's first moment of a near-zero gradient entry is itself tiny: 3 of
# 18,432 entries differed by ~3e-7 absolute after 5,700 steps, so its
# absolute floor is 1e-6; the parameters are held to rtol 1e-3 / atol 1e-5)
TOL = (("params", 1e-3, 1e-5), ("best", 1e-3, 1e-5), ("adam_m", 1e-3, 1e-6), ("adam_v", 1e-3, 1e-9))


def _compare(r1, r2, ref, hip, report=None):
    stats = {"epochs_run": [list(map(int, r1.epochs_run)), list(map(int, r2.epochs_run))],
             "best_epoch": [list(map(int, r1.best_epoch)), list(map(int, r2.best_epoch))]}
    for i, (a, b) in enumerate(zip(r1.tracking, r2.tracking)):
        a, b = np.array(a), np.array(b)
        stats[f"loss_rel_max_c{i}"] = float(np.max(np.abs(b - a) / np.abs(a)))
    for name, _, _ in TOL:
        x, y = getattr(hip.store, name).cpu().double(), getattr(ref.store, name).double()
        stats[f"{name}_abs_max"] = float((x - y).abs().max())
        stats[f"{name}_rel_max"] = float(((x - y).abs() / y.abs().clamp_min(1e-30)).max())
    print("long-horizon stats", json.dumps(stats), flush=True)   # on record even when an assertion fails
    if report is not None:
        report.update(stats)
    assert list(r1.epochs_run) == list(r2.epochs_run)
    assert list(r1.best_epoch) == list(r2.best_epoch)
    for a, b in zip(r1.tracking, r2.tracking):
        np.testing.assert_allclose(np.array(b), np.array(a), rtol=1e-4, atol=0)
    for name, rtol, atol in TOL:
        torch.testing.assert_close(getattr(hip.store, name).cpu().double(), getattr(ref.store, name).double(),
                                   rtol=rtol, atol=atol)
    assert torch.equal(hip.store.adam_step.cpu(), ref.store.adam_step)
    return stats


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mu", [0.0, 0.001], ids=["fedmse-sae", "fedprox"])
def test_paper_config_100_epochs_matches_torch_oracle(mu):
    from fedmse_decentralized_amd.engine.base import TrainHParams

    dev = torch.device("cuda", 0)
    ref, hip = _engines(_clients(), dev)
    if mu:
        anchor = ref.store.params + 0.01 * torch.randn(ref.store.params.shape,
                                                       generator=torch.Generator().manual_seed(5))
        from fedmse_decentralized_amd.models.layout import canonical_to_padded, padded_to_canonical

        anchor = canonical_to_padded(padded_to_canonical(anchor))
        ref.store.anchor.copy_(anchor)
        hip.store.anchor.copy_(anchor.to(dev))
    hp = TrainHParams(epochs=100, batch_size=12, lr=1e-5, shrink_lambda=10.0, fedprox_mu=mu, patience=10 ** 6)
    r1 = ref.train([0, 1], hp)
    r2 = hip.train([0, 1], hp)
    assert list(r2.epochs_run) == [100, 100]
    assert int(hip.store.adam_step[0]) == 100 * ((ref.store.train_off[1] - ref.store.train_off[0] + 11) // 12)
    stats = _compare(r1, r2, ref, hip)
    print("long-horizon", json.dumps(stats))


def _compare_exact(r1, r2, ref, hip, report):
    """The IEEE-Adam build: client 0 to the default build's tolerances; client 1,
    whose trajectory is the sensitive one at these hyper-parameters (the
    IEEE and the default builds themselves end 3.9e-5 apart in its
    parameters, each run deterministic: profiles/r4_train_hw_experiments.md),
    to 5e-4 in the losses and 2e-4 absolute in the parameters."""
    assert list(r1.epochs_run) == list(r2.epochs_run)
    assert list(r1.best_epoch) == list(r2.best_epoch)
    loss_tol = (1e-4, 5e-4)
    par_atol = (1e-5, 2e-4)
    for c in range(2):
        a, b = np.array(r1.tracking[c]), np.array(r2.tracking[c])
        rel = float(np.max(np.abs(b - a) / np.abs(a)))
        x = hip.store.params[c].cpu().double()
        y = ref.store.params[c].double()
        d = float((x - y).abs().max())
        report[f"c{c}"] = {"loss_rel_max": rel, "params_abs_max": d}
        assert rel <= loss_tol[c], (c, rel)
        assert d <= par_atol[c], (c, d)
    assert torch.equal(hip.store.adam_step.cpu(), ref.store.adam_step)


_CHILD = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
from test_long_horizon_gpu import _clients, _engines, _compare_exact
from fedmse_decentralized_amd.engine.base import TrainHParams
from fedmse_decentralized_amd.ops import _hip
ref, hip = _engines(_clients(), torch.device("cuda", 0))
hp = TrainHParams(epochs=100, batch_size=12, lr=1e-5, shrink_lambda=10.0, patience=10 ** 6)
r1 = ref.train([0, 1], hp)
r2 = hip.train([0, 1], hp)
st = {}
_compare_exact(r1, r2, ref, hip, st)
st["lib"] = _hip.lib_path()
print(json.dumps(st))
"""


@pytest.mark.timeout(600)
def test_exact_adam_build_matches_torch_oracle():
    """The IEEE-division Adam build (-DFEDMX_EXACT_ADAM=1, built by
    ``__graft_entry__.build()`` as ``libfedmx_hip_exact.so``) over the same
    100-epoch horizon, in a child process that loads that library
    (tolerances: ``_compare_exact``)."""
    from fedmse_decentralized_amd.ops import build

    lib = build.HIP_EXACT_LIB
    assert lib.exists(), f"{lib} missing: run __graft_entry__.build()"
    env = dict(os.environ, FEDMX_HIP_LIB=str(lib))
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=env, capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    st = json.loads(r.stdout.strip().splitlines()[-1])
    assert st["lib"].endswith("libfedmx_hip_exact.so")
    print("exact-adam long-horizon", json.dumps(st))
