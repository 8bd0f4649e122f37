"""Asynchronous validation of the helper-wave training kernel (one validator
workgroup per client beside the trainers, fedmx_train_hw.hip) against the
same kernel's synchronous epoch-end validation (``async_valid=False``):
bit-identical parameters, Adam state and step counts, best snapshots,
per-epoch train / valid losses, epochs run and best epochs -- including the
roll-back of a trainer that its validator stops after it has run ahead,
mid-epoch (epochs longer than AV_CHECK = 6 steps), at the odd tail step of an
epoch of exactly AV_CHECK + 1 steps, or at the epoch's end (shorter epochs),
and over two launches (persistent state, fresh launch numbers on the same
workspace).  The many-client cases (64 and 128 selected clients: grids of 128
and 256 workgroups, so trainer / validator pairs span every XCD pair) run
three launches each with the evaluation kernels of another federation
enqueued concurrently on a side stream, as the round loop does.  The FedProx and batch > 12 instantiations
keep the synchronous path (the asynchronous one spills registers in their
step loops); their cases check that it is the one that ran."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from fedmse_decentralized_amd.engine.base import TrainHParams
from fedmse_decentralized_amd.models.layout import canonical_to_padded, padded_to_canonical
from fedmse_decentralized_amd.ops import _hip

DEV = torch.device("cuda", 0)
STATE = ("params", "best", "adam_m", "adam_v", "adam_step")


def _pair(n_train, n_valid, seed):
    from test_kernels_gpu import _setup_pair   # (tests/ is on sys.path under pytest)

    _, a = _setup_pair(n_train=n_train, n_valid=n_valid, seed=seed)
    _, b = _setup_pair(n_train=n_train, n_valid=n_valid, seed=seed)
    anchor = a.store.params + 0.01 * torch.randn(a.store.params.shape, generator=torch.Generator().manual_seed(9),
                                                 device="cpu").to(DEV)
    anchor = canonical_to_padded(padded_to_canonical(anchor.cpu())).to(DEV)
    a.store.anchor.copy_(anchor)
    b.store.anchor.copy_(anchor)
    return a, b


# batch, lam, mu, lr, train rows of the two clients, epochs, patience, early stop expected
CASES = [
    (12, 5.0, 0.0, 3e-2, (301, 150), 8, 1, True),     # 26 / 13 steps: the stop lands mid-epoch
    (12, 1.0, 1e-3, 3e-2, (301, 150), 8, 1, True),    # FedProx: the synchronous path
    (64, 5.0, 0.0, 3e-2, (601, 300), 8, 1, True),     # batch 64 (16-row chunks): the synchronous path
    (12, 5.0, 0.0, 3e-2, (40, 30), 8, 1, True),       # 4 / 3 steps: decisions at the epoch's end
    (12, 5.0, 0.0, 3e-2, (80, 75), 8, 1, True),       # 7 steps (AV_CHECK + 1): the ping-pong loop's odd tail check
    (12, 5.0, 0.0, 1e-3, (301, 150), 4, 10 ** 6, False),   # no early stop: every epoch published
]


@pytest.mark.parametrize("batch,lam,mu,lr,n_train,epochs,patience,stops", CASES)
def test_async_validation_matches_synchronous(batch, lam, mu, lr, n_train, epochs, patience, stops):
    a, b = _pair(n_train, (70, 33), seed=21)
    hp = TrainHParams(epochs=epochs, batch_size=batch, lr=lr, shrink_lambda=lam, fedprox_mu=mu, patience=patience)
    ran = []
    for _ in range(2):
        ta, ea, ba = _hip.train(a.store, [0, 1], hp, a.dims, helper=True, async_valid=True)
        grid = _hip.lib().fedmx_train_hw_last_grid()
        tb, eb, bb = _hip.train(b.store, [0, 1], hp, b.dims, helper=True, async_valid=False)
        torch.cuda.synchronize()
        _hip.runtime(DEV).sync()
        # (FedProx and batch > 12 keep the synchronous epoch tail: FEDMX_HW_ASYNC_VALID = 1)
        assert grid == (4 if batch <= 12 and mu == 0 else 2), "validator workgroups where expected, and only there"
        assert _hip.lib().fedmx_train_hw_last_grid() == 2
        assert list(ea) == list(eb) and list(ba) == list(bb)
        assert min(ea) >= 1, "a launch reported failure"
        np.testing.assert_array_equal(np.array(ta), np.array(tb))   # (NaN where an epoch did not run)
        for name in STATE:
            assert torch.equal(getattr(a.store, name), getattr(b.store, name)), name
        ran += list(ea)
    if stops:
        assert min(ran) < epochs, f"no client stopped early ({ran}): the roll-back path was not exercised"
    else:
        assert ran == [epochs] * 4


def _many(k, seed):
    """Two HipEngines (and a third for the side-stream evaluation) on the
    same k clients of assorted sizes (35..300 training rows)."""
    from fedmse_decentralized_amd.engine.hip_engine import HipEngine
    from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS
    from fedmse_decentralized_amd.models.reference import init_client_params

    rng = np.random.default_rng(seed)
    n_tr = rng.integers(35, 300, size=k)
    n_va = rng.integers(9, 80, size=k)
    tr = [rng.normal(size=(int(n), 115)).astype(np.float32) for n in n_tr]
    va = [rng.normal(size=(int(n), 115)).astype(np.float32) for n in n_va]
    te = [rng.normal(size=(20, 115)).astype(np.float32) for _ in range(k)]
    lab = [np.r_[np.zeros(10), np.ones(10)].astype(np.int64) for _ in range(k)]
    init, _ = init_client_params(k, seed)
    engs = []
    for _ in range(3):
        e = HipEngine(DEFAULT_DIMS, DEV)
        e.setup(tr, va, te, lab, init)
        engs.append(e)
    return engs


@pytest.mark.parametrize("k", [64, 128])
def test_async_validation_many_clients_side_stream(k):
    """VERDICT r5 Next #2a: bit-identity of asynchronous and synchronous
    validation at 64 / 128 selected clients, 3 launches, with side-stream
    evaluation kernels competing for the CUs."""
    a, b, c = _many(k, seed=31 + k)
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    if 2 * k > cus:
        pytest.skip(f"{2 * k} workgroups do not fit {cus} CUs")
    side = torch.cuda.Stream(DEV)
    hp = TrainHParams(epochs=6, batch_size=12, lr=3e-2, shrink_lambda=5.0, patience=1)
    ids = list(range(k))
    ran = []
    for _ in range(3):
        with _hip.on_stream(side):
            c.evaluate_launch("hybrid")   # (results unused: CU competition only)
        ta, ea, ba = _hip.train(a.store, ids, hp, a.dims, helper=True, async_valid=True)
        grid = _hip.lib().fedmx_train_hw_last_grid()
        with _hip.on_stream(side):
            c.evaluate_launch("hybrid")
        tb, eb, bb = _hip.train(b.store, ids, hp, b.dims, helper=True, async_valid=False)
        torch.cuda.synchronize()
        _hip.runtime(DEV).sync()
        assert grid == 2 * k, "validator workgroups expected"
        assert min(ea) >= 1, f"a launch reported failure: {list(ea)}"
        assert list(ea) == list(eb) and list(ba) == list(bb)
        np.testing.assert_array_equal(np.array(ta), np.array(tb))
        for name in STATE:
            assert torch.equal(getattr(a.store, name), getattr(b.store, name)), name
        ran += list(ea)
    assert min(ran) < hp.epochs, "no client stopped early: the roll-back path was not exercised"
