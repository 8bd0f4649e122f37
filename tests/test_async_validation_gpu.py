"""Asynchronous validation of the helper-wave training kernel (one validator
workgroup per client beside the trainers, fedmx_train_hw.hip) against the
same kernel's synchronous epoch-end validation (``async_valid=False``):
bit-identical parameters, Adam state and step counts, best snapshots,
per-epoch train / valid losses, epochs run and best epochs -- including the
roll-back of a trainer that its validator stops after it has run ahead,
mid-epoch (epochs longer than AV_CHECK = 4 steps) or at the epoch's end
(shorter epochs), and over two launches (persistent state, fresh launch
numbers on the same workspace).  The FedProx and batch > 12 instantiations
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
