"""The torch engine (the oracle for the HIP kernels) reproduces the reference's
local training loop exactly: ``ClientTrainer.run`` with an ``nn.Module`` model,
``torch.optim.Adam`` created once, FedProx term, patience early stop
(`src/Trainer/client_trainer.py:360-419`)."""
import copy

import numpy as np
import torch

from fedmse_decentralized_amd.engine.base import TrainHParams
from fedmse_decentralized_amd.engine.torch_engine import TorchEngine
from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS, canonical_to_state_dict, state_dict_to_canonical
from fedmse_decentralized_amd.models.reference import ReferenceSAE, init_client_params


def _reference_run(model, optimizer, prev_global, x_train, x_valid, epochs, B, mu, patience):
    """Literal transcription of the reference loop semantics (DataLoader
    batching without shuffle; loss.item() accumulation in python floats)."""
    min_valid = float("inf")
    worse = 0
    tracking = []
    best = None
    for ep in range(epochs):
        model.train()
        epoch_loss = 0.0
        nb = 0
        for s in range(0, len(x_train), B):
            _, _, loss = model(x_train[s:s + B])
            if mu:
                prox = 0.0
                for p, gp in zip(model.parameters(), prev_global.parameters()):
                    prox += torch.sum(torch.square(p - gp))
                loss += mu * prox
            loss.backward()
            optimizer.step()
            optimizer.zero_grad()
            epoch_loss += loss.item()
            nb += 1
        epoch_loss /= nb
        model.eval()
        vl = 0.0
        nvb = 0
        with torch.no_grad():
            for s in range(0, len(x_valid), B):
                _, _, loss = model(x_valid[s:s + B])
                if mu:
                    prox = 0.0
                    for p, gp in zip(model.parameters(), prev_global.parameters()):
                        prox += torch.sum(torch.square(p - gp))
                    loss += mu * prox
                vl += loss.item()
                nvb += 1
        vl /= nvb
        tracking.append((epoch_loss, vl))
        if vl < min_valid:
            min_valid = vl
            best = copy.deepcopy(model.state_dict())
            worse = 0
        else:
            worse += 1
            if worse >= patience:
                break
    return tracking, best


def _run_pair(lam, mu, rounds=2, epochs=4):
    rng = np.random.default_rng(0)
    xt = rng.normal(size=(50, 115)).astype(np.float32)
    xv = rng.normal(size=(15, 115)).astype(np.float32)
    init, _ = init_client_params(1, 3)
    eng = TorchEngine(DEFAULT_DIMS, torch.device("cpu"))
    eng.setup([xt], [xv], [xv], [np.zeros(15, dtype=np.int64)], init)
    model = ReferenceSAE(DEFAULT_DIMS, shrink_lambda=lam)
    model.load_state_dict(canonical_to_state_dict(init[0]))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    prev = copy.deepcopy(model)
    hp = TrainHParams(epochs=epochs, batch_size=12, lr=1e-3, shrink_lambda=lam, fedprox_mu=mu, patience=1)
    for _ in range(rounds):
        res = eng.train([0], hp)
        trk, best = _reference_run(model, opt, prev, torch.from_numpy(xt), torch.from_numpy(xv), epochs, 12, mu, 1)
        assert res.tracking[0] == trk
        ours = eng.canonical(eng.store.params[0])
        assert torch.equal(ours, state_dict_to_canonical(model.state_dict()))
        assert torch.equal(eng.canonical(eng.store.best[0]), state_dict_to_canonical(best))
    return eng


def test_sae_training_bit_exact_vs_reference_loop():
    _run_pair(lam=5.0, mu=0.0)


def test_ae_training_bit_exact():
    _run_pair(lam=0.0, mu=0.0)


def test_fedprox_training_bit_exact():
    _run_pair(lam=5.0, mu=0.001)


def test_adam_state_persists_across_rounds():
    eng = _run_pair(lam=1.0, mu=0.0, rounds=2, epochs=2)
    assert int(eng.store.adam_step[0]) > 0
