"""Pure-PyTorch reference implementation of the (Shrink-)Autoencoder.

This is the numerical oracle for the fused HIP kernels and the execution
path of the ``torch`` engine (CPU tests, parity runs).  It reproduces the
reference model exactly:

* module tree and state-dict keys (`src/Model/Shrink_Autoencoder.py:21-116`,
  duplicate `src/Model/AutoEncoder.py:21-116`);
* initialisation order: ``nn.Linear`` default init first (consumes the torch
  RNG), then ``U(-1/sqrt(fan_in), 1/sqrt(fan_in))`` weights and zero biases
  (`src/Model/Shrink_Autoencoder.py:47-59`);
* loss ``MSE(x, y) + lambda * sum_b ||z_b||_2 / B``
  (`src/Model/Shrink_Autoencoder.py:152-153`); the AE uses ``lambda = 0``
  (`src/Model/AutoEncoder.py:148`).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import math
import threading

import torch
from torch import nn

from .layout import ModelDims, DEFAULT_DIMS, state_dict_to_canonical


class _Encoder(nn.Module):
    def __init__(self, d_in: int, hidden: int, latent: int):
        super().__init__()
        self.encoder_network = nn.Sequential(
            nn.Linear(d_in, hidden, bias=True), nn.ReLU(), nn.Linear(hidden, latent, bias=True))
        _reference_reinit(self)

    def forward(self, x):
        return self.encoder_network(x)


class _Decoder(nn.Module):
    def __init__(self, latent: int, hidden: int, d_out: int):
        super().__init__()
        self.decoder_network = nn.Sequential(
            nn.Linear(latent, hidden, bias=True), nn.ReLU(), nn.Linear(hidden, d_out, bias=True))
        _reference_reinit(self)

    def forward(self, z):
        return self.decoder_network(z)


def _reference_reinit(module: nn.Module) -> None:
    # Overwrite nn.Linear's default init: W ~ U(+-1/sqrt(fan_in)), b = 0.
    for layer in module.modules():
        if isinstance(layer, nn.Linear):
            bound = 1.0 / math.sqrt(layer.in_features)
            layer.weight.data.uniform_(-bound, bound)
            layer.bias.data.zero_()


class ReferenceSAE(nn.Module):
    """Shrink autoencoder (``shrink_lambda > 0``) or plain AE (``shrink_lambda = 0``).

    ``forward(x) -> (latent, output, loss)`` like the reference.
    """

    def __init__(self, dims: ModelDims = DEFAULT_DIMS, shrink_lambda: float = 10.0):
        super().__init__()
        self.dims = dims
        self.encoder = _Encoder(dims.d_in, dims.hidden, dims.latent)
        self.decoder = _Decoder(dims.latent, dims.hidden, dims.d_in)
        self.shrink_lambda = float(shrink_lambda)

    def loss(self, x, y, z):
        mse = nn.functional.mse_loss(y, x, reduction="mean")
        if self.shrink_lambda == 0.0:
            return mse
        return mse + self.shrink_lambda * (torch.sum(torch.linalg.vector_norm(z, dim=1)) / z.shape[0])

    def forward(self, x):
        z = self.encoder(x)
        y = self.decoder(z)
        return z, y, self.loss(x, y, z)


def init_client_params(num_clients: int, seed: int, dims: ModelDims = DEFAULT_DIMS
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Initial canonical parameters of ``num_clients`` models, built in the
    reference order from a torch RNG seeded with ``seed``
    (``set_seeds(run*10000)`` at `src/main.py:115`, models built at
    `src/main.py:230-236`).

    Returns ``(params [C, num_params], rng_state_after)`` — the CPU generator
    state after all inits, used by the compat RNG replay
    (`utils/rng_replay.py`).
    """
    out = []
    with GLOBAL_RNG_LOCK, torch.random.fork_rng(devices=[]):
        # the CPU generator only (torch.manual_seed would also seed every GPU
        # generator: ~18 ms per call once CUDA is up, and the inits never
        # draw from them)
        torch.random.default_generator.manual_seed(seed)
        for _ in range(num_clients):
            m = ReferenceSAE(dims, shrink_lambda=0.0)
            out.append(state_dict_to_canonical(m.state_dict(), dims))
        state = torch.get_rng_state()
    return torch.stack(out, 0), state


# the global torch CPU generator is process state: serialise the code paths
# that borrow it (in-process multi-rank tests run ranks on threads)
GLOBAL_RNG_LOCK = threading.RLock()


# ----------------------------------------------------------------------------
# Functional forms on canonical parameter vectors (used by the torch engine).
# ----------------------------------------------------------------------------

def unflatten(flat: torch.Tensor, dims: ModelDims = DEFAULT_DIMS) -> List[torch.Tensor]:
    out = []
    off = 0
    for _, s in dims.shapes():
        n = 1
        for v in s:
            n *= v
        out.append(flat[off:off + n].view(s))
        off += n
    return out


def functional_forward(tensors: List[torch.Tensor], x: torch.Tensor):
    w1, b1, w2, b2, w3, b3, w4, b4 = tensors
    h1 = torch.relu(nn.functional.linear(x, w1, b1))
    z = nn.functional.linear(h1, w2, b2)
    h3 = torch.relu(nn.functional.linear(z, w3, b3))
    y = nn.functional.linear(h3, w4, b4)
    return z, y


def functional_loss(x, y, z, shrink_lambda: float):
    mse = nn.functional.mse_loss(y, x, reduction="mean")
    if shrink_lambda == 0.0:
        return mse
    return mse + shrink_lambda * (torch.sum(torch.linalg.vector_norm(z, dim=1)) / z.shape[0])


def rowwise_sse(flat: torch.Tensor, x: torch.Tensor, dims: ModelDims = DEFAULT_DIMS,
                chunk: Optional[int] = None):
    """Per-row sum of squared reconstruction error and latents (no grad)."""
    with torch.no_grad():
        t = unflatten(flat, dims)
        z, y = functional_forward(t, x)
        return ((y - x) ** 2).sum(dim=1), z
