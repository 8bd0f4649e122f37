"""Packed parameter layouts for the 4-layer (Shrink-)Autoencoder.

The reference model is ``Linear(in,27)-ReLU-Linear(27,7)`` (encoder) and
``Linear(7,27)-ReLU-Linear(27,out)`` (decoder)
(`src/Model/Shrink_Autoencoder.py:40-42`, `:95-97`).  Its state dict holds
eight tensors in this order::

    encoder.encoder_network.0.weight [H, D]   encoder.encoder_network.0.bias [H]
    encoder.encoder_network.2.weight [Z, H]   encoder.encoder_network.2.bias [Z]
    decoder.decoder_network.0.weight [H, Z]   decoder.decoder_network.0.bias [H]
    decoder.decoder_network.2.weight [D, H]   decoder.decoder_network.2.bias [D]

Two flat layouts are used by the framework:

* **canonical** – the eight tensors concatenated in state-dict order
  (6,764 floats for D=115, H=27, Z=7).  This is the exchange format for
  checkpoints and reports.
* **padded** ("kernel") – four *bias-augmented* matrices with MFMA-friendly
  power-of-two shapes.  The bias of every layer lives in the last padded
  column of its weight matrix and the activation feeding that layer carries
  a constant 1 in that column, so ``y = W_aug @ [x; 1]``.  This lets the
  fused HIP kernels treat bias gradients as one more column of the weight
  gradient (one Adam code path, no separate column-sum reductions)::

        W1a [HP=32][DP=128]   W1a[h][DP-1] = b1[h]
        W2a [ZP=16][HP=32]    W2a[z][HP-1] = b2[z]
        W3a [HP=32][ZP=16]    W3a[h][ZP-1] = b3[h]
        W4a [DP=128][HP=32]   W4a[d][HP-1] = b4[d]

  Everything outside the real weight/bias positions is exactly zero and stays
  zero under training (gradients there are masked to zero).  Total
  ``P_PAD = 9216`` floats (36,864 B) per client; the device-resident client
  state (params, Adam m/v, FedProx anchor, best snapshot) and the RCCL
  all-gather payload all use this layout.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache
from typing import Dict, List, Tuple

import torch

DP = 128  # padded input/output width (D <= DP-1: last column holds the bias "1")
HP = 32   # padded hidden width      (H <= HP-1)
ZP = 16   # padded latent width      (Z <= ZP-1)

OFF_W1 = 0
OFF_W2 = OFF_W1 + HP * DP
OFF_W3 = OFF_W2 + ZP * HP
OFF_W4 = OFF_W3 + HP * ZP
P_PAD = OFF_W4 + DP * HP  # 9216

STATE_KEYS = (
    "encoder.encoder_network.0.weight",
    "encoder.encoder_network.0.bias",
    "encoder.encoder_network.2.weight",
    "encoder.encoder_network.2.bias",
    "decoder.decoder_network.0.weight",
    "decoder.decoder_network.0.bias",
    "decoder.decoder_network.2.weight",
    "decoder.decoder_network.2.bias",
)


@dataclass(frozen=True)
class ModelDims:
    """Logical model dimensions (reference defaults: 115/27/7)."""

    d_in: int = 115
    hidden: int = 27
    latent: int = 7

    def __post_init__(self):
        if not (1 <= self.d_in <= DP - 1):
            raise ValueError(f"d_in must be in [1, {DP - 1}], got {self.d_in}")
        if not (1 <= self.hidden <= HP - 1):
            raise ValueError(f"hidden must be in [1, {HP - 1}], got {self.hidden}")
        if not (1 <= self.latent <= ZP - 1):
            raise ValueError(f"latent must be in [1, {ZP - 1}], got {self.latent}")

    # -- canonical layout -------------------------------------------------
    def shapes(self) -> List[Tuple[str, Tuple[int, ...]]]:
        D, H, Z = self.d_in, self.hidden, self.latent
        return [
            (STATE_KEYS[0], (H, D)), (STATE_KEYS[1], (H,)),
            (STATE_KEYS[2], (Z, H)), (STATE_KEYS[3], (Z,)),
            (STATE_KEYS[4], (H, Z)), (STATE_KEYS[5], (H,)),
            (STATE_KEYS[6], (D, H)), (STATE_KEYS[7], (D,)),
        ]

    @property
    def num_params(self) -> int:
        n = 0
        for _, s in self.shapes():
            k = 1
            for v in s:
                k *= v
            n += k
        return n


DEFAULT_DIMS = ModelDims()


@lru_cache(maxsize=16)
def padded_index(dims: ModelDims) -> Tuple[torch.Tensor, List[Tuple[int, int]]]:
    """Gather index mapping canonical flat position -> padded flat position.

    Returns ``(idx, segments)`` where ``idx[j]`` is the padded offset of
    canonical element ``j`` and ``segments[t] = (start, end)`` are the
    canonical ranges of the eight state-dict tensors (used for per-tensor
    norms, e.g. the verifier's parameter drift,
    `src/Trainer/model_verifier.py:79-84`).
    """
    D, H, Z = dims.d_in, dims.hidden, dims.latent
    parts = []
    # W1 [H, D] -> W1a[h][d]
    h = torch.arange(H).view(H, 1)
    d = torch.arange(D).view(1, D)
    parts.append((OFF_W1 + h * DP + d).reshape(-1))
    parts.append(OFF_W1 + torch.arange(H) * DP + (DP - 1))           # b1
    z = torch.arange(Z).view(Z, 1)
    hh = torch.arange(H).view(1, H)
    parts.append((OFF_W2 + z * HP + hh).reshape(-1))                  # W2 [Z, H]
    parts.append(OFF_W2 + torch.arange(Z) * HP + (HP - 1))           # b2
    h2 = torch.arange(H).view(H, 1)
    z2 = torch.arange(Z).view(1, Z)
    parts.append((OFF_W3 + h2 * ZP + z2).reshape(-1))                 # W3 [H, Z]
    parts.append(OFF_W3 + torch.arange(H) * ZP + (ZP - 1))           # b3
    d2 = torch.arange(D).view(D, 1)
    h3 = torch.arange(H).view(1, H)
    parts.append((OFF_W4 + d2 * HP + h3).reshape(-1))                 # W4 [D, H]
    parts.append(OFF_W4 + torch.arange(D) * HP + (HP - 1))           # b4
    segments = []
    start = 0
    for p in parts:
        segments.append((start, start + p.numel()))
        start += p.numel()
    idx = torch.cat(parts).to(torch.int64)
    assert idx.numel() == dims.num_params
    return idx, segments


def segment_ids_padded(dims: ModelDims) -> torch.Tensor:
    """int32 [P_PAD]: state-dict tensor id (0..7) of each padded slot, -1 for padding."""
    idx, segs = padded_index(dims)
    out = torch.full((P_PAD,), -1, dtype=torch.int32)
    for t, (a, b) in enumerate(segs):
        out[idx[a:b]] = t
    return out


def canonical_to_padded(flat: torch.Tensor, dims: ModelDims = DEFAULT_DIMS) -> torch.Tensor:
    """[..., num_params] -> [..., P_PAD] (zeros elsewhere)."""
    idx, _ = padded_index(dims)
    idx = idx.to(flat.device)
    out = flat.new_zeros(flat.shape[:-1] + (P_PAD,))
    out[..., idx] = flat
    return out


def padded_to_canonical(padded: torch.Tensor, dims: ModelDims = DEFAULT_DIMS) -> torch.Tensor:
    idx, _ = padded_index(dims)
    return padded.index_select(-1, idx.to(padded.device))


def state_dict_to_canonical(state: Dict[str, torch.Tensor], dims: ModelDims = DEFAULT_DIMS) -> torch.Tensor:
    return torch.cat([state[k].detach().reshape(-1).to(torch.float32).cpu() for k, _ in dims.shapes()])


def canonical_to_state_dict(flat: torch.Tensor, dims: ModelDims = DEFAULT_DIMS) -> "Dict[str, torch.Tensor]":
    from collections import OrderedDict

    out = OrderedDict()
    off = 0
    for k, s in dims.shapes():
        n = 1
        for v in s:
            n *= v
        out[k] = flat[off:off + n].reshape(s).clone()
        off += n
    return out


def padded_views(p: torch.Tensor):
    """Views (W1a, W2a, W3a, W4a) of one padded parameter vector [P_PAD]."""
    return (
        p[OFF_W1:OFF_W2].view(HP, DP),
        p[OFF_W2:OFF_W3].view(ZP, HP),
        p[OFF_W3:OFF_W4].view(HP, ZP),
        p[OFF_W4:P_PAD].view(DP, HP),
    )


def real_mask_padded(dims: ModelDims = DEFAULT_DIMS) -> torch.Tensor:
    """bool [P_PAD]: True at real (weight or bias) positions."""
    return segment_ids_padded(dims) >= 0
