"""Execution engines (see ``engine/base.py``)."""
from __future__ import annotations

import torch

from .base import ClientStore, Engine, TrainHParams, TrainResult
from .torch_engine import TorchEngine


def make_engine(backend: str, dims, device) -> Engine:
    device = torch.device(device)
    if backend == "auto":
        backend = "hip" if device.type == "cuda" else "torch"
    if backend == "torch":
        return TorchEngine(dims, device)
    if backend == "hip":
        if device.type != "cuda":
            raise RuntimeError("the hip backend needs a GPU device")
        from .hip_engine import HipEngine

        return HipEngine(dims, device)
    raise ValueError(f"unknown backend {backend!r}")


__all__ = ["ClientStore", "Engine", "TrainHParams", "TrainResult", "TorchEngine", "make_engine"]
