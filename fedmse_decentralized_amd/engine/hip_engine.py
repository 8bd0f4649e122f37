"""HIP engine: every compute primitive on hand-written gfx950 kernels.

* ``train``        -> ``fedmx_train`` (persistent fused local training, one
                      workgroup per client, all selected clients in one launch)
* ``forward_rows`` -> ``fedmx_forward_rows`` (any list of model x row-block
                      pairs in one launch)
* ``weighted_sum`` -> ``fedmx_weighted_sum``;  ``param_drift`` -> ``fedmx_param_drift``
* ``cen_scores``   -> ``fedmx_cen_score``;     ``auc`` -> ``fedmx_auc``
* ``standardize_ddof1`` -> ``fedmx_standardize_ddof1``

The kernels have no PyTorch fallback: a missing or failing library raises.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

from ..models.layout import segment_ids_padded
from ..ops import _hip, _host
from .base import Engine, TrainHParams, TrainResult


class HipEngine(Engine):
    name = "hip"

    def __init__(self, dims, device):
        super().__init__(dims, device)
        if self.device.type != "cuda":
            raise RuntimeError("HipEngine requires a GPU device")
        _hip.lib()  # load (and fail loudly) up front
        self._seg = segment_ids_padded(dims).to(self.device)

    def train(self, local_ids: Sequence[int], hp: TrainHParams) -> TrainResult:
        tracking, epochs_run, best_epoch, _ = _hip.train(self.store, list(local_ids), hp, self.dims)
        tr = tracking.cpu().numpy()
        er = epochs_run.cpu().numpy().astype(np.int64)
        be = best_epoch.cpu().numpy().astype(np.int64)
        track = [[(float(tr[i, e, 0]), float(tr[i, e, 1])) for e in range(int(er[i]))] for i in range(len(local_ids))]
        return TrainResult(list(local_ids), er, track, be)

    def train_async(self, local_ids: Sequence[int], hp: TrainHParams):
        """Launch without reading results back (bench / overlap)."""
        return _hip.train(self.store, list(local_ids), hp, self.dims)

    def forward_rows(self, params, items, want_sse=True, want_latent=False):
        if not items:
            return [], []
        return _hip.forward_rows(params, items, self.dims, want_sse, want_latent)

    def weighted_sum(self, stack, weights):
        return _hip.weighted_sum(stack, weights)

    def param_drift(self, hist, new):
        return _hip.param_drift(hist, new, self._seg)

    def cen_scores(self, train_lat, test_lat):
        return _hip.cen_scores(train_lat, test_lat, self.dims.latent)

    def auc(self, scores, labels):
        f32_scale = 1.0
        out = _hip.auc(list(scores), list(labels), f32_scale).cpu().numpy()
        for i in np.flatnonzero(out == -1.0):   # class too large for the LDS sort: exact host path
            s = scores[i].detach().double().cpu().numpy()
            out[i] = _host.roc_auc(np.nan_to_num(s), labels[i].cpu().numpy())
        return out

    def standardize_ddof1(self, x):
        return _hip.standardize_ddof1(x.contiguous(), self.dims.d_in)
