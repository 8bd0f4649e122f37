"""Batched evaluation of many clients (reference ``Evaluator.evaluate``,
`src/Evaluator/evaluator.py:50-127`).

The reference evaluates the N clients one after another, 12 rows per
forward, and moves every score/latent to the host for sklearn/scipy.  Here
all hosted clients are evaluated with a handful of launches:

* ``autoencoder``: one ``forward_rows`` over every client's test set
  (per-row SSE); anomaly score = SSE / D (``MSELoss(reduction='none')
  .mean(1)``); AUC on the device.
* ``hybrid`` (SAE-CEN): one ``forward_rows`` returning latents for every
  client's train and test sets; CEN scaler + distance and AUC on the device
  (`src/Model/Centroid.py:15-35`).

``metric="classification"`` returns F1 at threshold 0.5 (plus P/R),
``metric="time"`` the wall time of the scoring pass (the reference's
``"time"`` branch is broken).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .metrics import classification_metrics


@dataclass
class EvalResult:
    metrics: np.ndarray                       # [k] per evaluated client
    extra: Dict[str, np.ndarray] = field(default_factory=dict)
    latents: Optional[List[Tuple[np.ndarray, np.ndarray]]] = None  # (test_latent, labels) per client


def evaluate_clients(engine, local_ids: Sequence[int], model_type: str, metric: str = "AUC",
                     keep_latents: bool = False) -> EvalResult:
    st = engine.store
    D = engine.dims.d_in
    t0 = time.perf_counter()
    if model_type == "autoencoder":
        items = [(c, st.rows("test", c)) for c in local_ids]
        sse, _ = engine.forward_rows(st.params, items, want_sse=True, want_latent=False)
        scores = [s / D for s in sse]
        test_lat = None
    elif model_type == "hybrid":
        items = []
        for c in local_ids:
            items.append((c, st.rows("train", c)))
            items.append((c, st.rows("test", c)))
        _, lat = engine.forward_rows(st.params, items, want_sse=False, want_latent=True)
        tr = lat[0::2]
        test_lat = lat[1::2]
        scores = engine.cen_scores(tr, test_lat)
    else:
        raise ValueError(f"unknown model_type {model_type!r}")
    labels = [st.test_label[int(st.test_off[c]):int(st.test_off[c + 1])] for c in local_ids]
    extra = {}
    if metric == "AUC":
        vals = engine.auc(scores, labels)
    elif metric == "classification":
        f1s, ps, rs = [], [], []
        for s, c in zip(scores, local_ids):
            f1, p, r = classification_metrics(st.labels(c), s.detach().cpu().numpy())
            f1s.append(f1)
            ps.append(p)
            rs.append(r)
        vals = np.asarray(f1s)
        extra = {"precision": np.asarray(ps), "recall": np.asarray(rs)}
    elif metric == "time":
        engine.synchronize()
        vals = np.full(len(local_ids), time.perf_counter() - t0)
    else:
        raise ValueError(f"unknown metric {metric!r}")
    latents = None
    if keep_latents and test_lat is not None:
        latents = [(l.detach().cpu().numpy().astype(np.float32), st.labels(c).astype(np.float32))
                   for l, c in zip(test_lat, local_ids)]
    return EvalResult(np.asarray(vals, dtype=np.float64), extra, latents)
