"""Federated partitioning utilities.

Re-implements what the data-preparation notebook does with FedArtML
(`Notebook/N-BaIoT/Data-Examination.ipynb:1553-1555`, `:1988-1990`):
a Dirichlet(alpha) split of class-labelled rows across clients
(alpha=1000 ~ IID, small alpha ~ label-skewed non-IID), followed by the
per-client rare-class filter (classes with fewer than ``min_count`` rows
dropped, `:1839`).  Also the Jensen-Shannon distance between client label
distributions that the notebook reports as its heterogeneity measure
(`:2634`, `:2706`).
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np


def dirichlet_proportions(n_clients: int, n_classes: int, alpha: float, rng: np.random.Generator) -> np.ndarray:
    """[n_clients, n_classes] mixture weights, each row sums to 1."""
    p = rng.dirichlet(np.full(n_classes, float(alpha)), size=n_clients)
    return p


def dirichlet_split(labels: np.ndarray, n_clients: int, alpha: float, rng: np.random.Generator,
                    min_count: int = 0) -> List[np.ndarray]:
    """Split row indices by class with per-class Dirichlet(alpha) client shares."""
    labels = np.asarray(labels)
    classes = np.unique(labels)
    buckets: List[list] = [[] for _ in range(n_clients)]
    for c in classes:
        idx = np.flatnonzero(labels == c)
        rng.shuffle(idx)
        share = rng.dirichlet(np.full(n_clients, float(alpha)))
        cuts = (np.cumsum(share)[:-1] * len(idx)).astype(np.int64)
        for k, part in enumerate(np.split(idx, cuts)):
            buckets[k].append(part)
    out = []
    for k in range(n_clients):
        idx = np.concatenate(buckets[k]) if buckets[k] else np.zeros(0, dtype=np.int64)
        if min_count > 0 and idx.size:
            lab = labels[idx]
            keep = np.ones(idx.size, dtype=bool)
            for c in np.unique(lab):
                m = lab == c
                if m.sum() < min_count:
                    keep &= ~m
            idx = idx[keep]
        out.append(np.sort(idx))
    return out


def js_distance(p: np.ndarray, q: np.ndarray, base: Optional[float] = 2.0) -> float:
    """Jensen-Shannon distance between two discrete distributions (scipy semantics)."""
    p = np.asarray(p, dtype=np.float64)
    q = np.asarray(q, dtype=np.float64)
    p = p / p.sum()
    q = q / q.sum()
    m = 0.5 * (p + q)

    def _kl(a, b):
        mask = a > 0
        return float(np.sum(a[mask] * np.log(a[mask] / b[mask])))

    js = 0.5 * _kl(p, m) + 0.5 * _kl(q, m)
    if base is not None:
        js /= np.log(base)
    return float(np.sqrt(max(js, 0.0)))


def federation_heterogeneity(proportions: np.ndarray) -> float:
    """Mean pairwise JS distance between client class distributions."""
    n = proportions.shape[0]
    if n < 2:
        return 0.0
    d = [js_distance(proportions[i], proportions[j]) for i in range(n) for j in range(i + 1, n)]
    return float(np.mean(d))
