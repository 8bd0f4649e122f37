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


# -- the notebook's other preparation steps ------------------------------------

def subsample_rows(n_rows: int, fraction: float, rng: np.random.Generator) -> np.ndarray:
    """Row indices of a per-device random subsample of ``int(fraction * n)``
    rows without replacement — the notebook keeps 5 % of every N-BaIoT
    device's benign rows and 0.5 % of its attack rows
    (`Data-Examination.ipynb:661`, `:670`)."""
    k = int(fraction * n_rows)
    return np.sort(rng.choice(n_rows, size=k, replace=False)) if k > 0 else np.zeros(0, dtype=np.int64)


def holdout_split(n_rows: int, fraction: float, rng: np.random.Generator):
    """(held-out, remaining) row indices: the notebook holds out
    ``int(0.4 * n)`` benign rows as the cross-device ``test_normal`` pool
    before federating the rest (`Data-Examination.ipynb:1271`)."""
    held = np.sort(rng.choice(n_rows, size=int(fraction * n_rows), replace=False))
    rest = np.setdiff1d(np.arange(n_rows), held, assume_unique=True)
    return held, rest


def split_by_balancedness(labels: np.ndarray, n_clients: int, classes_per_client: int, balancedness: float,
                          rng: np.random.Generator, shuffle: bool = True) -> List[np.ndarray]:
    """The notebook's hand-rolled ``split_data`` (`Data-Examination.ipynb:1290`).

    Client sizes: equal when ``balancedness >= 1``; otherwise geometric
    (``balancedness ** i``, normalised, mixed 10 % uniform / 90 % geometric,
    floored, smallest first).  Each client starts at a random class and takes
    up to ``size // classes_per_client`` rows per class, cycling through the
    classes until its budget is spent.  Returns each client's row indices (in
    take order).  Unlike the notebook, a budget that the remaining rows cannot
    cover ends the client's loop instead of spinning forever.
    """
    labels = np.asarray(labels, dtype=np.int64)
    n = labels.shape[0]
    n_labels = int(labels.max()) + 1 if n else 0
    if balancedness >= 1.0:
        per_client = [n // n_clients] * n_clients
        per_class = [per_client[0] // classes_per_client] * n_clients
    else:
        fr = balancedness ** np.linspace(0, n_clients - 1, n_clients)
        fr = fr / fr.sum()
        fr = 0.1 / n_clients + (1 - 0.1) * fr
        per_client = [int(np.floor(f * n)) for f in fr][::-1]
        per_class = [max(1, nd // classes_per_client) for nd in per_client]
    if sum(per_client) > n:
        raise ValueError("impossible split: the client budgets exceed the data")
    pools = [list(np.flatnonzero(labels == c)) for c in range(n_labels)]
    if shuffle:
        for p in pools:
            rng.shuffle(p)
    out = []
    for i in range(n_clients):
        idx: List[int] = []
        budget = per_client[i]
        c = int(rng.integers(n_labels))
        while budget > 0 and any(pools):
            take = min(per_class[i], len(pools[c]), budget)
            idx += pools[c][:take]
            pools[c] = pools[c][take:]
            budget -= take
            c = (c + 1) % n_labels
        out.append(np.asarray(idx, dtype=np.int64))
    return out


def split_fixed_label_percentage(labels: np.ndarray, label_distribution, label_percentage: float = 0.1
                                 ) -> List[np.ndarray]:
    """The notebook's ``split_data_with_fixed_label_percentage``
    (`Data-Examination.ipynb:2226`): client k receives, for each label in
    ``label_distribution[k]``, the first ``floor(count(label) * pct)`` rows of
    that label still unassigned (counts taken over the whole input)."""
    labels = np.asarray(labels)
    uniq, cnt = np.unique(labels, return_counts=True)
    count = dict(zip(uniq.tolist(), cnt.tolist()))
    taken = np.zeros(labels.shape[0], dtype=bool)
    out = []
    for client_labels in label_distribution:
        parts = []
        for lab in client_labels:
            k = int(np.floor(count.get(lab, 0) * label_percentage))
            avail = np.flatnonzero((labels == lab) & ~taken)[:k]
            taken[avail] = True
            parts.append(avail)
        out.append(np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64))
    return out
