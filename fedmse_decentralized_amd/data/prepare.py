"""Per-client split / scaling / test-set assembly (reference `src/main.py:126-223`).

For every client, in device-list order:

1. shuffle the normal rows and the abnormal rows (pandas ``sample(frac=1)`` on
   the global numpy RNG seeded with ``data_seed``, `src/main.py:116-117`,
   `:140-142`; reproduced exactly with a ``RandomState`` permutation);
2. split normal rows ``int(0.4n)`` train / ``int(0.1n)`` valid / ``int(0.4n)``
   dev / rest test (`src/main.py:151-159`);
3. fit a StandardScaler on train, transform valid/test/abnormal
   (`src/main.py:161-165`);
4. with ``new_device`` (default) append the other-device ``test_normal`` rows
   (label 0) to the test set, then all abnormal rows (label 1)
   (`src/main.py:167-178`).

Then the shared dev set: ``min_len`` rows sampled from every client's dev
split, concatenated and standardised by a fresh scaler
(`src/main.py:213-223`).  Everything is float32 at the end (the reference
casts per item in ``IoTDataset.__getitem__``, `src/DataLoader/dataloader.py:73-76`).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from .scaler import IoTDataProcessor
from .synthetic import ClientRaw


@dataclass
class ClientData:
    name: str
    train: np.ndarray          # float32 [n_train, D]
    valid: np.ndarray          # float32 [n_valid, D]
    test: np.ndarray           # float32 [n_test, D]
    test_label: np.ndarray     # int64   [n_test] (1 = abnormal)
    dev_raw: np.ndarray        # float64 [n_dev, D] unscaled dev split (for the shared dev set)
    n_normal: int = 0
    n_abnormal: int = 0
    meta: dict = field(default_factory=dict)


def split_sizes(n: int):
    tr = int(0.4 * n)
    va = int(0.1 * n)
    de = int(0.4 * n)
    te = n - tr - va - de
    return tr, va, de, te


def prepare_client(raw: ClientRaw, rs: np.random.RandomState, new_device: bool = True,
                   scaler: str = "standard") -> ClientData:
    normal = raw.normal[rs.permutation(raw.normal.shape[0])]
    abnormal = raw.abnormal[rs.permutation(raw.abnormal.shape[0])]
    tr, va, de, _ = split_sizes(normal.shape[0])
    train_n = normal[:tr]
    valid_n = normal[tr:tr + va]
    dev_n = normal[tr + va:tr + va + de]
    test_n = normal[tr + va + de:]
    proc = IoTDataProcessor(scaler)
    train, _ = proc.fit_transform(train_n)
    valid, _ = proc.transform(valid_n)
    test, test_lab = proc.transform(test_n)
    abn, abn_lab = proc.transform(abnormal, type="abnormal")
    if new_device:
        newn, newn_lab = proc.transform(raw.test_normal)
        test = np.concatenate([test, newn], 0)
        test_lab = np.concatenate([test_lab, newn_lab], 0)
    test = np.concatenate([test, abn], 0)
    test_lab = np.concatenate([test_lab, abn_lab], 0)
    return ClientData(
        name=raw.name,
        train=train.astype(np.float32), valid=valid.astype(np.float32),
        test=test.astype(np.float32), test_label=test_lab.astype(np.int64),
        dev_raw=dev_n, n_normal=normal.shape[0], n_abnormal=abnormal.shape[0],
    )


def build_dev_set(clients: Sequence[ClientData], rs: np.random.RandomState, scaler: str = "standard") -> np.ndarray:
    min_len = min(c.dev_raw.shape[0] for c in clients)
    parts = []
    for c in clients:
        n = c.dev_raw.shape[0]
        idx = rs.permutation(n)[:min_len]   # DataFrame.sample(n=min_len) without replacement
        parts.append(c.dev_raw[idx])
    dev = np.concatenate(parts, 0)
    proc = IoTDataProcessor(scaler)
    dev_p, _ = proc.fit_transform(dev)
    return dev_p.astype(np.float32)


def prepare_federation(raws: Sequence[ClientRaw], data_seed: int, new_device: bool = True,
                       scaler: str = "standard", rs: Optional[np.random.RandomState] = None):
    """Returns ``(clients, dev_set)`` with the reference numpy-RNG order."""
    if rs is None:
        rs = np.random.RandomState(data_seed)
    clients = [prepare_client(r, rs, new_device, scaler) for r in raws]
    dev = build_dev_set(clients, rs, scaler)
    return clients, dev
