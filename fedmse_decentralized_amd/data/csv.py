"""Client CSV directories (reference ``load_data``, `src/DataLoader/dataloader.py:22-30`).

Every ``*.csv`` file in a directory is read headerless and concatenated in
(sorted) file-name order.  Parsing is done by the native multi-threaded
reader in ``libfedmx_host.so``; results are cached per process, keyed by
path and mtime, because the reference re-reads every split for every sweep
combination.
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import numpy as np

from ..ops import _host

_CACHE: Dict[Tuple[str, float], np.ndarray] = {}


def load_data(path: str, cache: bool = True) -> np.ndarray:
    if not os.path.isdir(path):
        raise FileNotFoundError(f"data directory not found: {path}")
    files = sorted(f for f in os.listdir(path) if ".csv" in f)
    if not files:
        raise FileNotFoundError(f"no .csv files in {path}")
    parts = []
    for f in files:
        full = os.path.join(path, f)
        key = (os.path.abspath(full), os.path.getmtime(full))
        arr = _CACHE.get(key) if cache else None
        if arr is None:
            arr = _host.read_csv(full)
            if cache:
                _CACHE[key] = arr
        parts.append(arr)
    return parts[0] if len(parts) == 1 else np.concatenate(parts, axis=0)


def clear_cache() -> None:
    _CACHE.clear()
