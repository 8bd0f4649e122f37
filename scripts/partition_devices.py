"""Federate per-device traffic into the reference's client layout — the
pipeline of `Notebook/N-BaIoT/Data-Examination.ipynb`:

  1. per device, a random subsample of its benign rows (5 %) and attack rows
     (0.5 %)  (:661, :670)
  2. 40 % of the benign rows held out as the cross-device ``test_normal``
     pool (:1271)
  3. benign, attack and test_normal rows each split over the clients by
     device label: Dirichlet(alpha) shares (FedArtML ``method="dirichlet"``,
     alpha 1000 ~ IID; :1553, :1988, :2325), or the notebook's hand-rolled
     balancedness splitter (:1290); per-client classes with fewer than
     ``--min-count`` rows dropped (:1839)
  4. written as headerless 115-column CSVs under
     ``Data/Client-k/{normal,abnormal,test_normal}/data.csv`` plus a
     device-list JSON (`src/Configuration/*.json` schema) that
     ``main.py --config-file`` reads.

Devices are given as NAME=BENIGN_GLOB:ATTACK_GLOB (CSV files with a header
row, as the N-BaIoT download ships them):

  python scripts/partition_devices.py --out /data/fed --clients 10 --alpha 1000 \\
      --device Danmini=raw/Danmini/benign_traffic.csv:raw/Danmini/*_attacks/*.csv ...
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fedmse_decentralized_amd.data import partition as P  # noqa: E402


def _read(pattern: str, header: bool) -> np.ndarray:
    import pandas as pd

    files = sorted(glob.glob(pattern))
    if not files:
        raise SystemExit(f"no files match {pattern}")
    parts = [pd.read_csv(f, header=0 if header else None).to_numpy(dtype=np.float64) for f in files]
    return np.concatenate(parts, 0)


def federate(normal, abnormal, n_clients: int, alpha: float, rng: np.random.Generator, normal_frac=0.05,
             abnormal_frac=0.005, holdout=0.4, min_count=10, method="dirichlet", balancedness=1.0,
             classes_per_client=3):
    """normal / abnormal: lists (one per device) of [rows, features] arrays.
    Returns per-client dicts {normal, abnormal, test_normal}."""
    nx, ny, ax, ay = [], [], [], []
    for d, (nr, ar) in enumerate(zip(normal, abnormal)):
        s = P.subsample_rows(nr.shape[0], normal_frac, rng)
        nx.append(nr[s])
        ny.append(np.full(s.size, d))
        s = P.subsample_rows(ar.shape[0], abnormal_frac, rng)
        ax.append(ar[s])
        ay.append(np.full(s.size, d))
    nx, ny, ax, ay = map(np.concatenate, (nx, ny, ax, ay))
    held, rest = P.holdout_split(nx.shape[0], holdout, rng)
    pools = {"normal": (nx[rest], ny[rest]), "abnormal": (ax, ay), "test_normal": (nx[held], ny[held])}
    out = [dict() for _ in range(n_clients)]
    for split, (x, y) in pools.items():
        if method == "dirichlet":
            parts = P.dirichlet_split(y, n_clients, alpha, rng, min_count=min_count)
        else:
            parts = P.split_by_balancedness(y, n_clients, classes_per_client, balancedness, rng)
        for k, idx in enumerate(parts):
            out[k][split] = x[idx]
    return out


def write_clients(out_dir: str, clients, name_prefix: str = "Client", config_name: str = "federated.json") -> str:
    data_dir = os.path.join(out_dir, "Data")
    cfg_dir = os.path.join(out_dir, "Configuration")
    os.makedirs(cfg_dir, exist_ok=True)
    devices = []
    for i, c in enumerate(clients):
        base = f"{name_prefix}-{i + 1}"
        for split in ("normal", "abnormal", "test_normal"):
            d = os.path.join(data_dir, base, split)
            os.makedirs(d, exist_ok=True)
            np.savetxt(os.path.join(d, "data.csv"), c[split], delimiter=",", fmt="%.10g")
        devices.append({"id": i + 1, "name": base, "normal_data_path": f"{base}/normal",
                        "abnormal_data_path": f"{base}/abnormal", "test_normal_data_path": f"{base}/test_normal"})
    path = os.path.join(cfg_dir, config_name)
    with open(path, "w") as f:
        json.dump({"data_path": "Data", "devices_list": devices}, f, indent=4)
    return path


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--device", action="append", required=True, help="NAME=BENIGN_GLOB:ATTACK_GLOB")
    p.add_argument("--out", required=True)
    p.add_argument("--clients", type=int, default=10)
    p.add_argument("--alpha", type=float, default=1000.0, help="Dirichlet concentration (1000 ~ IID)")
    p.add_argument("--method", choices=["dirichlet", "balancedness"], default="dirichlet")
    p.add_argument("--balancedness", type=float, default=1.0)
    p.add_argument("--classes-per-client", type=int, default=3)
    p.add_argument("--normal-frac", type=float, default=0.05)
    p.add_argument("--abnormal-frac", type=float, default=0.005)
    p.add_argument("--holdout", type=float, default=0.4)
    p.add_argument("--min-count", type=int, default=10)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--no-header", action="store_true", help="CSV files have no header row")
    p.add_argument("--config-name", default="federated.json")
    a = p.parse_args(argv)
    normal, abnormal = [], []
    for spec in a.device:
        name, globs = spec.split("=", 1)
        bg, ag = globs.split(":", 1)
        normal.append(_read(bg, not a.no_header))
        abnormal.append(_read(ag, not a.no_header))
        print(f"{name}: {normal[-1].shape[0]} benign, {abnormal[-1].shape[0]} attack rows")
    clients = federate(normal, abnormal, a.clients, a.alpha, np.random.default_rng(a.seed), a.normal_frac,
                       a.abnormal_frac, a.holdout, a.min_count, a.method, a.balancedness, a.classes_per_client)
    path = write_clients(a.out, clients, config_name=a.config_name)
    for i, c in enumerate(clients):
        print(f"Client-{i + 1}: " + ", ".join(f"{k} {v.shape[0]}" for k, v in c.items()))
    print(path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
