"""How separable are the shipped N-BaIoT non-IID CSVs?  (profiles/r5_noniid_vs_reference.md)

For each client whose abnormal data ships, on exactly the test set the
federation evaluates (held-out normal + other-device ``test_normal`` rows
(label 0) + every abnormal row (label 1), standardised by the client's
train-split scaler, `src/main.py:139-178` as data/prepare.py implements it):
the ROC-AUC of two detectors that need no training --
distance to the train mean, and the distance to the nearest training row
(1-NN, a strong non-parametric one-class detector) -- next to the
reference's shipped per-client AUC range (Exp10, every round and run).

    python scripts/noniid_knn_ceiling.py
"""
from __future__ import annotations

import random
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from fedmse_decentralized_amd.config import ExperimentConfig  # noqa: E402
from fedmse_decentralized_amd.eval.metrics import roc_auc  # noqa: E402
from fedmse_decentralized_amd.federation import load_federation_data  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent))
import noniid_vs_reference as nvr  # noqa: E402


def main():
    cfg = ExperimentConfig(config_file=nvr.REF_CFG, network_size=10, log_level="ERROR")
    clients, _ = load_federation_data(cfg, random.Random(cfg.data_seed))
    ref = nvr.load_rounds(nvr.REF_EXP)
    print("| position | client | test rows (normal / abnormal) | mean-distance AUC | 1-NN AUC | reference AUC range (Exp10) |")
    print("|---|---|---|---|---|---|")
    for i, c in enumerate(clients):
        if c.n_abnormal == 0:
            continue
        tr = torch.tensor(c.train, dtype=torch.float64)
        te = torch.tensor(c.test, dtype=torch.float64)
        y = c.test_label
        d_mean = (te - tr.mean(0)).norm(dim=1).numpy()
        d_nn = torch.cdist(te, tr).min(1).values.numpy()
        rv = [row[i] for runs in ref.values() for rr in runs.values() for row in rr]
        print(f"| {i} | {c.name} | {int((y == 0).sum())} / {int(y.sum())} | {roc_auc(y, d_mean):.4f} | "
              f"{roc_auc(y, d_nn):.4f} | {min(rv):.4f}-{max(rv):.4f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
