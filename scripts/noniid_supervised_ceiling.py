"""A real separability ceiling for the non-IID test sets (VERDICT r5 Next #6a).

For each client whose abnormal data ships, on exactly the test set the
federation evaluates (held-out normal + other-device ``test_normal`` rows
(label 0) + every abnormal row (label 1), standardised by the client's
train-split scaler; ``data/prepare.py``, `src/main.py:139-178`): the
out-of-fold ROC-AUC of a SUPERVISED gradient-boosted classifier
(``sklearn`` HistGradientBoostingClassifier, 5-fold stratified
cross-validation on the test set itself, labels visible to it).  A one-class
detector trained on normal rows only -- the autoencoders of the federation --
cannot be expected to beat a classifier that sees both classes of the very
rows it is scored on, so this AUC is a practical upper bound for the
federation's AUC on that client.  (Round 5 cited a 1-nearest-neighbour
one-class detector as a ceiling; 1-NN is no upper bound -- an autoencoder
can beat it -- and is kept below only as a reference point.)

    python scripts/noniid_supervised_ceiling.py --config /root/reference/src/Configuration/scen2-nba-iot-10clients_noniid.json
    python scripts/noniid_supervised_ceiling.py --config /root/reference/src/Configuration/kitsune-iot-10clients_noniid.json --drop 7
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from fedmse_decentralized_amd.config import ExperimentConfig  # noqa: E402
from fedmse_decentralized_amd.eval.metrics import roc_auc  # noqa: E402
from fedmse_decentralized_amd.federation import load_federation_data  # noqa: E402


def derived_config(path: str, drop) -> str:
    """The device list with devices ``drop`` removed (e.g. a client whose
    ``normal/`` training data does not ship) and an absolute data path."""
    d = json.load(open(path))
    d["data_path"] = os.path.normpath(os.path.join(os.path.dirname(path), "..", d["data_path"]))
    if not os.path.isdir(d["data_path"]):
        d["data_path"] = os.path.normpath(os.path.join(os.path.dirname(path), d["data_path"]))
    d["devices_list"] = [x for x in d["devices_list"] if x["id"] not in set(drop)]
    fd, out = tempfile.mkstemp(suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(d, f)
    return out


def supervised_auc(x: np.ndarray, y: np.ndarray, seed: int = 0) -> float:
    from sklearn.ensemble import HistGradientBoostingClassifier
    from sklearn.model_selection import StratifiedKFold

    oof = np.zeros(len(y), dtype=np.float64)
    for tr, te in StratifiedKFold(n_splits=5, shuffle=True, random_state=seed).split(x, y):
        clf = HistGradientBoostingClassifier(max_iter=300, learning_rate=0.1, random_state=seed)
        clf.fit(x[tr], y[tr])
        oof[te] = clf.predict_proba(x[te])[:, 1]
    return float(roc_auc(y, oof))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--drop", type=int, nargs="*", default=[], help="device ids to leave out (no normal data)")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    path = derived_config(args.config, args.drop)
    n = len(json.load(open(path))["devices_list"])
    cfg = ExperimentConfig(config_file=path, network_size=n, log_level="ERROR")
    clients, _ = load_federation_data(cfg, random.Random(cfg.data_seed))
    rows = []
    print("| position | client | test rows (normal / abnormal) | supervised GBDT, 5-fold CV AUC (ceiling) | "
          "1-NN one-class AUC (reference point) |")
    print("|---|---|---|---|---|")
    for i, c in enumerate(clients):
        if c.n_abnormal == 0:
            print(f"| {i} | {c.name} | {int(len(c.test_label))} / 0 | (no abnormal data) | |")
            continue
        y = np.asarray(c.test_label).astype(np.int64)
        x = np.asarray(c.test, dtype=np.float32)
        sup = supervised_auc(x, y)
        tr = torch.tensor(c.train, dtype=torch.float64)
        te = torch.tensor(c.test, dtype=torch.float64)
        nn1 = float(roc_auc(y, torch.cdist(te, tr).min(1).values.numpy()))
        rows.append({"position": i, "client": c.name, "normal": int((y == 0).sum()), "abnormal": int(y.sum()),
                     "supervised_cv_auc": sup, "one_nn_auc": nn1})
        print(f"| {i} | {c.name} | {int((y == 0).sum())} / {int(y.sum())} | {sup:.4f} | {nn1:.4f} |", flush=True)
    if args.json:
        json.dump({"config": args.config, "drop": args.drop, "clients": rows}, open(args.json, "w"), indent=1)
    os.unlink(path)
    return 0


if __name__ == "__main__":
    sys.exit(main())
