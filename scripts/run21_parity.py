"""Replay of the reference's shipped run (`src/run21.log`) on its own data.

`src/run21.log` is the only measured run the reference ships: Kitsune IID-10
(`Data/Kitsune-Network-Attack-Dataset/Client_Data_IID`), 10 clients, 50 %
participation, 3 rounds x 5 local epochs, lr 1e-3, shrink lambda 5, batch 12,
data seed 1234, 6 model x update combinations, CPU-only laptop (banner at
`src/run21.log:9-25`).  This script runs the same sweep
through ``main.run_sweep`` (``--compat reference`` replays the reference's RNG
consumption, so client selection, elections and verification follow the
reference's trajectory), then parses the log's per-client AUC lines
("AUC for ...", 10 per round) and prints, per combination and round, our
AUCs against the log's.

    python scripts/run21_parity.py [--data-root DIR] [--backend torch|hip] [--compat reference|fixed]
                                   [--out FILE.jsonl]

DIR defaults to the reference checkout's Kitsune IID directory.  The log is
read as UTF-16 text (nothing in it is executed).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

REF = "/root/reference"
LOG = os.path.join(REF, "src/run21.log")
DATA = os.path.join(REF, "Data/Kitsune-Network-Attack-Dataset/Client_Data_IID")
COMBOS = [("hybrid", "avg"), ("hybrid", "fedprox"), ("hybrid", "mse_avg"),
          ("autoencoder", "avg"), ("autoencoder", "fedprox"), ("autoencoder", "mse_avg")]


def parse_log(path: str, clients: int = 10):
    """Per combination: the log's groups of 10 per-client AUC lines (one per
    evaluation, in order) and its 'Best AUC' summary."""
    with open(path, "rb") as f:
        text = f.read().decode("utf-16")
    parts = re.split(r"Starting combination \d+/\d+", text)[1:]
    if len(parts) != len(COMBOS):
        raise ValueError(f"{path}: {len(parts)} combinations, expected {len(COMBOS)}")
    groups = []
    for part in parts:
        a = [float(m) for m in re.findall(r"AUC for [^:]+: ([0-9.eE+-]+)", part)]
        groups.append(np.asarray(a[: len(a) // clients * clients]).reshape(-1, clients))
    best = {f"{m} + {u}": float(v) for m, u, v in re.findall(r"(\w+) \+ (\w+): Best AUC = ([0-9.]+)", text)}
    return groups, best


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--data-root", default=DATA)
    p.add_argument("--log", default=LOG)
    p.add_argument("--backend", default="torch")
    p.add_argument("--compat", default="reference")
    p.add_argument("--out", default=None)
    args = p.parse_args()

    import torch

    import main as driver
    from fedmse_decentralized_amd.config import ExperimentConfig
    from fedmse_decentralized_amd.utils.logging import setup_logging

    setup_logging("WARNING")
    ref_aucs, ref_best = parse_log(args.log)
    out = tempfile.mkdtemp(prefix="fedmx_run21_")
    # the reference's Kitsune device list (src/Configuration/kitsune-iot-10clients_noniid.json
    # layout), pointed at the IID split run21 used
    dl = {"data_path": os.path.abspath(args.data_root), "devices_list": [
        {"id": i, "name": f"Kitsune-Client-{i}", "normal_data_path": f"Client-{i}/normal",
         "abnormal_data_path": f"Client-{i}/abnormal", "test_normal_data_path": f"Client-{i}/test_normal"}
        for i in range(1, 11)]}
    cfg_path = os.path.join(out, "kitsune_iid10.json")
    with open(cfg_path, "w") as f:
        json.dump(dl, f)
    device = "cuda" if args.backend == "hip" and torch.cuda.is_available() else "cpu"
    cfg = ExperimentConfig(config_file=cfg_path, network_size=10, num_participants=0.5, epoch=5, num_rounds=3,
                           lr_rate=1e-3, shrink_lambda=5, batch_size=12, data_seed=1234, num_runs=1,
                           model_types=["hybrid", "autoencoder"], update_types=["avg", "fedprox", "mse_avg"],
                           backend=args.backend, device=device, compat=args.compat, save_checkpoints=False,
                           output_root=out, log_level="WARNING")
    t0 = time.perf_counter()
    best = driver.run_sweep(cfg)
    wall = time.perf_counter() - t0
    from fedmse_decentralized_amd.io import reports

    lines = []
    for ci, (m, u) in enumerate(COMBOS):
        path = reports.results_path(cfg, 0, m, u)
        ours = [json.loads(s)["client_metrics"] for s in open(path) if s.strip()]
        for r, row in enumerate(ours):
            ref = ref_aucs[ci][r] if r < ref_aucs[ci].shape[0] else None
            rec = {"model": m, "update": u, "round": r + 1,
                   "ours_mean": round(float(np.mean(row)), 6),
                   "ref_mean": round(float(np.mean(ref)), 6) if ref is not None else None,
                   "max_abs_diff": round(float(np.max(np.abs(np.asarray(row) - ref))), 6) if ref is not None else None}
            lines.append(rec)
            print(json.dumps(rec), flush=True)
        key = f"{m} + {u}"
        rec = {"model": m, "update": u, "ours_rounds": len(ours), "ref_evaluations": int(ref_aucs[ci].shape[0]),
               "ours_best": round(best[m][u], 10), "ref_best": ref_best.get(key)}
        lines.append(rec)
        print(json.dumps(rec), flush=True)
    summary = {"backend": args.backend, "compat": args.compat, "sweep_wall_s": round(wall, 2),
               "ref_log": os.path.relpath(args.log, REF) if args.log.startswith(REF) else args.log}
    print(json.dumps(summary), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            for r in lines + [summary]:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
