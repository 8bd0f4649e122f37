"""Paper-headline configuration on the reference's own N-BaIoT IID-10 CSVs.

FedMSE paper setting (README of the reference): 10 gateways, 50 %
participation, 20 rounds x 100 local epochs, lr 1e-5, shrink lambda 10; every
model x update combination of the paper's IID table
(`src/Visualization/results_visualization.ipynb:29-50`: mean AUC over the
gateways).  Prints one JSON line per combination: mean / std / min / max of
the final round's per-client AUCs and the combination's wall clock.

    python scripts/real_data_paper.py --data-root DIR [--backend hip|torch] [--compat fixed|reference]

DIR holds ``Client-k/{normal,abnormal,test_normal}/*.csv`` (the reference's
``Data/N-BaIoT/IID-10-Client_Data``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

PAPER_IID = {  # mean AUC %, results_visualization.ipynb:33-50
    ("autoencoder", "avg"): 99.07, ("autoencoder", "fedprox"): 98.95, ("autoencoder", "mse_avg"): 98.92,
    ("hybrid", "avg"): 98.76, ("hybrid", "fedprox"): 98.53, ("hybrid", "mse_avg"): 99.01,
}
# SAE-CEN + MSEAvg against the client ratio, IID (results_visualization.ipynb:325-346)
PAPER_RATIO_IID = {0.5: 99.01, 0.6: 98.96, 0.7: 98.44, 0.8: 98.71, 0.9: 98.60, 1.0: 98.69}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--data-root", required=True)
    p.add_argument("--backend", default="auto")
    p.add_argument("--compat", default="fixed")
    p.add_argument("--rounds", type=int, default=20)
    p.add_argument("--epochs", type=int, default=100)
    p.add_argument("--combos", default="all", help="e.g. hybrid:mse_avg,autoencoder:avg")
    p.add_argument("--participation", type=float, nargs="+", default=[0.5],
                   help="client ratio sweep (paper table: 0.5 .. 1.0)")
    args = p.parse_args()

    import torch

    from fedmse_decentralized_amd.config import ExperimentConfig
    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.utils.logging import setup_logging

    setup_logging("WARNING")
    clients = sorted((d for d in os.listdir(args.data_root) if d.startswith("Client-")),
                     key=lambda s: int(s.split("-")[1]))
    cfg_json = {"data_path": os.path.abspath(args.data_root), "devices_list": [
        {"id": i + 1, "name": f"NBa-Scen2-{c}", "normal_data_path": f"{c}/normal",
         "abnormal_data_path": f"{c}/abnormal", "test_normal_data_path": f"{c}/test_normal"}
        for i, c in enumerate(clients)]}
    out = tempfile.mkdtemp(prefix="fedmx_paper_")
    cfg_path = os.path.join(out, "nbaiot_iid10.json")
    with open(cfg_path, "w") as f:
        json.dump(cfg_json, f)
    device = "cuda" if torch.cuda.is_available() and args.backend != "torch" else "cpu"
    combos = list(PAPER_IID) if args.combos == "all" else [tuple(c.split(":")) for c in args.combos.split(",")]
    todo = [(mt, ut, part) for mt, ut in combos for part in args.participation]
    for model_type, update_type, part in todo:
        cfg = ExperimentConfig(config_file=cfg_path, network_size=len(clients), num_participants=part,
                               epoch=args.epochs, num_rounds=args.rounds, lr_rate=1e-5, shrink_lambda=10,
                               model_types=[model_type], update_types=[update_type], backend=args.backend,
                               device=device, compat=args.compat, global_early_stop=False,
                               save_checkpoints=True, output_root=out, log_level="WARNING")
        t0 = time.perf_counter()
        fed = Federation(cfg, model_type, update_type, 0).setup()
        best = fed.run_all()
        if device == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        m = np.asarray(fed.last_metrics, dtype=np.float64)
        print(json.dumps({
            "model": model_type, "update": update_type, "participation": part, "backend": fed.engine.name,
            "compat": args.compat,
            "rounds": fed.round_idx, "final_auc_mean_pct": round(100 * float(m.mean()), 3),
            "final_auc_std_pct": round(100 * float(m.std()), 3), "final_auc_min_pct": round(100 * float(m.min()), 3),
            "best_auc_pct": round(100 * best, 3),
            "paper_iid_mean_pct": (PAPER_IID.get((model_type, update_type)) if part == 0.5 else
                                   PAPER_RATIO_IID.get(part) if (model_type, update_type) == ("hybrid", "mse_avg")
                                   else None),
            "wall_s": round(dt, 2)}), flush=True)


if __name__ == "__main__":
    main()
