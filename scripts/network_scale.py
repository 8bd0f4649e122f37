"""Detection AUC against federation size and participation (the reference's
network-scale and client-ratio tables).

The reference publishes SAE-CEN + MSEAvg (FedMSE) AUC at 10/20/30/40/50
clients and at 50-100 % participation, IID and non-IID
(`src/Visualization/results_visualization.ipynb:427-448`, `:529-550`,
`:223-244`, `:325-346`).  This script runs one federation per
(clients, participation, IID/non-IID) point on synthetic N-BaIoT-shaped data
and prints one JSON line per point: the final round's mean / min client AUC,
the mean over the last 10 rounds, the best round, and rounds/s.

  python scripts/network_scale.py --clients 10 20 40 50 80 256 --rounds 50 --out profiles/x.jsonl
  python scripts/network_scale.py --clients 10 --participation 0.5 0.6 0.7 0.8 0.9 1.0 --rounds 20
  python scripts/network_scale.py --backend torch --device cpu --clients 10 20 --rounds 50   # CPU oracle
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_point(n: int, part: float, iid: bool, a) -> dict:
    from fedmse_decentralized_amd.config import ExperimentConfig
    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.parallel.comm import LoopbackComm

    cfg = ExperimentConfig(
        num_participants=part, epoch=a.epochs, num_rounds=a.rounds, lr_rate=a.lr, shrink_lambda=a.shrink_lambda,
        network_size=n, batch_size=12, model_types=[a.model_type], update_types=[a.update_type],
        synthetic=a.data_kind, synthetic_iid=iid, compat=a.compat, backend=a.backend, init_mode=a.init_mode,
        global_early_stop=False, save_checkpoints=False, output_root=tempfile.mkdtemp(prefix="fedmx_scale_"),
        log_level="WARNING")
    comm = LoopbackComm(a.device) if a.device else None
    fed = Federation(cfg, a.model_type, a.update_type, run=0, comm=comm, write_reports=False).setup()
    t0 = time.perf_counter()
    res = [fed.run_round() for _ in range(a.rounds)]
    fed.finish()
    dt = time.perf_counter() - t0
    means = np.array([float(np.mean(r.metrics)) for r in res])
    last = np.asarray(res[-1].metrics, dtype=np.float64)
    rej = [sum(1 for v in (r.verification or []) if not v.get("is_verified", True)) for r in res]
    return {"clients": n, "participation": part, "iid": iid, "rounds": a.rounds, "backend": fed.engine.name,
            "init_mode": cfg.resolved_init_mode(), "compat": a.compat,
            "auc_mean_final": round(float(last.mean()), 5), "auc_min_final": round(float(last.min()), 5),
            "auc_mean_last10": round(float(means[-10:].mean()), 5),
            "auc_mean_best_round": round(float(means.max()), 5), "best_round": int(means.argmax()) + 1,
            "rejected_last10_mean": round(float(np.mean(rej[-10:])), 2),
            "rounds_per_sec": round(a.rounds / dt, 2)}


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--clients", type=int, nargs="+", default=[10, 20, 30, 40, 50])
    p.add_argument("--participation", type=float, nargs="+", default=[0.5])
    p.add_argument("--split", choices=["iid", "noniid", "both"], default="both")
    p.add_argument("--rounds", type=int, default=50)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--shrink-lambda", type=float, default=5.0)
    p.add_argument("--data-kind", default="nbaiot", choices=["nbaiot", "kitsune"])
    p.add_argument("--model-type", default="hybrid")
    p.add_argument("--update-type", default="mse_avg")
    p.add_argument("--compat", default="fixed")
    p.add_argument("--init-mode", default="auto")
    p.add_argument("--backend", default="auto")
    p.add_argument("--device", default=None)
    p.add_argument("--out", default=None)
    a = p.parse_args(argv)
    from fedmse_decentralized_amd.utils.logging import setup_logging

    setup_logging("ERROR")
    splits = {"iid": [True], "noniid": [False], "both": [True, False]}[a.split]
    out = open(a.out, "a") if a.out else None
    for iid in splits:
        for n in a.clients:
            for part in a.participation:
                rec = run_point(n, part, iid, a)
                line = json.dumps(rec)
                print(line, flush=True)
                if out:
                    out.write(line + "\n")
                    out.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
