"""Per-round detection AUC of one federation (does the 64-client
Kitsune non-IID AUC fall with more rounds, and is it the bench's 20-round
episode reset of the aggregation caps?).

Runs the same federation bench.py runs (synthetic data, compat fixed, no
artefacts) for R rounds and prints one JSON line per round: mean / min
client AUC, aggregator, how many receivers rejected the aggregate, and the
mean number of local epochs the selected clients ran.  ``--episode 0`` never
resets the aggregation caps (the reference's behaviour within one run);
``--episode 20`` resets them every 20 rounds as bench.py does.

  python scripts/auc_trajectory.py --clients 64 --data-kind kitsune --non-iid --rounds 60
  python scripts/auc_trajectory.py --backend torch --device cpu --clients 64 ... --rounds 3
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--clients", type=int, default=64)
    p.add_argument("--rounds", type=int, default=60)
    p.add_argument("--episode", type=int, default=20, help="reset aggregation caps every N rounds (0: never)")
    p.add_argument("--data-kind", default="kitsune", choices=["nbaiot", "kitsune"])
    p.add_argument("--non-iid", action="store_true")
    p.add_argument("--model-type", default="hybrid")
    p.add_argument("--update-type", default="mse_avg")
    p.add_argument("--shrink-lambda", type=float, default=5.0)
    p.add_argument("--backend", default="auto")
    p.add_argument("--device", default=None)
    p.add_argument("--out", default=None)
    a = p.parse_args(argv)

    from fedmse_decentralized_amd.config import ExperimentConfig
    from fedmse_decentralized_amd.federation import Federation
    from fedmse_decentralized_amd.parallel.comm import LoopbackComm
    from fedmse_decentralized_amd.utils.logging import setup_logging

    setup_logging("WARNING")
    cfg = ExperimentConfig(
        num_participants=0.5, epoch=5, num_rounds=a.rounds, lr_rate=1e-3, shrink_lambda=a.shrink_lambda,
        network_size=a.clients, batch_size=12, model_types=[a.model_type], update_types=[a.update_type],
        synthetic=a.data_kind, synthetic_iid=not a.non_iid, compat="fixed", backend=a.backend,
        global_early_stop=False, save_checkpoints=False, output_root=tempfile.mkdtemp(prefix="fedmx_auc_"),
        log_level="WARNING")
    comm = LoopbackComm(a.device) if a.device else None
    fed = Federation(cfg, a.model_type, a.update_type, run=0, comm=comm, write_reports=False).setup()
    out = open(a.out, "w") if a.out else None
    for r in range(a.rounds):
        if a.episode and r and r % a.episode == 0:
            fed.reset_aggregation_counts()
        res = fed.run_round()
        m = np.asarray(res.metrics, dtype=np.float64)
        vr = res.verification or []
        ep = list(res.epochs_run.values()) if isinstance(res.epochs_run, dict) else []
        rec = {"round": r + 1, "auc_mean": round(float(m.mean()), 6), "auc_min": round(float(m.min()), 6),
               "aggregator": res.aggregator,
               "rejected": int(sum(1 for v in vr if not v.get("is_verified", True))),
               "epochs_mean": round(float(np.mean(ep)), 2) if ep else None}
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
    fed.finish()
    if out:
        out.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
