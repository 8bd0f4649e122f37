"""Machine-readable reports, schema- and byte-compatible with the reference.

* Results JSONL, one line per round (`src/main.py:342-355`):
  ``{round, client_metrics[N], update_type, model_type, global_loss}``
  where ``global_loss = min(client_metrics)`` (Q18).
* Verification JSONL (`src/main.py:313-326`, B.2):
  ``{round, verification_results: [{client_id, rejected_updates, is_verified}]}``.
* Training summary JSON, indent 4 (`src/main.py:390-400`, B.3).

Written with ``json.dump`` + ``"\\n"`` exactly like the reference, so files
are byte-identical for identical values.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Sequence


def results_path(cfg, run: int, model_type: str, update_type: str) -> str:
    directory = os.path.join(cfg.checkpoint_dir, f"Run_{run}", cfg.metric)
    return os.path.join(directory, f"{cfg.scen_name}_{cfg.num_participants}_{model_type}_{update_type}_results.json")


def _append_line(path: str, obj, files=None) -> None:
    line = json.dumps(obj) + "\n"   # json.dump(obj, f); f.write("\n") writes these bytes
    if files is not None:
        files.append(path, line.encode())
        return
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "a") as f:
        f.write(line)


def append_round_result(cfg, run: int, rnd: int, metrics: Sequence[float], model_type: str, update_type: str,
                        files=None) -> str:
    path = results_path(cfg, run, model_type, update_type)
    # an undefined metric (NaN: a client with no abnormal test rows) is written
    # as null and left out of global_loss (the reference would write NaN and
    # take an order-dependent min)
    vals = [None if s != s else float(s) for s in metrics]
    defined = [v for v in vals if v is not None]
    _append_line(path, {
        "round": rnd + 1,
        "client_metrics": vals,
        "update_type": update_type,
        "model_type": model_type,
        "global_loss": min(defined) if defined else (float("inf") if not len(metrics) else None),
    }, files)
    return path


def verification_path(cfg, run: int) -> str:
    return os.path.join(cfg.checkpoint_dir, f"Run_{run}", "verification_results.json")


def append_verification(cfg, run: int, rnd: int, results: List[Dict], files=None) -> str:
    path = verification_path(cfg, run)
    _append_line(path, {"round": rnd + 1, "verification_results": results}, files)
    return path


def write_summary(cfg, best_metrics: Dict[str, Dict[str, float]]) -> str:
    path = os.path.join(cfg.checkpoint_dir, "training_summary.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump({
            "best_metrics": best_metrics,
            "metric_type": cfg.metric,
            "num_runs": cfg.num_runs,
            "network_size": cfg.network_size,
            "experiment_name": cfg.experiment_name,
        }, f, indent=4)
    return path
