"""Results tables from the per-round report files (the tabular half of the
reference's `src/Visualization/results_visualization.ipynb`; the
figures are `scripts/plots.py`).

Reads every ``*_results.json`` (one JSON line per round:
``{round, client_metrics, update_type, model_type, global_loss}``) under a
results directory — ours or the reference's shipped
`src/Checkpoint/Results/Update/**` — and prints, per combination, the
per-round mean / min / max client metric and the final-round summary, next to
the FedMSE paper's published averages when the
combination has one.

    python scripts/results_table.py Checkpoint/Results/Update/10
    python scripts/results_table.py /root/reference/src/Checkpoint/Results/Update/10 --per-round
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys

import numpy as np

# FedMSE paper, 10 gateways, 50 % participation, mean AUC %
PAPER_IID = {("autoencoder", "avg"): 99.07, ("autoencoder", "fedprox"): 98.95, ("autoencoder", "mse_avg"): 98.92,
             ("hybrid", "avg"): 98.76, ("hybrid", "fedprox"): 98.53, ("hybrid", "mse_avg"): 99.01}
PAPER_NONIID = {("autoencoder", "avg"): 94.74, ("autoencoder", "fedprox"): 93.98, ("autoencoder", "mse_avg"): 92.87,
                ("hybrid", "avg"): 96.93, ("hybrid", "fedprox"): 97.28, ("hybrid", "mse_avg"): 97.30}


def load_results(root: str):
    out = {}
    for path in sorted(glob.glob(os.path.join(root, "**", "*_results.json"), recursive=True)):
        rows = []
        with open(path) as f:
            for line in f:
                line = line.strip()
                if line:
                    rows.append(json.loads(line))
        rows = [r for r in rows if "client_metrics" in r]   # (not verification_results.json)
        if rows:
            out[path] = rows
    return out


def _vals(row) -> np.ndarray:
    """A round's client metrics; null (a client without abnormal test rows) -> NaN, left out of the stats."""
    return np.asarray([np.nan if v is None else v for v in row["client_metrics"]], dtype=np.float64)


def table(results, per_round: bool = False) -> str:
    lines = ["| file | model | update | rounds | final mean | final min | final max | best round mean | paper IID | paper non-IID |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    detail = []
    for path, rows in results.items():
        mt, ut = rows[-1].get("model_type", "?"), rows[-1].get("update_type", "?")
        means = [float(np.nanmean(_vals(r))) for r in rows]
        last = _vals(rows[-1])
        rel = os.path.relpath(path)
        lines.append(f"| `{rel}` | {mt} | {ut} | {len(rows)} | {np.nanmean(last):.4f} | {np.nanmin(last):.4f} | {np.nanmax(last):.4f} | "
                     f"{max(means):.4f} | {PAPER_IID.get((mt, ut), '')} | {PAPER_NONIID.get((mt, ut), '')} |")
        if per_round:
            detail += ["", f"### {rel}", "", "| round | mean | min | max |", "|---|---|---|---|"]
            for r in rows:
                m = _vals(r)
                detail.append(f"| {r['round']} | {np.nanmean(m):.4f} | {np.nanmin(m):.4f} | {np.nanmax(m):.4f} |")
    return "\n".join(lines + detail) + "\n"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--per-round", action="store_true")
    a = ap.parse_args(argv)
    res = load_results(a.root)
    if not res:
        print(f"no *_results.json under {a.root}", file=sys.stderr)
        return 1
    sys.stdout.write(table(res, a.per_round))
    return 0


if __name__ == "__main__":
    sys.exit(main())
