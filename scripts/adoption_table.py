"""Markdown tables from scripts/adoption_ablation.py records.

  python scripts/adoption_table.py profiles/r4_adoption.jsonl
"""
from __future__ import annotations

import json
import sys
from collections import defaultdict

import numpy as np


def load(path):
    runs = defaultdict(list)
    with open(path) as f:
        for line in f:
            r = json.loads(line)
            runs[(r["clients"], r["iid"], r["mode"], r.get("drift_rel"))].append(r)
    return runs


def summary(runs) -> str:
    out = ["| clients | split | mode | adoption, mean rounds 2-50 | rounds 10-20 with adoption >= 50 % | "
           "AUC round 1 | AUC round 10 | AUC round 50 | AUC mean rounds 41-50 | AUC min round 50 |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    for (n, iid, mode, rel), rs in sorted(runs.items(), key=lambda kv: (kv[0][0], not kv[0][1], kv[0][2],
                                                                          kv[0][3] or 0)):
        rs = sorted(rs, key=lambda r: r["round"])
        ad = np.array([r["adoption"] for r in rs])
        auc = np.array([r["auc_mean"] for r in rs])
        name = mode if mode == "local" else ("aggregate, drift <= 3.0 (reference)" if not rel else
                                             f"aggregate, drift <= {rel} x norm")
        w = [r["adoption"] for r in rs if 10 <= r["round"] <= 20]
        out.append(f"| {n} | {'IID' if iid else 'non-IID'} | {name} | "
                   f"{'-' if mode == 'local' else f'{100 * ad[1:].mean():.1f} %'} | "
                   f"{'-' if mode == 'local' else f'{sum(1 for a in w if a >= 0.5)} / {len(w)}'} | "
                   f"{100 * auc[0]:.2f} | {100 * auc[min(9, len(auc) - 1)]:.2f} | {100 * auc[-1]:.2f} | "
                   f"{100 * auc[-10:].mean():.2f} | {100 * rs[-1]['auc_min']:.2f} |")
    return "\n".join(out)


def health(runs) -> str:
    out = ["| clients | split | mode | round | AUC mean | client 0 latent std (mean over dims) | dead encoder units | "
           "client 0 dev MSE |", "|---|---|---|---|---|---|---|---|"]
    for (n, iid, mode, rel), rs in sorted(runs.items(), key=lambda kv: (kv[0][0], not kv[0][1], kv[0][2],
                                                                          kv[0][3] or 0)):
        if rel or n != 64:
            continue
        for r in sorted(rs, key=lambda r: r["round"]):
            if "c0_z_std_mean" in r and r["round"] in (1, 6, 11, 21, 31, 41, 50):
                out.append(f"| {n} | {'IID' if iid else 'non-IID'} | {mode} | {r['round']} | "
                           f"{100 * r['auc_mean']:.2f} | {r['c0_z_std_mean']:.4f} | {r['c0_dead_h1']} | "
                           f"{r['c0_dev_mse']:.4f} |")
    return "\n".join(out)


def main(argv=None):
    argv = argv or sys.argv[1:]
    runs = load(argv[0])
    print(summary(runs))
    print()
    print(health(runs))
    return 0


if __name__ == "__main__":
    sys.exit(main())
