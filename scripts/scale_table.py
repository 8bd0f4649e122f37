"""Markdown tables of scripts/network_scale.py records against the reference's
published SAE-CEN + MSEAvg (FedMSE) AUCs.

  python scripts/scale_table.py profiles/r3_network_scale_hip.jsonl [more.jsonl ...]

Published values (%, FedMSE paper numbers hard-coded in the reference's
results notebook):
* network scale 10/20/30/40/50 clients, IID:    `results_visualization.ipynb:427-448`
* network scale, non-IID:                        `results_visualization.ipynb:529-550`
* client ratio 50..100 %, IID:                   `results_visualization.ipynb:325-346`
* client ratio, non-IID:                         `results_visualization.ipynb:223-244`
"""
from __future__ import annotations

import json
import sys
from collections import defaultdict

SCALE_REF = {True: {10: 99.01, 20: 98.54, 30: 98.34, 40: 98.45, 50: 98.20},
             False: {10: 97.30, 20: 97.29, 30: 97.73, 40: 97.77, 50: 98.52}}
RATIO_REF = {True: {0.5: 99.01, 0.6: 98.96, 0.7: 98.44, 0.8: 98.71, 0.9: 98.60, 1.0: 98.69},
             False: {0.5: 97.30, 0.6: 97.08, 0.7: 97.00, 0.8: 97.21, 0.9: 97.11, 1.0: 97.21}}


def load(paths):
    recs = []
    for p in paths:
        with open(p) as f:
            recs += [json.loads(ln) for ln in f if ln.strip()]
    # one record per point (the 10-client 50 % point is in both sweeps)
    uniq = {}
    for r in recs:
        uniq[(r["backend"], r.get("init_mode"), r["iid"], r["clients"], r["participation"], r["rounds"])] = r
    return list(uniq.values())


def tables(recs) -> str:
    out = []
    by = defaultdict(list)
    for r in recs:
        by[(r["backend"], r.get("init_mode", "?"), r["iid"])].append(r)
    for (backend, init, iid), rs in sorted(by.items(), key=lambda kv: (kv[0][0], kv[0][1], not kv[0][2])):
        split = "IID" if iid else "non-IID"
        scale = [r for r in rs if r["participation"] == 0.5]
        ratio = [r for r in rs if r["clients"] == 10]
        if len({r["clients"] for r in scale}) > 1:
            out += [f"### network scale, {split} ({backend} engine, init {init}, participation 50 %)", "",
                    "| clients | rounds | final mean AUC % | final min % | mean of last 10 rounds % | best round % (round) "
                    "| paper % | rejected / round (last 10) | rounds/s |",
                    "|---|---|---|---|---|---|---|---|---|"]
            for r in sorted(scale, key=lambda r: r["clients"]):
                ref = SCALE_REF[iid].get(r["clients"])
                out.append(f"| {r['clients']} | {r['rounds']} | {100 * r['auc_mean_final']:.2f} | "
                           f"{100 * r['auc_min_final']:.2f} | {100 * r['auc_mean_last10']:.2f} | "
                           f"{100 * r['auc_mean_best_round']:.2f} ({r['best_round']}) | "
                           f"{ref if ref is not None else '—'} | {r['rejected_last10_mean']} | {r['rounds_per_sec']} |")
            vals = [100 * r["auc_mean_last10"] for r in scale]
            out += ["", f"spread of the last-10-round means over N: {max(vals) - min(vals):.2f} points", ""]
        if len({r["participation"] for r in ratio}) > 1:
            out += [f"### client ratio, {split} ({backend} engine, init {init}, 10 clients)", "",
                    "| participation | rounds | final mean AUC % | final min % | mean of last 10 rounds % | "
                    "best round % (round) | paper % |", "|---|---|---|---|---|---|---|"]
            for r in sorted(ratio, key=lambda r: r["participation"]):
                ref = RATIO_REF[iid].get(round(r["participation"], 1))
                out.append(f"| {int(round(100 * r['participation']))} % | {r['rounds']} | "
                           f"{100 * r['auc_mean_final']:.2f} | {100 * r['auc_min_final']:.2f} | "
                           f"{100 * r['auc_mean_last10']:.2f} | {100 * r['auc_mean_best_round']:.2f} "
                           f"({r['best_round']}) | {ref if ref is not None else '—'} |")
            out.append("")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    sys.stdout.write(tables(load(sys.argv[1:])))
