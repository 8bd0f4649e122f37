"""Non-IID accuracy against the reference's own shipped run (VERDICT r4 Next #2a).

The reference ships a complete N-BaIoT non-IID experiment,
`/root/reference/src/Checkpoint/Results/Update/10/nonIID_Exp10_Rerun_5epoch_10client_lr0001_lamda1_ratio50.0/`:
six combinations x 2 runs at 5 local epochs, lr 1e-3, shrink lambda 1, 50 %
participation, with its per-round per-client AUC files and
``training_summary.json``.  Its per-round files have 5 rows for the first
combination (hybrid + avg, run 0) and fewer after it: the module-global
early-stop state, so ``num_rounds`` was 5.

This script compares one of our result trees (``main.py --config-file
/root/reference/src/Configuration/scen2-nba-iot-10clients_noniid.json --epoch 5
--num-rounds 5 --lr-rate 1e-3 --shrink-lambda 1 --num-runs 2 ...``) with it:

* rounds per combination and run (the early-stop pattern);
* best AUC per combination (``training_summary.json``: max over clients of
  the final round, max over runs), ours over the 7 clients whose ``abnormal/``
  data ships, the reference's over its 10 and over the same 7 positions;
* per-client AUC over every round and run, per combination: mean / min / max
  over the 7 complete clients, ours vs the reference's same client positions.

The client order of the per-round files is the reference's device sampling
(``random.Random(1234).sample(devices_list, 10)``, `src/main.py:116,126`),
which this framework replays; the three clients without abnormal data
(`/root/reference/.MISSING_LARGE_BLOBS:4-6`) are the positions whose AUC we
report as null.

    python scripts/noniid_vs_reference.py OURS_EXPERIMENT_DIR [--out profiles/r5_noniid_vs_reference.md]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import random
import sys

import numpy as np

REF_EXP = ("/root/reference/src/Checkpoint/Results/Update/10/"
           "nonIID_Exp10_Rerun_5epoch_10client_lr0001_lamda1_ratio50.0")
REF_CFG = "/root/reference/src/Configuration/scen2-nba-iot-10clients_noniid.json"
COMBOS = [(m, u) for m in ("hybrid", "autoencoder") for u in ("avg", "fedprox", "mse_avg")]


def load_rounds(exp_dir: str):
    """{(model, update): {run: [client_metrics per round]}} with None for null."""
    out = {}
    for f in sorted(glob.glob(os.path.join(exp_dir, "Run_*", "AUC", "*_results.json"))):
        run = int(f.split("Run_")[1].split(os.sep)[0])
        rows = [json.loads(ln) for ln in open(f) if ln.strip()]
        if not rows:
            continue
        key = (rows[0]["model_type"], rows[0]["update_type"])
        out.setdefault(key, {})[run] = [[None if v is None or v != v else float(v) for v in r["client_metrics"]]
                                        for r in rows]
    return out


def sampled_names():
    dl = json.load(open(REF_CFG))["devices_list"]
    return [d["name"] for d in random.Random(1234).sample(dl, len(dl))]


def _stats(vals):
    v = np.asarray([x for x in vals if x is not None], dtype=np.float64)
    return (float(v.mean()), float(v.min()), float(v.max()), int(v.size)) if v.size else (np.nan,) * 3 + (0,)


def compare(ours_dir: str) -> str:
    ref = load_rounds(REF_EXP)
    ours = load_rounds(ours_dir)
    names = sampled_names()
    ref_sum = json.load(open(os.path.join(REF_EXP, "training_summary.json")))["best_metrics"]
    our_sum_path = os.path.join(ours_dir, "training_summary.json")
    our_sum = json.load(open(our_sum_path))["best_metrics"] if os.path.exists(our_sum_path) else {}
    # positions of the clients whose abnormal data ships: ours report a number there
    any_rows = next(iter(next(iter(ours.values())).values()))
    complete = [i for i, v in enumerate(any_rows[0]) if v is not None]
    missing = [names[i] for i in range(len(names)) if i not in complete]
    L = []
    L.append(f"Client order (reference device sampling, seed 1234): {', '.join(n.split('-')[-1] for n in names)} "
             f"(client numbers).  Without abnormal data here: {', '.join(missing)} -> AUC null, "
             f"left out below; compared positions: {len(complete)}.")
    L.append("")
    L.append("### Rounds run per combination (run 0 / run 1)")
    L.append("")
    L.append("| combination | reference | ours |")
    L.append("|---|---|---|")
    for k in COMBOS:
        r = ref.get(k, {})
        o = ours.get(k, {})
        L.append(f"| {k[0]} + {k[1]} | {len(r.get(0, []))} / {len(r.get(1, []))} | "
                 f"{len(o.get(0, []))} / {len(o.get(1, []))} |")
    L.append("")
    L.append("### Best AUC per combination (training_summary.json: max over clients of the final models, max over runs)")
    L.append("")
    L.append("| combination | reference (10 clients) | reference (7 positions) | ours (7 clients) | ours - ref(7) |")
    L.append("|---|---|---|---|---|")
    for m, u in COMBOS:
        r10 = ref_sum[m][u]
        r7 = max(max(x for i, x in enumerate(runs[-1]) if i in complete) for runs in ref[(m, u)].values())
        o7 = max(max(x for x in runs[-1] if x is not None) for runs in ours[(m, u)].values()) \
            if (m, u) in ours else float("nan")
        if our_sum:
            o7 = our_sum[m][u]
        L.append(f"| {m} + {u} | {r10:.5f} | {r7:.5f} | {o7:.5f} | {o7 - r7:+.5f} |")
    L.append("")
    L.append("### Per-client AUC over every round and run (the 7 complete clients)")
    L.append("")
    L.append("| combination | ref mean | ref min | ref max | ours mean | ours min | ours max | n ref / ours |")
    L.append("|---|---|---|---|---|---|---|---|")
    allr, allo = [], []
    for k in COMBOS:
        rv = [row[i] for runs in ref.get(k, {}).values() for row in runs for i in complete]
        ov = [row[i] for runs in ours.get(k, {}).values() for row in runs for i in complete]
        allr += rv
        allo += ov
        a, b = _stats(rv), _stats(ov)
        L.append(f"| {k[0]} + {k[1]} | {a[0]:.4f} | {a[1]:.4f} | {a[2]:.4f} | {b[0]:.4f} | {b[1]:.4f} | "
                 f"{b[2]:.4f} | {a[3]} / {b[3]} |")
    a, b = _stats(allr), _stats(allo)
    L.append(f"| all | {a[0]:.4f} | {a[1]:.4f} | {a[2]:.4f} | {b[0]:.4f} | {b[1]:.4f} | {b[2]:.4f} | "
             f"{a[3]} / {b[3]} |")
    L.append("")
    L.append("### Per client (all combinations, rounds and runs)")
    L.append("")
    L.append("| position | client | ref mean | ref range | ours mean | ours range |")
    L.append("|---|---|---|---|---|---|")
    for i in complete:
        rv = [row[i] for runs in ref.values() for rr in runs.values() for row in rr]
        ov = [row[i] for runs in ours.values() for rr in runs.values() for row in rr]
        a, b = _stats(rv), _stats(ov)
        L.append(f"| {i} | {names[i]} | {a[0]:.4f} | {a[1]:.4f}-{a[2]:.4f} | {b[0]:.4f} | {b[1]:.4f}-{b[2]:.4f} |")
    return "\n".join(L) + "\n"


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("ours", help="our experiment directory (Checkpoint/Results/Update/10/<name>)")
    p.add_argument("--out", default=None)
    a = p.parse_args(argv)
    text = compare(a.ours)
    if a.out:
        with open(a.out, "a") as f:
            f.write(text)
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
