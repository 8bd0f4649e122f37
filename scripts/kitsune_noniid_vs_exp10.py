"""Is the reference's shipped non-IID run (Exp10) consistent with the
Kitsune non-IID device list?  (VERDICT r5 Next #6b)

Exp10 (`/root/reference/src/Checkpoint/Results/Update/10/nonIID_Exp10_...`)
never names its device list; round 5 showed it is not reproducible from the
shipped N-BaIoT non-IID CSVs.  This compares it with our runs of the Kitsune
non-IID list (`/root/reference/src/Configuration/kitsune-iot-10clients_noniid.json`)
at Exp10's settings (5 local epochs, lr 1e-3, lambda 1, 50 % participation,
2 runs, six combinations, 5 rounds), on its 8 complete clients (client 5
ships without ``abnormal/``, client 7 without ``abnormal/`` and ``normal/``:
`/root/reference/.MISSING_LARGE_BLOBS:1-3`; the run uses the 8 others, so
device positions cannot be matched one to one and the comparison is of
per-client AUC distributions and per-combination bests).

    python scripts/kitsune_noniid_vs_exp10.py OURS_EXP_DIR [OURS_EXP_DIR_2 ...]
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import noniid_vs_reference as nvr  # noqa: E402


def per_client(rounds):
    """{combo: [(client position, mean, min, max) ...]} over every round and run."""
    out = {}
    for key, runs in rounds.items():
        cols = {}
        for rr in runs.values():
            for row in rr:
                for i, v in enumerate(row):
                    if v is not None:
                        cols.setdefault(i, []).append(v)
        out[key] = sorted((i, float(np.mean(v)), float(np.min(v)), float(np.max(v))) for i, v in cols.items())
    return out


def summarize(label, d):
    ours = nvr.load_rounds(d)
    summ = json.load(open(os.path.join(d, "training_summary.json")))["best_metrics"]
    pc = per_client(ours)
    return label, ours, summ, pc


def main(dirs):
    ref = nvr.load_rounds(nvr.REF_EXP)
    ref_sum = json.load(open(os.path.join(nvr.REF_EXP, "training_summary.json")))["best_metrics"]
    ref_pc = per_client(ref)
    runs = [summarize(os.path.basename(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(d)))))
                      or d, d) for d in dirs]
    lines = ["| combination | Exp10 best | " + " | ".join(f"{lab} best" for lab, *_ in runs) + " |",
             "|---|---|" + "---|" * len(runs)]
    for m, u in nvr.COMBOS:
        cells = [f"{s.get(m, {}).get(u, float('nan')):.4f}" for _, _, s, _ in runs]
        lines.append(f"| {m} + {u} | {ref_sum[m][u]:.4f} | " + " | ".join(cells) + " |")
    lines.append("")
    lines.append("Per-client AUC over every round and run (mean, min-max), clients sorted by mean:")
    lines.append("")
    lines.append("| combination | Exp10 (10 N-BaIoT positions) | " + " | ".join(lab for lab, *_ in runs) + " |")
    lines.append("|---|---|" + "---|" * len(runs))

    def cell(v):
        v = sorted(v, key=lambda t: -t[1])
        return "<br>".join(f"{a:.4f} ({b:.4f}-{c:.4f})" for _, a, b, c in v)

    for combo in nvr.COMBOS:
        row = [cell(ref_pc.get(combo, []))] + [cell(pc.get(combo, [])) for *_, pc in runs]
        lines.append(f"| {combo[0]} + {combo[1]} | " + " | ".join(row) + " |")
    lines.append("")
    # pooled statistics
    def pooled(pc):
        v = [t[1] for lst in pc.values() for t in lst]
        mn = [t[2] for lst in pc.values() for t in lst]
        return np.mean(v), np.min(mn), np.median(v)
    lines.append("| run | pooled per-client mean AUC | lowest single AUC | median per-client mean |")
    lines.append("|---|---|---|---|")
    a = pooled(ref_pc)
    lines.append(f"| Exp10 | {a[0]:.4f} | {a[1]:.4f} | {a[2]:.4f} |")
    for lab, _, _, pc in runs:
        a = pooled(pc)
        lines.append(f"| {lab} | {a[0]:.4f} | {a[1]:.4f} | {a[2]:.4f} |")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1:])
