"""Figures of the reference's visualisation notebooks.

* ``scale``   — detection AUC against the federation size, ours next to the
  FedMSE paper's network-scale bars (`src/Visualization/results_visualization.ipynb:427-448`,
  `:529-550`), from ``scripts/network_scale.py`` records;
* ``ratio``   — AUC against the client participation ratio, next to the
  paper's client-ratio bars (`results_visualization.ipynb:223-244`, `:325-346`);
* ``combos``  — final-round mean AUC of every model x update combination from
  a results directory (``*_results.json`` reports), next to the paper's
  per-algorithm averages (`results_visualization.ipynb:29-50`, `:130-147`);
* ``tsne``    — 2-D t-SNE of one client's test-set latents from a
  ``--save-latents`` LatentData pickle written by this framework
  (`src/Visualization/latent_visualization.ipynb:35-111`: normal vs abnormal
  rows, one panel per update type).

    python scripts/plots.py scale profiles/r3_network_scale_hip.jsonl --out profiles/plots/network_scale.png
    python scripts/plots.py ratio profiles/r3_client_ratio_hip.jsonl --out profiles/plots/client_ratio.png
    python scripts/plots.py combos Checkpoint/Results/Update/10 --out combos.png
    python scripts/plots.py tsne Checkpoint/LatentData/10/<exp>/Run_0 --device NBa-Synth-Client-5 --out tsne.png
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import pickle
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import matplotlib  # noqa: E402

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

from results_table import PAPER_IID, PAPER_NONIID, load_results  # noqa: E402
from scale_table import RATIO_REF, SCALE_REF  # noqa: E402
from scale_table import load as load_scale  # noqa: E402


COLORS = {"fedmx HIP (shared init)": "tab:blue", "fedmx CPU oracle (shared init)": "tab:orange",
          "fedmx HIP (per-client init, reference)": "tab:gray", "FedMSE paper": "tab:red",
          "fedmx (final round)": "tab:blue", "paper IID": "tab:red", "paper non-IID": "tab:pink"}


def _grouped_bars(ax, groups, series, ylabel, title):
    """series: [(label, {group: value or None})]"""
    n = len(series)
    width = 0.8 / max(n, 1)
    x = np.arange(len(groups))
    for i, (label, vals) in enumerate(series):
        ys = [vals.get(g) for g in groups]
        xs = [x[j] + (i - (n - 1) / 2) * width for j, y in enumerate(ys) if y is not None]
        ax.bar(xs, [y for y in ys if y is not None], width=width, label=label, color=COLORS.get(label))
    ax.set_xticks(x)
    ax.set_xticklabels([str(g) for g in groups])
    ax.set_ylabel(ylabel)
    ax.set_title(title)
    ax.legend(fontsize=7, loc="lower left")
    lo = min((v for _, s in series for v in s.values() if v is not None), default=90.0)
    ax.set_ylim(max(0.0, min(lo - 1.0, 95.0)), 100.0)
    ax.grid(axis="y", alpha=0.3)


def plot_sweep(paths, key, ref, xlabel, out, title):
    recs = load_scale(paths)
    fig, axes = plt.subplots(1, 2, figsize=(12, 4.2))
    for ax, iid in zip(axes, (True, False)):
        rs = [r for r in recs if r["iid"] == iid and (key == "clients" and r["participation"] == 0.5
                                                      or key == "participation" and r["clients"] == 10)]
        groups = sorted({r[key] for r in rs} | set(ref[iid]))
        series = []
        for (backend, init), label in ((("hip", "shared"), "fedmx HIP (shared init)"),
                                       (("torch", "shared"), "fedmx CPU oracle (shared init)"),
                                       (("hip", "per_client"), "fedmx HIP (per-client init, reference)")):
            vals = {r[key]: 100 * r["auc_mean_last10"] for r in rs if r["backend"] == backend
                    and r.get("init_mode") == init}
            if vals:
                series.append((label, vals))
        series.append(("FedMSE paper", {g: v for g, v in ref[iid].items()}))
        _grouped_bars(ax, groups, series, "mean client AUC % (last 10 of 50 rounds)",
                      f"{title}, {'IID' if iid else 'non-IID'}")
        ax.set_xlabel(xlabel)
    fig.tight_layout()
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    fig.savefig(out, dpi=110)
    return out


def plot_combos(root, out):
    res = load_results(root)
    groups, ours = [], {}
    for path, rows in res.items():
        mt, ut = rows[-1].get("model_type", "?"), rows[-1].get("update_type", "?")
        g = f"{'SAE-CEN' if mt == 'hybrid' else 'AE'}\n{ut}"
        groups.append(g)
        ours[g] = 100 * float(np.mean(rows[-1]["client_metrics"]))
    lab = {f"{'SAE-CEN' if mt == 'hybrid' else 'AE'}\n{ut}": (mt, ut) for mt, ut in PAPER_IID}
    fig, ax = plt.subplots(figsize=(8, 4))
    _grouped_bars(ax, groups, [("fedmx (final round)", ours),
                               ("paper IID", {g: PAPER_IID.get(lab.get(g)) for g in groups}),
                               ("paper non-IID", {g: PAPER_NONIID.get(lab.get(g)) for g in groups})],
                  "mean client AUC %", "detection AUC per model x aggregation")
    fig.tight_layout()
    fig.savefig(out, dpi=110)
    return out


def plot_tsne(run_dir, device, out, rnd=None, seed=0):
    from sklearn.manifold import TSNE

    files = sorted(glob.glob(os.path.join(run_dir, "latent_hybrid_*.pkl")))
    if not files:
        raise SystemExit(f"no latent_hybrid_*.pkl under {run_dir} (run with --save-latents)")
    fig, axes = plt.subplots(1, len(files), figsize=(5 * len(files), 4.5), squeeze=False)
    for ax, path in zip(axes[0], files):
        with open(path, "rb") as f:   # a file this framework wrote (io.checkpoint.save_latents)
            data = pickle.load(f)
        rounds = sorted(data)
        r = rounds[-2] if rnd is None and len(rounds) > 1 else (rounds[-1] if rnd is None else rnd)
        lat, lab = data[r][device]
        emb = TSNE(n_components=2, random_state=seed, init="pca", perplexity=min(30, max(5, len(lat) // 4))
                   ).fit_transform(np.asarray(lat, dtype=np.float64))
        lab = np.asarray(lab)
        ax.scatter(emb[lab == 0, 0], emb[lab == 0, 1], s=4, alpha=0.5, color="tab:blue", label="Normal")
        ax.scatter(emb[lab == 1, 0], emb[lab == 1, 1], s=4, alpha=0.5, color="tab:red", label="Abnormal")
        ax.set_title(f"{os.path.basename(path)[7:-4]}  round {r + 1}")
        ax.legend(fontsize=8)
    fig.suptitle(f"t-SNE of {device}'s test-set latents")
    fig.tight_layout()
    fig.savefig(out, dpi=110)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["scale", "ratio", "combos", "tsne"])
    ap.add_argument("inputs", nargs="+")
    ap.add_argument("--out", required=True)
    ap.add_argument("--device", default=None)
    ap.add_argument("--round", type=int, default=None)
    a = ap.parse_args(argv)
    if a.kind == "scale":
        print(plot_sweep(a.inputs, "clients", SCALE_REF, "clients", a.out, "SAE-CEN + MSEAvg vs network size"))
    elif a.kind == "ratio":
        print(plot_sweep(a.inputs, "participation", RATIO_REF, "participation ratio", a.out,
                         "SAE-CEN + MSEAvg vs client ratio (10 clients)"))
    elif a.kind == "combos":
        print(plot_combos(a.inputs[0], a.out))
    else:
        if not a.device:
            raise SystemExit("--device NAME is required for tsne")
        print(plot_tsne(a.inputs[0], a.device, a.out, a.round))
    return 0


if __name__ == "__main__":
    sys.exit(main())
