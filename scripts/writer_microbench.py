"""Artefact-writer cost per round on this host's filesystem: the native batched
model.cpt + tracking writer (1/2/4 threads), the per-client Python writers it
replaced, and the JSONL reports of a 64-client round (bench temp dir)."""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedmse_decentralized_amd.io import checkpoint as ck  # noqa: E402
from fedmse_decentralized_amd.io.files import ArtifactFiles  # noqa: E402
from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS, P_PAD, padded_index  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    cidx = padded_index(DEFAULT_DIMS)[0].numpy()
    snap = torch.randn(2 * n, P_PAD).numpy()
    root = tempfile.mkdtemp(prefix="fedmx_wbench_")
    dirs = [os.path.join(root, f"c{i}") for i in range(n)]
    for d in dirs:
        os.makedirs(d)
    trk = [[(1.0 + i, 2.0 + i) for i in range(3)] for _ in range(n)]
    out = {}
    files = ArtifactFiles()
    for th in (1, 2, 4):
        ts = []
        for rep in range(30):
            t0 = time.perf_counter()
            ck.write_round_artifacts(files, dirs, snap, list(range(n)), [True] * n, trk, cidx, DEFAULT_DIMS,
                                     n_threads=th)
            ts.append(time.perf_counter() - t0)
        out[f"native_{th}thr_us"] = round(1e6 * float(np.median(ts[5:])), 1)
    ts = []
    for rep in range(30):
        t0 = time.perf_counter()
        for j, d in enumerate(dirs):
            ck.save_model_cpt_fast(d, snap[j][cidx], DEFAULT_DIMS, files=files)
            ck.save_tracking(d, trk[j], files=files)
        ts.append(time.perf_counter() - t0)
    out["python_per_client_us"] = round(1e6 * float(np.median(ts[5:])), 1)
    vr = [{"client_id": c, "rejected_updates": 0, "is_verified": True} for c in range(2 * n)]
    p1, p2 = os.path.join(root, "v.json"), os.path.join(root, "r.json")
    ts = []
    for rep in range(30):
        t0 = time.perf_counter()
        files.append(p1, (json.dumps({"round": rep, "verification_results": vr}) + "\n").encode())
        files.append(p2, (json.dumps({"round": rep, "client_metrics": list(np.random.rand(2 * n)),
                                      "update_type": "mse_avg", "model_type": "hybrid", "global_loss": 0.5})
                          + "\n").encode())
        ts.append(time.perf_counter() - t0)
    out["jsonl_reports_us"] = round(1e6 * float(np.median(ts[5:])), 1)
    out["clients"] = n
    print(json.dumps(out))


if __name__ == "__main__":
    main()
