"""Is the IEEE-Adam build's long-horizon divergence (client 1 only) rounding
chaos or nondeterminism?  Runs the 100-epoch paper-config training of
tests/test_long_horizon_gpu.py with the library named by FEDMX_HIP_LIB and
saves the final state; compare runs with --compare.

  FEDMX_HIP_LIB=... python scripts/r4_exact_diag.py --out a.npz
  python scripts/r4_exact_diag.py --compare a.npz b.npz
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(out, epochs, seed):
    import torch

    from test_long_horizon_gpu import _clients, _engines
    from fedmse_decentralized_amd.engine.base import TrainHParams
    from fedmse_decentralized_amd.ops import _hip

    ref, hip = _engines(_clients(seed), torch.device("cuda", 0))
    hp = TrainHParams(epochs=epochs, batch_size=12, lr=1e-5, shrink_lambda=10.0, patience=10 ** 6)
    r = hip.train([0, 1], hp)
    np.savez(out, params=hip.store.params.cpu().numpy(), m=hip.store.adam_m.cpu().numpy(),
             v=hip.store.adam_v.cpu().numpy(), tracking=np.array(r.tracking), lib=_hip.lib_path())
    print("saved", out, _hip.lib_path())


def compare(paths):
    a = np.load(paths[0])
    for p in paths[1:]:
        b = np.load(p)
        for k in ("params", "m", "v", "tracking"):
            d = np.abs(a[k].astype(np.float64) - b[k].astype(np.float64))
            per_client = d.reshape(d.shape[0], -1).max(axis=1) if d.ndim > 1 else d.max()
            print(f"{os.path.basename(paths[0])} vs {os.path.basename(p)} {k}: identical={bool((a[k] == b[k]).all())}"
                  f" max|d| per client {np.array2string(np.asarray(per_client), precision=3)}")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--out")
    p.add_argument("--epochs", type=int, default=100)
    p.add_argument("--seed", type=int, default=3)
    p.add_argument("--compare", nargs="+")
    a = p.parse_args()
    if a.compare:
        compare(a.compare)
    else:
        run(a.out, a.epochs, a.seed)
