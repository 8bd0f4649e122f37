"""The oracle's own divergence from 1-ulp-perturbed copies of itself over the
long-horizon test's 100 epochs (CPU only): every perturbation of
``tests/test_long_horizon_gpu._perturbations`` for each (mu, batch) case,
max |oracle - perturbed oracle| per client and tensor, and the per-epoch
loss's max relative difference.  The test's absolute ceilings
(``SENS_CEIL``) come from this record (a chaotic-size regression
must not pass by widening its own tolerance).

    python scripts/long_horizon_sensitivity.py > profiles/r6_long_horizon_sensitivity.json
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "4")))


def main():
    from test_long_horizon_gpu import _clients, _diffs, _engines, _perturbations, _set_anchor

    from fedmse_decentralized_amd.engine.base import TrainHParams

    clients = _clients()
    out = {}
    for mu in (0.0, 0.001):
        for batch in (12, 64):
            hp = TrainHParams(epochs=100, batch_size=batch, lr=1e-5, shrink_lambda=10.0, fedprox_mu=mu,
                              patience=10 ** 6)
            ref, _ = _engines(clients, None)
            _set_anchor([ref], mu)
            r1 = ref.train([0, 1], hp)
            runs = []
            for p_init in _perturbations(hp):
                p, _ = _engines(clients, None, p_init)
                _set_anchor([p], mu)
                rp = p.train([0, 1], hp)
                runs.append(_diffs(r1, ref, rp, p))
            agg = {c: {k: max(r[c][k] for r in runs) for k in runs[0][c]} for c in (0, 1)}
            key = f"mu={mu} batch={batch}"
            out[key] = {"max_over_perturbations": agg, "per_perturbation": runs}
            print(key, json.dumps(agg), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
