"""Long-run parity of the device-resident round protocol against the
host-decision path on the benchmark's own configuration (10 N-BaIoT-shaped
clients, 5 local epochs, batch 12, FedMSE, fixed compat): every round's
selection, aggregator, verification results and AUCs, and the final
parameters, must be identical (the GPU tests cover 4-6 rounds on small
clients; this covers the bench shapes over many rounds, where a near-tie in
a vote or a verification threshold would show up).

    python scripts/device_vs_host_long.py [--rounds 40] [--update-type mse_avg]
"""
from __future__ import annotations

import argparse
import json
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fedmse_decentralized_amd import federation  # noqa: E402
from fedmse_decentralized_amd.config import ExperimentConfig  # noqa: E402
from fedmse_decentralized_amd.federation import Federation  # noqa: E402


def run(device_protocol: bool, rounds: int, update_type: str, out: str):
    federation._PREP_CACHE.clear()
    cfg = ExperimentConfig(synthetic="nbaiot", network_size=10, num_rounds=rounds, epoch=5, batch_size=12,
                           lr_rate=1e-3, shrink_lambda=5, output_root=out, backend="hip", device="cuda",
                           log_level="WARNING", compat="fixed", global_early_stop=False, save_checkpoints=False,
                           model_types=["hybrid"], update_types=[update_type], device_protocol=device_protocol)
    fed = Federation(cfg, "hybrid", update_type, 0).setup()
    assert (fed._fast is not None) == device_protocol
    res = []
    for r in range(rounds):
        if r and r % 20 == 0:
            fed.reset_aggregation_counts()   # bench.py's 20-round episodes
        res.append(fed.run_round())
    fed.finish()
    torch.cuda.synchronize()
    rows = [dict(sel=list(x.selected), agg=x.aggregator, ver=x.verification, auc=[float(v) for v in x.metrics])
            for x in res]
    return fed, rows


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=40)
    p.add_argument("--update-type", default="mse_avg")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    with tempfile.TemporaryDirectory() as d:
        fd, dev = run(True, a.rounds, a.update_type, d + "/dev")
        fh, host = run(False, a.rounds, a.update_type, d + "/host")
    first_diff = next((i for i, (x, y) in enumerate(zip(dev, host)) if x != y), None)
    same_params = bool(torch.equal(fd.engine.store.params, fh.engine.store.params))
    rec = dict(rounds=a.rounds, update_type=a.update_type, identical_rounds=first_diff is None,
               first_differing_round=first_diff, identical_params=same_params,
               aggregators=[r["agg"] for r in dev], final_auc_mean=float(np.mean(dev[-1]["auc"])),
               rejections=int(sum(1 for r in dev for v in r["ver"] if not v["is_verified"])))
    line = json.dumps(rec)
    print(line)
    if a.out:
        Path(a.out).write_text(line + "\n")
    return 0 if (first_diff is None and same_params) else 1


if __name__ == "__main__":
    sys.exit(main())
