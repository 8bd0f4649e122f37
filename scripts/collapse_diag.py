"""Per-round health diagnostics of a federation's aggregate model.

Large federations (many separately initialised clients) were seen to lose
detection quality after a few rounds ("Missing #1").  This script
runs one federation and logs, per round, for the model every client ends the
round with (client 0's parameters after adoption) and for the aggregate:

* mean / min AUC over clients, rejections,
* latent norm and per-dimension latent std on the shared dev set,
* dead hidden units of the encoder (never active on the dev sample),
* ||W2|| (encoder's latent layer), ||W3|| (decoder's first layer),
* FedMSE weight entropy (relative to uniform) and the dev-MSE spread.

Usage:
  python scripts/collapse_diag.py --clients 64 --rounds 10 --backend torch --compat fixed [--init-mode shared]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fedmse_decentralized_amd import federation as fedmod  # noqa: E402
from fedmse_decentralized_amd.config import ExperimentConfig  # noqa: E402
from fedmse_decentralized_amd.models.layout import padded_to_canonical  # noqa: E402
from fedmse_decentralized_amd.models.reference import functional_forward, unflatten  # noqa: E402


def model_health(flat_padded: torch.Tensor, dims, dev: torch.Tensor) -> dict:
    t = unflatten(padded_to_canonical(flat_padded.detach().float().cpu(), dims), dims)
    w1, b1, w2, b2, w3, b3, w4, b4 = t
    x = dev[:, :dims.d_in]
    with torch.no_grad():
        h1 = torch.relu(torch.nn.functional.linear(x, w1, b1))
        z, y = functional_forward(t, x)
    zn = torch.linalg.vector_norm(z, dim=1)
    return {
        "z_norm_mean": float(zn.mean()),
        "z_std_min": float(z.std(0).min()),
        "z_std_mean": float(z.std(0).mean()),
        "dead_h1": int(((h1 > 0).sum(0) == 0).sum()),
        "w2_norm": float(torch.linalg.vector_norm(w2)),
        "w3_norm": float(torch.linalg.vector_norm(w3)),
        "dev_mse": float(((y - x) ** 2).mean()),
    }


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--backend", default="torch")
    ap.add_argument("--compat", default="fixed")
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--shrink-lambda", type=float, default=5.0)
    ap.add_argument("--update-type", default="mse_avg")
    ap.add_argument("--model-type", default="hybrid")
    ap.add_argument("--participation", type=float, default=0.5)
    ap.add_argument("--non-iid", action="store_true")
    ap.add_argument("--kind", default="nbaiot")
    ap.add_argument("--dev-rows", type=int, default=4096, help="dev rows used for the health statistics")
    ap.add_argument("--extra", default="{}", help="JSON dict of further ExperimentConfig overrides")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "8")))
    cfg = ExperimentConfig(
        num_participants=a.participation, epoch=a.epochs, num_rounds=a.rounds, lr_rate=a.lr,
        shrink_lambda=a.shrink_lambda, network_size=a.clients, model_types=[a.model_type],
        update_types=[a.update_type], synthetic=a.kind, synthetic_iid=not a.non_iid, compat=a.compat,
        backend=a.backend, global_early_stop=False, save_checkpoints=False,
        output_root=tempfile.mkdtemp(prefix="fedmx_diag_"), log_level="WARNING", **json.loads(a.extra))
    plans = []
    orig = fedmod.make_plan

    def spy(update_type, selected, aggregator, dev_mse, compat, **kw):
        p = orig(update_type, selected, aggregator, dev_mse, compat, **kw)
        plans.append((p, dict(dev_mse)))
        return p

    fedmod.make_plan = spy
    drifts = []
    from fedmse_decentralized_amd.protocol import verification as vmod
    orig_decide = vmod.Verifier.decide

    def decide_spy(self, client_id, st, version, perf_new, drift, current_round):
        d = orig_decide(self, client_id, st, version, perf_new, drift, current_round)
        if d.drift:
            drifts.append(d.drift)
        return d

    vmod.Verifier.decide = decide_spy
    fed = fedmod.Federation(cfg, a.model_type, a.update_type, run=0, write_reports=False).setup()
    if fed._fast is not None:
        raise SystemExit("diagnostics need the host-decision path (plans are read on the host); "
                         "use --backend torch or --extra '{\"device_protocol\": false}'")
    g = torch.Generator().manual_seed(0)
    dev = fed.dev_set.detach().float().cpu()
    dev = dev[torch.randperm(dev.shape[0], generator=g)[: a.dev_rows]]
    out = open(a.out, "w") if a.out else None
    rec0 = {"round": 0, **model_health(fed.engine.store.params[0], fed.dims, dev)}
    print(json.dumps(rec0), flush=True)
    for r in range(a.rounds):
        t0 = time.perf_counter()
        drifts.clear()
        res = fed.run_round()
        agg = fed.versions.get(r)
        rej = sum(1 for v in res.verification if not v["is_verified"])
        rec = {"round": r + 1, "auc_mean": round(float(np.mean(res.metrics)), 5),
               "auc_min": round(float(np.min(res.metrics)), 5), "rejected": rej,
               "receivers": len(res.verification), "aggregator": res.aggregator,
               "sec": round(time.perf_counter() - t0, 2)}
        if drifts:
            rec.update(drift_med=round(float(np.median(drifts)), 4), drift_max=round(float(np.max(drifts)), 4))
        if plans:
            p, dm = plans[-1]
            w = np.array([x for _, x in p], dtype=np.float64)
            w = w / w.sum()
            ent = -float(np.sum(w * np.log(np.maximum(w, 1e-300)))) / math.log(len(w)) if len(w) > 1 else 1.0
            mses = np.array(list(dm.values()))
            rec.update(w_entropy_rel=round(ent, 4), w_max=round(float(w.max()), 4),
                       devmse_min=round(float(mses.min()), 4), devmse_max=round(float(mses.max()), 4))
        if agg is not None:
            rec.update({"agg_" + k: v for k, v in model_health(agg, fed.dims, dev).items()})
        rec.update({"c0_" + k: v for k, v in model_health(fed.engine.store.params[0], fed.dims, dev).items()})
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
            out.flush()


if __name__ == "__main__":
    main()
