"""Per-kernel timing on one GPU (torch CUDA events, median over repeats).

Workload = the flagship round's shapes: 10 N-BaIoT-sized clients, 5 trained
per round for E epochs at batch 12; evaluation of all 10 clients.
Prints one JSON object with microseconds per launch and derived per-step
costs of the fused training kernel.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

from fedmse_decentralized_amd.data.prepare import prepare_federation  # noqa: E402
from fedmse_decentralized_amd.data.synthetic import SyntheticSpec, generate_federation  # noqa: E402
from fedmse_decentralized_amd.engine.base import TrainHParams  # noqa: E402
from fedmse_decentralized_amd.engine.hip_engine import HipEngine  # noqa: E402
from fedmse_decentralized_amd.eval.evaluator import evaluate_clients  # noqa: E402
from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS  # noqa: E402
from fedmse_decentralized_amd.models.reference import init_client_params  # noqa: E402
from fedmse_decentralized_amd.ops import _hip  # noqa: E402


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts)), float(np.min(ts))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--clients", type=int, default=10)
    p.add_argument("--train-clients", type=int, default=5)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--train-only", action="store_true", help="only the training-kernel timings (A/B of builds)")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    raws = generate_federation(SyntheticSpec(kind="nbaiot", n_clients=args.clients, seed=1))
    clients, dev_set = prepare_federation(raws, 1234)
    init, _ = init_client_params(args.clients, 0)
    eng = HipEngine(DEFAULT_DIMS, dev)
    eng.setup([c.train for c in clients], [c.valid for c in clients], [c.test for c in clients],
              [c.test_label for c in clients], init)
    out = {}
    sel = list(range(args.train_clients))
    # fixed-epoch training (patience large so every epoch runs)
    hp = TrainHParams(epochs=args.epochs, batch_size=12, lr=1e-3, shrink_lambda=5.0, patience=10 ** 6)
    n_train = [c.train.shape[0] for c in clients[:args.train_clients]]
    n_valid = [c.valid.shape[0] for c in clients[:args.train_clients]]
    steps = max((n + 11) // 12 for n in n_train) * args.epochs
    vsteps = max((n + 11) // 12 for n in n_valid) * args.epochs
    med, mn = timeit(lambda: eng.train_async(sel, hp), reps=args.reps)
    out["train_launch_us"] = med
    out["train_launch_us_min"] = mn
    out["train_steps_per_client"] = steps
    out["valid_batches_per_client"] = vsteps
    out["us_per_train_step_upper"] = med / steps
    hp1 = TrainHParams(epochs=args.epochs, batch_size=12, lr=1e-3, shrink_lambda=5.0, patience=10 ** 6)
    med1, _ = timeit(lambda: eng.train_async([0], hp1), reps=args.reps)
    out["train_launch_1client_us"] = med1
    hpp = TrainHParams(epochs=args.epochs, batch_size=12, lr=1e-3, shrink_lambda=5.0, fedprox_mu=0.001,
                       patience=10 ** 6)
    out["train_launch_fedprox_us"] = timeit(lambda: eng.train_async(sel, hpp), reps=args.reps)[0]
    _hip.TRAIN_COMPACT = False   # identity internal order (no padded k-steps skipped)
    out["train_launch_identity_order_us"] = timeit(lambda: eng.train_async(sel, hp), reps=args.reps)[0]
    _hip.TRAIN_COMPACT = True
    # batch 64 (the thesis's GPU runs): helper-wave kernel (16-row chunks) vs the 4-wave kernel
    hp64 = TrainHParams(epochs=args.epochs, batch_size=64, lr=1e-3, shrink_lambda=5.0, patience=10 ** 6)
    out["train_launch_b64_us"] = timeit(lambda: eng.train_async(sel, hp64), reps=args.reps)[0]
    hp64p = TrainHParams(epochs=args.epochs, batch_size=64, lr=1e-3, shrink_lambda=5.0, fedprox_mu=0.001,
                         patience=10 ** 6)
    out["train_launch_b64_fedprox_us"] = timeit(lambda: eng.train_async(sel, hp64p), reps=args.reps)[0]
    prev, _hip.TRAIN_HELPER = _hip.TRAIN_HELPER, False
    out["train_launch_b64_4wave_us"] = timeit(lambda: eng.train_async(sel, hp64), reps=args.reps)[0]
    _hip.TRAIN_HELPER = prev
    if args.train_only:
        print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in out.items()}))
        return
    allc = list(range(args.clients))
    items = [(c, eng.store.rows("test", c)) for c in allc]
    out["fwd_sse_all_test_us"] = timeit(lambda: eng.forward_rows(eng.store.params, items, True, False))[0]
    items2 = []
    for c in allc:
        items2 += [(c, eng.store.rows("train", c)), (c, eng.store.rows("test", c))]
    out["fwd_latent_train_test_us"] = timeit(lambda: eng.forward_rows(eng.store.params, items2, False, True))[0]
    _, lat = eng.forward_rows(eng.store.params, items2, False, True)
    out["cen_us"] = timeit(lambda: eng.cen_scores(lat[0::2], lat[1::2]))[0]
    sc = eng.cen_scores(lat[0::2], lat[1::2])
    labs = [eng.store.test_label[int(eng.store.test_off[c]):int(eng.store.test_off[c + 1])] for c in allc]
    out["auc_us"] = timeit(lambda: _hip.auc(sc, labs))[0]
    V = eng.to_device(clients[0].valid)
    out["standardize_us"] = timeit(lambda: eng.standardize_ddof1(V))[0]
    stack = eng.store.params[:5].contiguous()
    out["weighted_sum_us"] = timeit(lambda: eng.weighted_sum(stack, [0.2] * 5))[0]
    out["param_drift_us"] = timeit(lambda: eng.param_drift(stack[:2], stack[3]))[0]
    t0 = time.perf_counter()
    for _ in range(20):
        evaluate_clients(eng, allc, "hybrid", "AUC")
    out["evaluate_hybrid_host_us"] = (time.perf_counter() - t0) / 20 * 1e6
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in out.items()}))


if __name__ == "__main__":
    main()
