"""Batched-forward cost of the per-round FedMSE dev-set scoring as the
federation grows (weak scaling: 10 clients per GPU, dev set = 10*N*~660 rows,
each rank scores its ~5 selected models on the whole dev set)."""
from __future__ import annotations

import json
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS, canonical_to_padded  # noqa: E402
from fedmse_decentralized_amd.models.reference import init_client_params  # noqa: E402
from fedmse_decentralized_amd.ops import _hip  # noqa: E402


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))


def main():
    dev = torch.device("cuda", 0)
    init, _ = init_client_params(8, 0)
    params = canonical_to_padded(init).to(dev)
    out = {}
    for n_gpus in (1, 2, 4, 8):
        rows = 6600 * n_gpus
        x = torch.zeros(rows, 128, device=dev)
        x[:, :115] = torch.randn(rows, 115, device=dev)
        items = [(m, x) for m in range(5)]
        plan = _hip.FwdPlan(params, items, DEFAULT_DIMS, want_sse=True, want_latent=False)   # cached launch
        us = timeit(plan.run)
        out[f"N{n_gpus}_blocks"] = plan.nblocks
        out[f"N{n_gpus}_5x{rows}_us"] = round(us, 1)
        out[f"N{n_gpus}_TFLOPs"] = round(5 * rows * 2 * 6588 / us / 1e6, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
