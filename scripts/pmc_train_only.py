"""Five 5-client training launches of the benchmark workload (bench_kernels
--train-only's first timing, nothing else), for per-kernel PMC passes:

  FEDMX_HIP_LIB=... rocprofv3 --kernel-trace --pmc <counters> -- python3 scripts/pmc_train_only.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fedmse_decentralized_amd.data.prepare import prepare_federation  # noqa: E402
from fedmse_decentralized_amd.data.synthetic import SyntheticSpec, generate_federation  # noqa: E402
from fedmse_decentralized_amd.engine.base import TrainHParams  # noqa: E402
from fedmse_decentralized_amd.engine.hip_engine import HipEngine  # noqa: E402
from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS  # noqa: E402
from fedmse_decentralized_amd.models.reference import init_client_params  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    raws = generate_federation(SyntheticSpec(kind="nbaiot", n_clients=10, seed=1))
    clients, _ = prepare_federation(raws, 1234)
    init, _ = init_client_params(10, 0)
    eng = HipEngine(DEFAULT_DIMS, dev)
    eng.setup([c.train for c in clients], [c.valid for c in clients], [c.test for c in clients],
              [c.test_label for c in clients], init)
    hp = TrainHParams(epochs=5, batch_size=12, lr=1e-3, shrink_lambda=5.0, patience=10 ** 6)
    for _ in range(5):
        eng.train_async(list(range(5)), hp)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
