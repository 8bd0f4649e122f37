"""Write a synthetic N-BaIoT / Kitsune-shaped federation to disk in the
reference's CSV layout plus a device-list JSON (see
``fedmse_decentralized_amd.data.synthetic.write_dataset``).

    python scripts/make_synthetic_dataset.py /tmp/fedmx_data --kind nbaiot --clients 10
    python main.py --config-file /tmp/fedmx_data/Configuration/synthetic-nbaiot-10clients.json
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fedmse_decentralized_amd.data.synthetic import SyntheticSpec, write_dataset  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--kind", default="nbaiot", choices=["nbaiot", "kitsune"])
    ap.add_argument("--clients", type=int, default=10)
    ap.add_argument("--non-iid", action="store_true")
    ap.add_argument("--seed", type=int, default=2025)
    a = ap.parse_args(argv)
    path = write_dataset(a.out, SyntheticSpec(kind=a.kind, n_clients=a.clients, iid=not a.non_iid, seed=a.seed))
    print(path)


if __name__ == "__main__":
    main()
