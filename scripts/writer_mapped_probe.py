"""Does reading the best-model snapshot out of the device-mapped host ring
(hipHostMalloc mapped|coherent) slow the artefact writer?  Times
write_round_artifacts from (a) ordinary numpy memory, (b) the mapped ring,
(c) the mapped ring copied to ordinary memory first."""
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
from fedmse_decentralized_amd.ops import _hiprt  # noqa: E402


def med(fn, reps=20):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(1e6 * float(np.median(ts[3:])), 1)


def main():
    n = 32
    torch.zeros(1, device="cuda")
    cidx = padded_index(DEFAULT_DIMS)[0].numpy()
    host = np.random.default_rng(0).normal(size=(64, P_PAD)).astype(np.float32)
    mb = _hiprt.MappedBuffer(host.nbytes)
    mapped = mb.view(0, np.float32, host.size).reshape(64, P_PAD)
    mapped[:] = host
    root = tempfile.mkdtemp(prefix="fedmx_wprobe_")
    dirs = [os.path.join(root, f"c{i}") for i in range(n)]
    trk = [[(1.0 + i, 2.0 + i) for i in range(3)] for _ in range(n)]
    files = ArtifactFiles()
    rows = list(range(n))
    out = {
        "numpy_snapshot_us": med(lambda: ck.write_round_artifacts(files, dirs, host, rows, [True] * n, trk, cidx)),
        "mapped_snapshot_us": med(lambda: ck.write_round_artifacts(files, dirs, mapped, rows, [True] * n, trk, cidx)),
        "mapped_copy_first_us": med(lambda: ck.write_round_artifacts(files, dirs, np.array(mapped[:n]), rows,
                                                                     [True] * n, trk, cidx)),
        "copy_mapped_32rows_us": med(lambda: np.array(mapped[:n])),
        "copy_numpy_32rows_us": med(lambda: np.array(host[:n])),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
