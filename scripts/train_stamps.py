"""In-kernel phase timing of the fused training kernel (s_memtime stamps).

Loads the ``-DFEDMX_STAMPS=1`` build (``libfedmx_hip_stamps.so``), trains the
flagship round's 5 clients once and prints, per wave, the counter ticks spent
in each phase of one training step (epoch 0, step STAMP_STEP), of one
validation tile, and of the launch prologue / epilogue.  The default kernel
for the reference shapes is the helper-wave kernel (``fedmx_train_hw.hip``:
waves 0-3 run the step's chain, 4-7 the W4 gradient + Adam); ``--four-waves``
stamps the 4-wave kernel (``fedmx_train.hip``) instead.  ``--json out`` also
writes every repetition's table.  s_memtime counts shader-clock cycles (round
1: a 9,500-tick step against 3.9 us of launch time per step, ~2.4 GHz).
"""
from __future__ import annotations

import json
import os
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
sys.path.insert(0, ROOT)
PLAIN = "--plain" in sys.argv   # regular build, no stamps (for PMC counter runs)
LIBNAME = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else "libfedmx_hip_stamps.so"
if not PLAIN:
    os.environ["FEDMX_HIP_LIB"] = os.path.join(ROOT, "fedmse_decentralized_amd/ops/lib", LIBNAME)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from fedmse_decentralized_amd.data.prepare import prepare_federation  # noqa: E402
from fedmse_decentralized_amd.data.synthetic import SyntheticSpec, generate_federation  # noqa: E402
from fedmse_decentralized_amd.engine.base import TrainHParams  # noqa: E402
from fedmse_decentralized_amd.engine.hip_engine import HipEngine  # noqa: E402
from fedmse_decentralized_amd.models.layout import DEFAULT_DIMS  # noqa: E402
from fedmse_decentralized_amd.models.reference import init_client_params  # noqa: E402
from fedmse_decentralized_amd.ops import _hip, build  # noqa: E402

PHASES4 = [
    (0, 1, "L1 partial write"), (1, 2, "barrier #1"), (2, 3, "fwd reduce + L2..L4 + loss"),
    (3, 4, "prefetch + dY/transposes + dH3 partial + stage"), (4, 5, "dW4 mfma"),
    (6, 7, "barrier #2"), (7, 8, "dH3 reduce + dZ + dH1 (batch-major)"), (8, 9, "dW1 mfma + small tile"),
    (9, 10, "adam W1"), (10, 11, "next L1 + adam W4/small + publish"), (0, 11, "TRAIN STEP TOTAL"),
    (16, 17, "valid: one chunk (one wave)"), (14, 15, "valid: epoch pass (per wave)"),
    (28, 29, "prologue (state load)"),
    (12, 13, "epoch end (reduce + snapshot)"), (30, 31, "epilogue (write back)"),
]
# helper-wave kernel: rows 0-3 = main waves, 4-7 = helpers (fedmx_train_hw.hip HSTAMP points)
PHASES_HW = [
    (0, 1, "main: L1 partial write"), (1, 2, "main: barrier #1 wait"),
    (2, 3, "main: L1 reduce + L2..L4 + loss"), (3, 4, "main: prefetch + dY + dH3 partial + stage"),
    (4, 7, "main: barrier #2 wait"), (7, 8, "main: dH3 reduce + dZ + dH1"),
    (8, 9, "main: dW1 + small-tile MFMAs"), (9, 10, "main: adam W1"),
    (10, 11, "main: next L1 + adam small + publish"), (0, 11, "main: STEP (stamp 0 -> 11)"),
    (0, 2, "helper: barrier #1 wait"), (2, 7, "helper: barrier #2 wait"), (7, 8, "helper: dW4 MFMAs"),
    (8, 10, "helper: adam W4"), (10, 11, "helper: publish W4 + scalars"),
    (16, 17, "valid: one 16-row tile (one wave)"), (14, 15, "valid: epoch pass (per wave)"),
    (12, 13, "epoch tail (barriers, validation, exchange, snapshot)"),
    (18, 19, "async validation: epoch-0 end (snapshot, moments, publish)"),
    (20, 21, "async validation: epoch-1 decision check (step AV_CHECK)"),
    (28, 29, "prologue (state load, mains)"), (30, 31, "epilogue (write back, mains)"),
]
FOUR = "--four-waves" in sys.argv


def main():
    if not PLAIN and LIBNAME == "libfedmx_hip_stamps.so" and not build.HIP_STAMPS_LIB.exists():
        build.build_hip(extra_flags=["-DFEDMX_STAMPS=1"], target=build.HIP_STAMPS_LIB)
    dev = torch.device("cuda", 0)
    raws = generate_federation(SyntheticSpec(kind="nbaiot", n_clients=10, seed=1))
    clients, _ = prepare_federation(raws, 1234)
    init, _ = init_client_params(10, 0)
    eng = HipEngine(DEFAULT_DIMS, dev)
    eng.setup([c.train for c in clients], [c.valid for c in clients], [c.test for c in clients],
              [c.test_label for c in clients], init)
    mu = float(sys.argv[sys.argv.index("--mu") + 1]) if "--mu" in sys.argv else 0.0   # FedProx instantiation
    hp = TrainHParams(epochs=5, batch_size=12, lr=1e-3, shrink_lambda=5.0, patience=10 ** 6, fedprox_mu=mu)
    stamps = torch.zeros(8 * 32, dtype=torch.int64, device=dev)
    helper = not FOUR
    nw = 8 if helper else 4
    phases = PHASES_HW if helper else PHASES4
    if PLAIN:
        for _ in range(3):
            _hip.train(eng.store, list(range(5)), hp, eng.dims, helper=helper)
        torch.cuda.synchronize()
        print("plain train launches done")
        return
    out = {}
    for rep in range(4):
        _hip.train(eng.store, list(range(5)), hp, eng.dims, stamps=stamps, helper=helper)
        torch.cuda.synchronize()
        st = stamps.view(8, 32).cpu().numpy().astype(np.int64)[:nw]
        res = {}
        for a, b, name in phases:
            res[name] = [int(st[w, b] - st[w, a]) if st[w, a] and st[w, b] else None for w in range(nw)]
        if helper and not FOUR:
            # asynchronous validation, client 0: wall_clock64 ticks (100 MHz) in slots 22..27
            raw = stamps.cpu().numpy().astype(np.int64)
            names = {22: "trainer: epoch 1 published", 25: "validator: epoch 1 seen",
                     26: "validator: validation done", 27: "validator: decision stored",
                     23: "trainer: decision needed (step AV_CHECK)", 24: "trainer: decision received"}
            if raw[22]:
                res["async validation timeline (us after epoch 1 published)"] = {
                    v: round((int(raw[i]) - int(raw[22])) / 100.0, 2) for i, v in names.items() if raw[i]}
        out[f"rep{rep}"] = res
        stamps.zero_()
    last = out[f"rep{len(out) - 1}"]
    print(f"{'phase (ticks, rep ' + str(len(out) - 1) + ')':52s} " + " ".join(f"{'w' + str(w):>6s}" for w in range(nw)))
    for name, v in last.items():
        if isinstance(v, dict):
            print(name + ": " + ", ".join(f"{k} {x}" for k, x in v.items()))
            continue
        print(f"{name:52s} " + " ".join(f"{x:6d}" if x is not None else "     -" for x in v))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
