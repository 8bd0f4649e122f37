"""Build variants of the HIP library for A/B timing of the training kernel.

    python scripts/ab_variants.py build            # on the CPU host (hipcc cross-compiles)
    bash scripts/ab_train.sh                       # on the GPU box: times every built variant

Each variant is ``libfedmx_hip_<name>.so`` next to the main library, built
with the extra compiler flags below; ``scripts/ab_train.sh`` loads each one
through ``FEDMX_HIP_LIB`` in its own process.
"""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from fedmse_decentralized_amd.ops import build  # noqa: E402

VARIANTS = {
    "base": [],                                   # defaults: compact order, FMA Adam, iglp_opt(0), VGPR-form MFMA
    "sched0": ["-DFEDMX_SCHED_HINTS=0"],          # compiler schedule          (+2.5%, measured)
    "hint1": ["-DFEDMX_SCHED_HINTS=1"],           # 64 x (1 MFMA, 6 VALU)      (+9%)
    "sepadam": ["-DFEDMX_ADAM_FMA=0"],            # separately rounded Adam    (+3%)
    "dw4late": ["-DFEDMX_DW4_LATE=1"],            # dW4 products after barrier #2 (+0.5%)
    "split": ["-DFEDMX_SPLIT_CHAINS=1"],          # L2 / dZ as two accumulator chains (+0.3%)
    "novgprform": ["-mllvm", "-amdgpu-mfma-vgpr-form=0"],  # AGPR accumulators (+3.3%)
    "noslp": ["-fno-slp-vectorize"],              # no packed fp32 VALU        (+5%)
}


def main():
    names = sys.argv[2:] or list(VARIANTS)
    if sys.argv[1:2] == ["build"]:
        for n in names:
            t = build.LIBDIR / f"libfedmx_hip_{n}.so"
            build.build_hip(force=True, extra_flags=VARIANTS[n], target=t)
            print("built", t)
    elif sys.argv[1:2] == ["list"]:
        print(" ".join(names))


if __name__ == "__main__":
    main()
