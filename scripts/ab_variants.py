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

# Variants that still build.  The r1-r5 source switches (FEDMX_HW_ABLATE,
# FEDMX_ABLATE, FEDMX_HW_PACKED, FEDMX_DW4_LATE, FEDMX_W4_POS, FEDMX_SCHED_HINTS,
# FEDMX_HW_IGLP, FEDMX_HW_FLAGS, FEDMX_HW_XBIAS, FEDMX_HW_SCALED, FEDMX_ADAM_FMA,
# FEDMX_ADAM_SCALED, FEDMX_TRAIN_HW_DEFAULT, FEDMX_VERIFY_ABLATE and the
# per-instantiation masks) were removed from the kernels in round 6; their
# measured results, per round:
#   r2: compiler schedule +2.5 %, sched_group 1 MFMA / 6 VALU +9 %, separately
#       rounded Adam +3 %, dW4 after barrier #2 +0.5 %, W4 Adam after dH1 / after
#       the next L1 issue +2.5 / +2 %, 4-wave kernel for the compact shapes +3 %
#       (FedProx +8 %); timing-only ablations: no dW4 / W4 Adam -9.5 %, no W1
#       Adam -17 %, no small-tile Adam -3 %, no Adam -35 %; verification kernel
#       no forward 13.4 / no drift 18.9 / no adoption 21.4 of 24.6 us
#   r4: no iglp hint +12.6 %, iglp_opt(1) +1.6 %, helper->main LDS flags: FedProx
#       -3.3 % (kept for FedProx), plain +6 %; no barrier in the step loop: slower
#   r5: unscaled FMA Adam 897 vs 870 us; bias units / value masks / ping-pong per
#       instantiation (README table in fedmx_train_hw.hip); packed-fp32 Adam +2 %;
#       asynchronous-validation check step 2 / 4 / 8 / 10 / 12 / 40: within 1 us
# (profiles/r2_*, r3_train_hw_experiments.md, r4_train_hw_experiments.md,
# r5_train_kernel_ab.md; the source of every variant is in git history before
# round 6.)
VARIANTS = {
    "base": [],                                   # the production build
    "exact": ["-DFEDMX_EXACT_ADAM=1"],            # r4: IEEE sqrt / division Adam (torch's op sequence)
    "stamps": ["-DFEDMX_STAMPS=1"],               # in-kernel phase stamps (scripts/train_stamps.py --lib)
    "novgprform": ["-mllvm", "-amdgpu-mfma-vgpr-form=0"],  # AGPR accumulators (+3.3%)
    "noslp": ["-fno-slp-vectorize"],              # no packed fp32 VALU        (+5%)
    # r2 session 4 / r5 (r5sch): compiler scheduling knobs on the whole library,
    # train launch (r2 base 945.6 / 945.5 us on the same box; none kept; r5:
    # iterative-ilp crashes the compiler, max-memory-clause 922 us vs 842-846)
    "s_ilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],                  # 1001.9 / 1000.5
    "s_trk": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],                   # 970.6 / 1007.4
    "s_norp": ["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule=1"],  # 957.4 / 961.0
    "s_bias0": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],                # 947.1 / 945.3
    "s_cyc": ["-mllvm", "-misched-cyclicpath=1"],                           # 946.7 / 945.9
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
