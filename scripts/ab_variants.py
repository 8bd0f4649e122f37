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
    # (r3 Gram-form step variants gram0/gram1/gabl_*/stamps_gram*: commit 6472e1c, profiles/r3_gram_form.md)
    # r3: helper-wave kernel step-loop variants r0b0 r2b0 r0b1 r1b1 r2b1 r0b0k r2b1k r0b0p r1b0 r0b0q,
    # helper delays hd8/16/24, priorities hprio1/3 and (r2) hwprio1/3: all measured slower or
    # neutral (profiles/r3_train_hw_experiments.md); their switches were removed from the kernel
    # (source in git history, commit 5365856)
    # r4: pipelined W1 Adam (pipe, flags_pipe, flags2_pipe), the SPLIT step (hwsplit,
    # hwsplitd1/2) and grouped dH3 reads (red8) measured slower and were removed from
    # the kernel (profiles/r4_train_hw_experiments.md; source in git history, commit ef22669)
    # r5: the early helper start (early1/early2, +1.6 / +18 %) and main-wave priority
    # (mainprio, +0.6 %) likewise (profiles/r5_train_kernel_ab.md; commit 247945c)
    "hwscaled0": ["-DFEDMX_HW_SCALED=0"],           # r5: unscaled FMA Adam in the helper-wave kernel: 897 vs 870 us (-3.0 %)
    # r5: per-instantiation masks (bit 0 plain batch <= 12, 1 FedProx, 2 batch > 12); default 6 / 6 / 5
    "allon": ["-DFEDMX_HW_BIAS_UNITS=7", "-DFEDMX_HW_VALUE_MASKS=7", "-DFEDMX_HW_PINGPONG=7"],
    "r5base": ["-DFEDMX_HW_BIAS_UNITS=0", "-DFEDMX_HW_VALUE_MASKS=0", "-DFEDMX_HW_PINGPONG=0"],   # scaled Adam only
    "exact": ["-DFEDMX_EXACT_ADAM=1"],               # r4: IEEE sqrt / division Adam (torch's op sequence)
    "flags": ["-DFEDMX_HW_FLAGS=1"],                 # r4: mains-only layer-1 exchange + helper->main LDS flags
    "flags_madam": ["-DFEDMX_HW_FLAGS=1", "-DFEDMX_HW_ABLATE=32"],   # timing only: + mains skip W1 Adam
    "flags_hnone": ["-DFEDMX_HW_FLAGS=1", "-DFEDMX_HW_ABLATE=64"],   # timing only: + helpers idle
    # r4: per-epoch Adam-scalar table (ktab): +1.0 %, removed (commit 96da3e2)
    # r4: dH3 partial reads four at a time per tile, fenced (red4): +10.1 %, removed
    # r5: per-wave dZ partials exchanged at barrier #2 (dzp): plain +12 %, removed
    # r5: forward kernels' first row tile loaded before the parameter staging: no gain, removed
    # r5 (r5sch): LLVM scheduler strategies for the whole library (-mllvm -amdgpu-sched-strategy=max-ilp /
    #   iterative-minreg / max-memory-clause, -amdgpu-use-amdgpu-trackers, -misched-postra-direction=bottomup,
    #   -amdgpu-disable-unclustered-high-rp-reschedule; iterative-ilp crashes the compiler): plain train launch
    #   864 / 932 / 922 / 865 / 892 / 845 us vs 842-846 default -- none faster, removed
    "noiglp": ["-DFEDMX_HW_IGLP=-1"],               # r4: no iglp_opt hint in the step loop
    "iglp1": ["-DFEDMX_HW_IGLP=1"],                 # r4: iglp_opt(1) in the step loop
    "flags2": ["-DFEDMX_HW_FLAGS=2"],                # r4: no workgroup barrier in the step loop
    "packed": ["-DFEDMX_HW_PACKED=1"],               # packed-fp32 Adam (bit-identical)  966-974 vs 948-951 (+2 %)
    "abl_pf": ["-DFEDMX_HW_ABLATE=8"],               # timing only: prefetch always hits the cache
    "abl_hadam": ["-DFEDMX_HW_ABLATE=16"],           # timing only: helpers skip W4's Adam
    "abl_madam": ["-DFEDMX_HW_ABLATE=32"],           # timing only: mains skip W1's Adam
    "abl_hnone": ["-DFEDMX_HW_ABLATE=64"],           # timing only: helpers idle between barriers
    "base": [],                                   # defaults: compact order, FMA Adam, iglp_opt(0), VGPR-form MFMA
    "sched0": ["-DFEDMX_SCHED_HINTS=0"],          # compiler schedule          (+2.5%, measured)
    "hint1": ["-DFEDMX_SCHED_HINTS=1"],           # 64 x (1 MFMA, 6 VALU)      (+9%)
    "sepadam": ["-DFEDMX_ADAM_FMA=0"],            # separately rounded Adam    (+3%)
    "dw4late": ["-DFEDMX_DW4_LATE=1"],            # dW4 products after barrier #2 (+0.5%)
    "split_chains": ["-DFEDMX_SPLIT_CHAINS=7"],   # L2 / dZ as two accumulator chains everywhere (r5h: plain -0.7 %, b64 -0.3 %, FedProx +1.2 %: production mask 5)
    "nosplit": ["-DFEDMX_SPLIT_CHAINS=0"],        # one accumulator chain everywhere (the r5g build)
    "noav": ["-DFEDMX_HW_ASYNC_VALID=0"],         # epoch-end validation inside the trainer workgroup (synchronous)
    "avc4": ["-DFEDMX_HW_AV_CHECK=4"],            # the trainer needs epoch e's decision before step 4 of e+1
    "avc8": ["-DFEDMX_HW_AV_CHECK=8"],            # ... before step 8 (r5avc: 844 / 844 us vs 843 / 845, also 10 / 12: same)
    "avc40": ["-DFEDMX_HW_AV_CHECK=40"],          # ... before step 40 (never waits: the fixed cost of the path)
    "avc2": ["-DFEDMX_HW_AV_CHECK=2"],            # ... before step 2
    "av3": ["-DFEDMX_HW_ASYNC_VALID=3"],          # asynchronous validation for FedProx too
    "av7": ["-DFEDMX_HW_ASYNC_VALID=7"],          # ... and for batch > 12
    "stamps_avc4": ["-DFEDMX_STAMPS=1", "-DFEDMX_HW_AV_CHECK=4"],   # timeline of the step-4 check (scripts/train_stamps.py --lib)
    "novgprform": ["-mllvm", "-amdgpu-mfma-vgpr-form=0"],  # AGPR accumulators (+3.3%)
    "noslp": ["-fno-slp-vectorize"],              # no packed fp32 VALU        (+5%)
    "w4pos1": ["-DFEDMX_W4_POS=1"],               # W4 Adam after dH1, fenced   (+2.5%)
    "w4pos2": ["-DFEDMX_W4_POS=2"],               # W4 Adam after the next L1 issue, fenced (+2%)
    "nohw": ["-DFEDMX_TRAIN_HW_DEFAULT=0"],       # 4-wave kernel for the compact shapes too (+3%, FedProx +8%)
    "scaled": ["-DFEDMX_ADAM_SCALED=1"],          # scaled-moment Adam, 5 VALU/param (+0.5%)
    # helper-wave kernel, timing-only ablations of the main waves' step (r2, base
    # 1.059 ms; per-step Adam constants on the mains: 0.992 ms without -> moved
    # to the helpers)
    "hwabl_loss": ["-DFEDMX_HW_ABLATE=2"],        # no loss accumulation          1.044 ms
    # (small tiles read as 16-byte D-layout copies instead of 16 scalar LDS reads:
    # 0.965 vs 0.966 ms, FedProx 1.089 vs 1.043 -- reverted)
    # (moving the loss share to the helpers measured 1.066 vs 0.966 ms: the helpers'
    # work between barrier #2 and #1 is on the step's path once it exceeds the
    # mains'; a per-chunk Adam-scalar table instead of per-step scalars: 0.974 ms)
    "hwabl_small": ["-DFEDMX_HW_ABLATE=4"],       # no small-tile gradient / Adam 1.024 ms
    # timing-only ablations (wrong numerics): what each optimizer piece costs
    # on the critical path (r2, base 1.095 ms)
    "abl_w4": ["-DFEDMX_ABLATE=1"],               # no dW4 / W4 Adam          0.991 ms (-9.5%)
    "abl_w1adam": ["-DFEDMX_ABLATE=2"],           # no W1 Adam                0.912 ms (-17%)
    "abl_small": ["-DFEDMX_ABLATE=4"],            # no small-tile Adam        1.063 ms (-3%)
    "abl_adam": ["-DFEDMX_ABLATE=8"],             # no Adam at all            0.708 ms (-35%)
    # r2 session 4: compiler scheduling knobs on the whole library, train launch
    # (base 945.6 / 945.5 us on the same box; none kept)
    "s_ilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],                  # 1001.9 / 1000.5
    "s_trk": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],                   # 970.6 / 1007.4
    "s_norp": ["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule=1"],  # 957.4 / 961.0
    "s_bias0": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],                # 947.1 / 945.3
    "s_cyc": ["-mllvm", "-misched-cyclicpath=1"],                           # 946.7 / 945.9
    # fused verification kernel, timing-only (r2, base 24.6 us; scripts/ab/r2_verify_ablate.sh)
    "vabl1": ["-DFEDMX_VERIFY_ABLATE=1"],         # no forward                13.4 us
    "vabl2": ["-DFEDMX_VERIFY_ABLATE=2"],         # no drift                  18.9 us
    "vabl4": ["-DFEDMX_VERIFY_ABLATE=4"],         # no adoption pass          21.4 us
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
