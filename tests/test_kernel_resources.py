"""Register budget of the helper-wave training kernel (VERDICT r5 Next #1b / #5;
CPU only: hipcc cross-compiles for gfx950).

The kernel runs 8 wave64 per workgroup, two per SIMD, so each wave has 256
registers (VGPR + AGPR) and no more; in round 5 the benchmark's
instantiation (plain, batch <= 12) sat at that ceiling with 68 VGPR spills and
248 B of scratch per lane.  Round 6 removed the experiment switches and
stopped the staging passes from keeping their ~40 LDS addresses live through
the launch (``stage_tid``).  This test pins what is left: no scratch access
inside the training-step loop (the MFMA-dense loop of the main waves), and at
most 2 spilled VGPRs / 16 B of scratch per lane for the whole plain
instantiation (two loop-invariant offsets reloaded at epoch ends).
"""
import re
import shutil

import pytest

from fedmse_decentralized_amd.ops import build

PLAIN = "_ZN5fedmx2hw15train_kernel_hwILb0ELb0EEEvNS_9TrainArgsE"

pytestmark = pytest.mark.skipif(shutil.which("hipcc") is None and not build.Path("/opt/rocm/bin/hipcc").exists(),
                                reason="needs hipcc")


def _loops(asm: str, fn: str):
    """(mfma count, scratch count) of every basic block of ``fn`` that ends
    in a branch back to itself or an earlier block (loop bodies), merged per
    loop as the blocks from its header to its latch."""
    body = asm[asm.index(f"\n{fn}:"):]
    body = body[:body.index("s_endpgm")]
    blocks, cur = [], {"name": "entry", "mfma": 0, "scratch": 0, "br": []}
    for line in body.splitlines():
        s = line.strip()
        m = re.match(r"^(\.LBB[\w_]+):", s)
        if m:
            blocks.append(cur)
            cur = {"name": m.group(1), "mfma": 0, "scratch": 0, "br": []}
            continue
        if not s or s.startswith((";", ".")):
            continue
        if "mfma" in s:
            cur["mfma"] += 1
        if s.startswith("scratch_"):
            cur["scratch"] += 1
        m = re.match(r"^s_(?:cbranch_\w+|branch)\s+(\.LBB[\w_]+)", s)
        if m:
            cur["br"].append(m.group(1))
    blocks.append(cur)
    idx = {b["name"]: i for i, b in enumerate(blocks)}
    loops = []
    for i, b in enumerate(blocks):
        for t in b["br"]:
            if t in idx and idx[t] <= i:
                seg = blocks[idx[t]:i + 1]
                loops.append((sum(x["mfma"] for x in seg), sum(x["scratch"] for x in seg), idx[t], i))
    return loops


def test_plain_training_kernel_register_budget():
    res = build.kernel_resources("fedmx_train_hw.hip", asm=True)
    r = res[PLAIN]
    print(build.train_resource_report())
    assert r["vgpr"] <= 256 and r["occupancy"] >= 2
    assert r["vgpr_spill"] <= 2, r
    assert r["scratch"] <= 16, r
    loops = _loops(res["__asm__"], PLAIN)
    # the training-step loop: the innermost loop with >= 150 MFMAs (ping-pong
    # of two steps, 83 each on the main waves; the epoch loop around it holds
    # the epoch-end work and may reload a spilled offset there)
    big = [lp for lp in loops if lp[0] >= 150]
    inner = [lp for lp in big if not any(o is not lp and lp[2] <= o[2] and o[3] <= lp[3] and (o[2], o[3]) != (lp[2], lp[3])
                                         for o in big)]
    assert inner, loops
    step = min(inner, key=lambda lp: lp[3] - lp[2])
    assert 150 <= step[0] <= 200, step
    assert step[1] == 0, f"scratch access inside the step loop: {step}"
