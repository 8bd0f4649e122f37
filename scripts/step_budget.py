"""Per-phase issue budget of one training step of the helper-wave kernel
(VERDICT r5 Next #1a): static instruction counts of each stamped phase of the
production step (the -DFEDMX_STAMPS=1 build's assembly, phases between
consecutive HSTAMP points) priced with the gfx950 issue costs, set against
the phase times the stamped build measured on the GPU
(``scripts/train_stamps.py --json``).

    python scripts/step_budget.py gpurun_out/s2/stamps.json > profiles/r6_step_budget.md

Issue prices (cycles per wave instruction, /opt/skills/guides/MI355X_MICROARCH.md
constants table): v_mfma_f32_16x16x4_f32 32 (it holds the SIMD's vector issue
for all 32: SQ_VALU_MFMA_COEXEC_CYCLES = 0, profiles/r5_pmc_train_hw.md),
VALU 4, transcendental (v_sqrt / v_rcp / v_rsq / v_exp / v_log) 8, f64 VALU 8,
packed fp32 (v_pk_*) 4, ds_* 4, s_nop N 4(N+1) (the wave's own stall: another
wave may issue meanwhile), other SALU 2, vector memory 4.  The residue of a
phase is measured minus the main wave's own issue minus the helper wave's
issue in the same window (both waves of a SIMD share its issue port): the
dependent-latency, LDS-wait and barrier-skew time no instruction filled.
"""
from __future__ import annotations

import json
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from fedmse_decentralized_amd.ops import build  # noqa: E402

KERNEL = "_ZN5fedmx2hw15train_kernel_hwILb0ELb0EEEvNS_9TrainArgsE"
TRANS = ("v_sqrt", "v_rcp", "v_rsq", "v_exp", "v_log", "v_sin", "v_cos")
# (stamp i, stamp j, name in scripts/train_stamps.py PHASES_HW)
MAIN_PHASES = [(0, 1, "main: L1 partial write"), (1, 2, "main: barrier #1 wait"),
               (2, 3, "main: L1 reduce + L2..L4 + loss"), (3, 4, "main: prefetch + dY + dH3 partial + stage"),
               (4, 7, "main: barrier #2 wait"), (7, 8, "main: dH3 reduce + dZ + dH1"),
               (8, 9, "main: dW1 + small-tile MFMAs"), (9, 10, "main: adam W1"),
               (10, 11, "main: next L1 + adam small + publish")]
HELPER_PHASES = [(0, 2, "helper: barrier #1 wait"), (2, 7, "helper: barrier #2 wait"), (7, 8, "helper: dW4 MFMAs"),
                 (8, 10, "helper: adam W4"), (10, 11, "helper: publish W4 + scalars")]
STEP = "main: STEP (stamp 0 -> 11)"


def price(op: str, text: str) -> tuple:
    """(category, issue cycles) of one instruction."""
    if "mfma" in op:
        return "mfma", 32
    if op.startswith("v_"):
        if op.startswith(TRANS):
            return "trans", 8
        if "_f64" in op:
            return "f64", 8
        return "valu", 4
    if op.startswith("ds_"):
        return "lds", 4
    if op == "s_nop":
        n = int(text.split()[1], 0) if len(text.split()) > 1 else 0
        return "nop", 4 * (n + 1)
    if op in ("s_waitcnt", "s_barrier", "s_sleep", "s_memtime", "s_setprio"):
        return "wait", 0
    if op.startswith("s_"):
        return "salu", 2
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem", 4
    return "other", 0


def stamp_asm() -> str:
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "k.s"
        cmd = [build.hipcc_path(), *build._hip_flags(["-DFEDMX_STAMPS=1"]), "--cuda-device-only", "-S",
               "-gline-tables-only", f"-I{build.CSRC / 'hip'}", str(build.CSRC / "hip" / "fedmx_train_hw.hip"),
               "-o", str(out)]
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        return out.read_text()


def phase_counts(asm: str):
    """{(role, i, j): counters} for the first stamped step of the main and
    helper loops: the instructions between the s_memtime of stamp i and the
    s_memtime of stamp j in program order."""
    src = (build.CSRC / "hip" / "fedmx_train_hw.hip").read_text().splitlines()
    files = {}
    for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', asm):
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
    body = asm[asm.index(f"\n{KERNEL}:"):]
    body = body[:body.index("s_endpgm")]
    events = []   # (kind, payload) in program order
    loc = None
    for line in body.splitlines():
        s = line.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = (files.get(m.group(1)), int(m.group(2)))
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0].rstrip(":")
        if op == "s_memtime":
            idx = None
            if loc and loc[0] == "fedmx_train_hw.hip" and 0 < loc[1] <= len(src):
                mm = re.search(r"HSTAMP\((\w+),\s*(\d+)\)", src[loc[1] - 1])
                if mm:
                    idx = (mm.group(1), int(mm.group(2)))
            events.append(("stamp", idx))
        else:
            events.append(("ins", (op, s)))
    # first occurrence of each stamp of the step (ms: main, hs: helper)
    res = {}
    for role, key in (("main", "ms"), ("helper", "hs")):
        pos = {}
        for k, (kind, pay) in enumerate(events):
            if kind == "stamp" and pay and pay[0] == key and pay[1] not in pos:
                pos[pay[1]] = k
        phases = MAIN_PHASES if role == "main" else HELPER_PHASES
        for i, j, _ in phases:
            if i not in pos or j not in pos or pos[j] < pos[i]:
                continue
            c = {}
            for kind, pay in events[pos[i] + 1:pos[j]]:
                if kind != "ins":
                    continue
                cat, cyc = price(*pay)
                n, t = c.get(cat, (0, 0))
                c[cat] = (n + 1, t + cyc)
            res[(role, i, j)] = c
    return res


def measured(stamps_json: str):
    """Median over repetitions and waves of each phase (``train_stamps.py
    --json``: {rep: {phase name: [8 waves]}}; main waves = 0-3, helpers 4-7;
    the helper-side phases of the JSON are stored in the helpers' columns)."""
    import numpy as np

    data = json.load(open(stamps_json))

    def med(name, rows):
        v = [r[name][w] for r in data.values() for w in rows
             if isinstance(r.get(name), list) and r[name][w] is not None]
        return float(np.median(v)) if v else float("nan")

    return med


def main():
    asm = stamp_asm()
    counts = phase_counts(asm)
    med = measured(sys.argv[1]) if len(sys.argv) > 1 else None
    print("# Training-step budget of the helper-wave kernel (round 6)\n")
    print("Phase times: shader-clock cycles, median over the stamped runs and over the four main / helper waves "
          "(`scripts/train_stamps.py --json`, epoch 0, step 20).  Issue: the static instruction mix of the phase in "
          "the stamped build's assembly, priced as in `scripts/step_budget.py`.\n")
    cats = ("mfma", "valu", "trans", "f64", "lds", "salu", "nop", "vmem")
    for role, phases in (("main", MAIN_PHASES), ("helper", HELPER_PHASES)):
        rows = range(0, 4) if role == "main" else range(4, 8)
        print(f"## {role} waves (stamp rows {rows.start}-{rows.stop - 1})\n")
        print("| phase | measured | " + " | ".join(f"{c} n / cyc" for c in cats) + " | issue | residue |")
        print("|---|---|" + "---|" * (len(cats) + 2))
        tot_m = tot_i = 0.0
        for i, j, name in phases:
            c = counts.get((role, i, j), {})
            m = med(name, rows) if med else float("nan")
            issue = sum(v[1] for k, v in c.items() if k != "nop")
            cells = " | ".join(f"{c.get(k, (0, 0))[0]} / {c.get(k, (0, 0))[1]}" for k in cats)
            short = name.split(": ", 1)[1]
            print(f"| {short} ({i}->{j}) | {m:.0f} | {cells} | {issue} | {m - issue:.0f} |")
            if m == m:
                tot_m += m
            tot_i += issue
        print(f"| **sum** | **{tot_m:.0f}** |" + " |" * len(cats) + f" **{tot_i:.0f}** | **{tot_m - tot_i:.0f}** |\n")
    if med:
        print(f"Measured step (main waves, stamp 0 -> 11): {med(STEP, range(0, 4)):.0f} cycles.\n")
    print(json.dumps({f"{r}:{i}->{j}": c for (r, i, j), c in counts.items()}), file=sys.stderr)


if __name__ == "__main__":
    main()
