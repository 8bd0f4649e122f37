"""In-order issue timeline of one wave's loop body from a gfx950 assembly
listing: an instruction-level stall view without a thread trace.

The pool's rocprofv3 has no thread-trace decoder (`--att` needs a decoder
library this ROCm image does not ship), so this is VERDICT r3 Next #2's
fallback: a critical-path analysis of the production build's ISA with
per-instruction latencies.  A wave issues in order, so one pass over the loop
body -- each instruction issuing at max(previous issue + its issue cost, the
time its operands are ready, the time its pipe is free, the time its
`s_waitcnt` is satisfied) -- gives the wave's own timeline, and the gap in
front of each instruction is the stall it pays, attributed to the operand or
counter that was last to arrive.

Latency model (cycles; `/opt/skills/guides/MI355X_MICROARCH.md` constants
table): `v_mfma_f32_16x16x4_f32` holds the matrix pipe 32 and the vector
issue 8 (the bf16 figure; for this fp32 MFMA the PMC counters show no VALU
co-execution at all, `SQ_VALU_MFMA_COEXEC_CYCLES` = 0: use `--mfma-hold 32`,
with which the co-simulated training step matches the measured one,
profiles/r4_step_isa_timeline.md), dependent result 40; VALU issue 4 (transcendental 8, f64 8),
result 8; `ds_read*` 64 (+16 for b128), `ds_write` 4 issue; LDS returns in
order (`lgkmcnt`); global loads 500 (L2 / MALL resident chunks); SALU 2;
`s_nop N` 4(N+1); `s_barrier` releases at its issue (the other waves are not
modelled: barrier waits are reported as measured by the stamped build,
profiles/r3_train_hw_experiments.md).  The helper wave that shares the SIMD
is not modelled either: its MFMAs and VALU compete for the same issue slots,
so the simulated step is a lower bound for the wave's own chain.

  hipcc ... -gline-tables-only --cuda-device-only -S fedmx_train_hw.hip -o k.s
  python scripts/isa_timeline.py k.s --kernel train_kernel_hwILb0ELb0 --cosim --mfma-hold 32 --lds-bw 64 --lds-queue 16
"""
from __future__ import annotations

import argparse
import collections
import re
import sys

MFMA_PIPE = {"v_mfma_f32_16x16x4_f32": (32, 40), "v_mfma_f32_32x32x2_f32": (64, 64)}
TRANS = ("v_rcp", "v_sqrt", "v_rsq", "v_exp", "v_log", "v_sin", "v_cos", "v_rcp_iflag")
LDS_LAT, LDS_B128, GLOBAL_LAT, VALU_LAT = 64, 16, 500, 8

_reg = re.compile(r"\b([vsa])\[(\d+):(\d+)\]|\b([vsa])(\d+)\b|\b(vcc|exec|scc|m0)\b")


def regs(text: str):
    out = []
    for m in _reg.finditer(text):
        if m.group(1):
            out += [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
        elif m.group(4):
            out.append(f"{m.group(4)}{m.group(5)}")
        else:
            out.append(m.group(6))
    return out


def split_operands(ops: str):
    parts, depth, cur = [], 0, ""
    for ch in ops:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur.strip())
    return parts


MFMA_VPORT_HOLD = 8   # cycles an MFMA holds the SIMD's vector issue (--mfma-hold)


def classify(op: str):
    """(kind, issue cycles, result latency)."""
    if op in MFMA_PIPE:
        return "mfma", MFMA_VPORT_HOLD, MFMA_PIPE[op][1]
    if op.startswith("ds_read") or op.startswith("ds_bpermute") or op.startswith("ds_swizzle") \
            or op.startswith("ds_permute") or op.startswith("ds_load"):
        return "lds_read", 4, LDS_LAT + (LDS_B128 if "b128" in op else 0)
    if op.startswith("ds_"):
        return "lds_write", 4, 0
    if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vmem_load", 4, GLOBAL_LAT
    if op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store", "global_atomic")):
        return "vmem_store", 4, 0
    if op.startswith(("s_nop", "s_sleep")):
        return "nop", 4, 0
    if op.startswith("s_waitcnt"):
        return "wait", 0, 0
    if op == "s_barrier":
        return "barrier", 4, 0
    if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
        return "valu", 4, VALU_LAT
    if op.startswith("v_"):
        if op.startswith(TRANS) or "_f64" in op:
            return "valu", 8, VALU_LAT + 4
        if op.startswith("v_pk_"):
            return "valu", 8, VALU_LAT
        return "valu", 4, VALU_LAT
    if op.startswith("s_"):
        return "salu", 2, 2
    return "other", 4, 4


NO_DEST = ("ds_write", "ds_store", "global_store", "buffer_store", "flat_store", "scratch_store", "s_cbranch",
           "s_branch", "s_waitcnt", "s_barrier", "s_nop", "s_sleep", "s_setprio", "s_cmp", "v_cmpx", "s_memtime",
           "s_sendmsg", "ds_nop", "s_endpgm")


def parse(lines):
    """[(op, dests, srcs, line, raw)] of instruction lines; tracks .loc."""
    out, loc = [], None
    for raw in lines:
        s = raw.split(";")[0].strip()
        if s.startswith(".loc"):
            p = s.split()
            loc = (int(p[1]), int(p[2]))
            continue
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        op, _, rest = s.partition(" ")
        ops = split_operands(rest)
        if op.startswith(NO_DEST) or not ops:
            dests, srcs = [], regs(rest)
        else:
            dests, srcs = regs(ops[0]), regs(",".join(ops[1:]))
        if op.startswith("v_cmp_") and not op.endswith("_e64"):
            dests = ["vcc"]
        if op.startswith(("s_cmp", "s_bitcmp")):
            dests = ["scc"]
        if op.startswith("v_cndmask_b32") and len(ops) == 3:
            srcs.append("vcc")
        if op.startswith("v_mfma"):
            srcs += dests   # accumulator read
        out.append((op, dests, srcs, loc, s))
    return out


def simulate(instrs, wait_lds_extra=0):
    t = 0
    ready = collections.defaultdict(int)
    mfma_free = 0
    lds_q, vm_q = [], []   # completion times, issue order
    rows = []
    for op, dests, srcs, loc, raw in instrs:
        kind, cost, lat = classify(op)
        earliest, why = t, "in-order"
        for r in srcs:
            if ready[r] > earliest:
                earliest, why = ready[r], f"operand {r}"
        if kind == "mfma" and mfma_free > earliest:
            earliest, why = mfma_free, "matrix pipe busy"
        if kind == "wait":
            m_l = re.search(r"lgkmcnt\((\d+)\)", raw)
            m_v = re.search(r"vmcnt\((\d+)\)", raw)
            if m_l:
                n = int(m_l.group(1))
                pend = [c for c in lds_q if c > t]
                if len(pend) > n:
                    c = sorted(pend)[len(pend) - n - 1]
                    if c > earliest:
                        earliest, why = c + wait_lds_extra, "lgkmcnt"
            if m_v:
                n = int(m_v.group(1))
                pend = [c for c in vm_q if c > t]
                if len(pend) > n:
                    c = sorted(pend)[len(pend) - n - 1]
                    if c > earliest:
                        earliest, why = c, "vmcnt"
        issue = earliest
        if kind == "nop":
            m = re.match(r"s_nop\s+(\d+)", raw)
            cost = 4 * (int(m.group(1)) + 1) if m else 4
        stall = issue - t
        t = issue + cost
        if kind == "mfma":
            mfma_free = issue + MFMA_PIPE[op][0]
        done = issue + lat
        if kind == "lds_read":
            done = max(done, (lds_q[-1] if lds_q else 0) + 4)   # in-order return
            lds_q.append(done)
        elif kind == "lds_write":
            lds_q.append(issue + 32)
        elif kind == "vmem_load":
            done = max(done, (vm_q[-1] if vm_q else 0) + 4)
            vm_q.append(done)
        elif kind == "vmem_store":
            vm_q.append(issue + 200)
        for r in dests:
            ready[r] = done if kind in ("lds_read", "vmem_load", "mfma", "valu", "salu") else issue + lat
        rows.append(dict(op=op, kind=kind, issue=issue, stall=stall, why=why if stall else "", loc=loc, raw=raw))
    return rows, t


class _Wave:
    def __init__(self, body, name):
        self.body, self.name = body, name
        self.pc, self.t_next = 0, 0
        self.ready = collections.defaultdict(int)
        self.lds_q, self.vm_q = [], []
        self.stall = collections.Counter()
        self.arrived = self.passed = 0
        self.iters = 0
        self.iter_start = [0]


def lds_bytes(op: str) -> int:
    """Bytes one wave64 LDS instruction moves."""
    m = re.search(r"b(\d+)", op)
    width = int(m.group(1)) // 8 if m else 4
    if "write2" in op or "read2" in op:
        width *= 2
    return 64 * width


def cosim(bodies, names, iters=6, max_cycles=2_000_000, lds_bw=0.0, lds_queue=None):
    """Cycle-stepped co-simulation of the waves sharing ONE SIMD (the main
    wave and its helper): one matrix pipe, one vector issue port (VALU issue
    4 cycles, an MFMA holds it 8), per-wave in-order issue, priority by age
    (the first body first), and the loop's workgroup barriers joined by both
    (the waves on the other SIMDs are taken to arrive with them).  lds_bw > 0:
    this SIMD's share of the CU's LDS bandwidth in bytes per cycle (the other
    three SIMDs taken to run the same stream), shared by both waves.
    lds_queue (cycles, with lds_bw): an LDS instruction cannot issue while
    the SIMD's LDS backlog exceeds it -- the wave stalls at issue, and so
    does everything behind it in program order (SQ_WAIT_INST_LDS)."""
    ws = [_Wave(b, n) for b, n in zip(bodies, names)]
    mfma_free = vport_free = lds_free = 0
    t = 0
    while t < max_cycles and min(w.iters for w in ws) < iters:
        for w in ws:
            if w.iters >= iters or w.t_next > t:
                continue
            op, dests, srcs, loc, raw = w.body[w.pc]
            kind, cost, lat = classify(op)
            why = None
            for r in srcs:
                if w.ready[r] > t:
                    why = "operand"
                    break
            if why is None and kind in ("valu", "mfma") and vport_free > t:
                why = "vector port (other wave)"
            if why is None and kind == "mfma" and mfma_free > t:
                why = "matrix pipe busy"
            if why is None and lds_queue is not None and kind in ("lds_read", "lds_write") and lds_free - t > lds_queue:
                why = "LDS issue (queue full)"
            if why is None and kind == "wait":
                for cnt, q in (("lgkmcnt", w.lds_q), ("vmcnt", w.vm_q)):
                    m = re.search(cnt + r"\((\d+)\)", raw)
                    if m and sum(1 for c in q if c > t) > int(m.group(1)):
                        why = cnt
            if why is None and kind == "barrier":
                if w.arrived <= w.passed:
                    w.arrived += 1   # this wave's (passed + 1)-th barrier
                if min(x.arrived for x in ws) < w.arrived:
                    why = "barrier"
                else:
                    w.passed += 1
            if why is not None:
                if why == "operand":
                    prod = max((r for r in srcs), key=lambda r: w.ready[r])
                    why = f"operand ({w.ready.get('_k_' + prod, '?')})"
                w.stall[why] += 1
                continue
            if kind == "nop":
                m = re.match(r"s_(nop|sleep)\s+(\d+)", raw)
                cost = (4 * (int(m.group(2)) + 1) if m.group(1) == "nop" else 64 * int(m.group(2))) if m else 4
            w.t_next = t + max(cost, 1)
            if kind in ("valu", "mfma"):
                vport_free = t + cost
            if kind == "mfma":
                mfma_free = t + MFMA_PIPE[op][0]
            done = t + lat
            if kind in ("lds_read", "lds_write") and lds_bw > 0:
                occ = lds_bytes(op) / lds_bw
                lds_free = max(t, lds_free) + occ
                done = lds_free + lat
            if kind == "lds_read":
                done = max(done, (w.lds_q[-1] if w.lds_q else 0) + 4)
                w.lds_q.append(done)
            elif kind == "lds_write":
                w.lds_q.append(max(t + 32, lds_free + 32 if lds_bw > 0 else 0))
            elif kind == "vmem_load":
                done = max(done, (w.vm_q[-1] if w.vm_q else 0) + 4)
                w.vm_q.append(done)
            elif kind == "vmem_store":
                w.vm_q.append(t + 200)
            for r in dests:
                w.ready[r] = done
                w.ready["_k_" + r] = kind
            w.pc += 1
            if w.pc == len(w.body):
                w.pc = 0
                w.iters += 1
                w.iter_start.append(t)
        t += 1
    return ws


def find_kernel(lines, name):
    st = next(i for i, l in enumerate(lines) if l.startswith("_Z") and name in l.split(":")[0])
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return st, en


def loops(lines, st, en):
    lab = {}
    for i in range(st, en):
        m = re.match(r"^(\.LBB\d+_\d+):", lines[i])
        if m:
            lab[m.group(1)] = i
    out = []
    for i in range(st, en):
        m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", lines[i])
        if m and m.group(1) in lab and lab[m.group(1)] < i:
            seg = lines[lab[m.group(1)]:i + 1]
            out.append(dict(label=m.group(1), start=lab[m.group(1)], end=i,
                            mfma=sum("v_mfma" in s for s in seg),
                            barriers=sum(s.strip() == "s_barrier" for s in seg)))
    return out


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("asm")
    p.add_argument("--kernel", default="train_kernel_hwILb0")
    p.add_argument("--loop", default="auto", help="label, or auto = innermost loop with 2 barriers, most MFMAs")
    p.add_argument("--top", type=int, default=25)
    p.add_argument("--lds-bw", type=float, default=0.0,
                   help="co-simulation: this SIMD's LDS bandwidth share, bytes/cycle (0: unlimited)")
    p.add_argument("--lds-queue", type=float, default=None,
                   help="co-simulation with --lds-bw: LDS backlog (cycles) above which an LDS instruction stalls at issue")
    p.add_argument("--mfma-hold", type=int, default=None,
                   help="cycles an MFMA holds the vector issue port (default 8; 32 = no VALU co-execution)")
    p.add_argument("--cosim", action="store_true",
                   help="also co-simulate the main loop with the helper loop (the 2-barrier loop with fewest MFMAs)")
    a = p.parse_args(argv)
    if a.mfma_hold is not None:
        global MFMA_VPORT_HOLD
        MFMA_VPORT_HOLD = a.mfma_hold
    lines = open(a.asm).read().split("\n")
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
        if m:
            files[int(m.group(1))] = m.group(2).split("/")[-1]
    st, en = find_kernel(lines, a.kernel)
    ls = loops(lines, st, en)
    if a.loop == "auto":
        cand = [x for x in ls if x["barriers"] == 2]
        lp = max(cand, key=lambda x: (x["mfma"], -(x["end"] - x["start"])))
    else:
        lp = next(x for x in ls if x["label"] == a.loop)
    body = parse(lines[lp["start"]:lp["end"] + 1])
    # two passes: the second starts with the registers / queues the first left
    rows, t = simulate(body + body)
    n = len(body)
    rows = rows[n:]
    t0 = rows[0]["issue"] - rows[0]["stall"]
    step = t - t0
    kinds = collections.Counter()
    stall_by = collections.Counter()
    for r in rows:
        kinds[r["kind"]] += 1
        if r["stall"]:
            cause = r["why"]
            if cause.startswith("operand"):
                # the producer kind of that operand
                reg = cause.split()[1]
                prod = next((q["kind"] for q in reversed(rows[:rows.index(r)]) if reg in
                             regs(split_operands(q["raw"].partition(" ")[2])[0] if q["raw"].partition(" ")[2]
                                  else "")), "previous step")
                cause = f"waits on {prod} result"
            stall_by[cause] += r["stall"]
    barriers = [i for i, r in enumerate(rows) if r["kind"] == "barrier"]
    print(f"loop {lp['label']} (asm lines {lp['start'] + 1}-{lp['end'] + 1}): {n} instructions, "
          f"{lp['mfma']} MFMA, {lp['barriers']} barriers")
    print(f"simulated step (one wave, barriers free): {step} cycles")
    print("instruction mix:", dict(kinds))
    busy = sum(classify(r["op"])[1] if r["kind"] != "nop" else 0 for r in rows)
    print(f"issue cycles (no stalls): {busy}; stall cycles: {sum(r['stall'] for r in rows)}")
    print("stall by cause:")
    for k, v in stall_by.most_common():
        print(f"  {k:34s} {v:6d}  ({100 * v / step:.1f} %)")
    seg_edges = [0] + [b + 1 for b in barriers] + [len(rows)]
    print("segments between barriers (issue span, MFMA, stall):")
    for s0, s1 in zip(seg_edges[:-1], seg_edges[1:]):
        seg = rows[s0:s1]
        if not seg:
            continue
        span = seg[-1]["issue"] - (seg[0]["issue"] - seg[0]["stall"])
        print(f"  instr {s0:4d}-{s1 - 1:4d}: {span:6d} cycles, {sum(r['kind'] == 'mfma' for r in seg):3d} MFMA, "
              f"stall {sum(r['stall'] for r in seg):6d}")
    # SIMD issue work (what an issue-bound step is made of): MFMA x hold +
    # VALU issue cycles, per barrier segment and per source line
    def work(r):
        k, cost, _ = classify(r["op"])
        return MFMA_PIPE[r["op"]][0] if k == "mfma" and MFMA_VPORT_HOLD >= 32 else (cost if k in ("mfma", "valu") else 0)
    print(f"SIMD issue work of this wave (MFMA hold {MFMA_VPORT_HOLD}): {sum(work(r) for r in rows)} cycles; by segment: " +
          ", ".join(str(sum(work(r) for r in rows[s0:s1])) for s0, s1 in zip(seg_edges[:-1], seg_edges[1:])))
    by_work = collections.Counter()
    for r in rows:
        if r["loc"]:
            by_work[(files.get(r["loc"][0], r["loc"][0]), r["loc"][1])] += work(r)
    print(f"top {a.top} source lines by SIMD issue work:")
    for (f, ln), v in by_work.most_common(a.top):
        print(f"  {f}:{ln:<5d} {v:6d}")
    by_loc = collections.Counter()
    for r in rows:
        if r["stall"] and r["loc"]:
            by_loc[(files.get(r["loc"][0], r["loc"][0]), r["loc"][1])] += r["stall"]
    print(f"top {a.top} source lines by stall cycles:")
    for (f, ln), v in by_loc.most_common(a.top):
        print(f"  {f}:{ln:<5d} {v:6d}")
    print(f"top {a.top} single stalls:")
    for r in sorted(rows, key=lambda r: -r["stall"])[:a.top]:
        loc = f"{files.get(r['loc'][0], r['loc'][0])}:{r['loc'][1]}" if r["loc"] else "-"
        print(f"  {r['stall']:5d} @ {r['issue'] - t0:6d}  {r['why']:22s} {loc:28s} {r['raw'][:70]}")
    if a.cosim:
        hl = min((x for x in ls if x["barriers"] == 2 and x is not lp and x["mfma"] < lp["mfma"]),
                 key=lambda x: (x["mfma"], x["end"] - x["start"]))
        hbody = parse(lines[hl["start"]:hl["end"] + 1])
        # both loops start right after their barrier #2 ... rotate each body so
        # it starts at its first barrier (same point of the step for both roles)
        def rot(b):
            i = next(k for k, x in enumerate(b) if x[0] == "s_barrier")
            return b[i:] + b[:i]
        ws = cosim([rot(body), rot(hbody)], ["main", "helper"], lds_bw=a.lds_bw, lds_queue=a.lds_queue)
        print(f"co-simulation on one SIMD: main loop {lp['label']} + helper loop {hl['label']} "
              f"({hl['mfma']} MFMA)")
        for w in ws:
            per = [b - a_ for a_, b in zip(w.iter_start[2:], w.iter_start[3:])]
            print(f"  {w.name}: cycles per step (iterations 3..): {per}")
            tot = sum(w.stall.values())
            print(f"    stalled-cycle causes over {w.iters} steps: " +
                  ", ".join(f"{k} {100 * v / tot:.0f}%" for k, v in w.stall.most_common()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
