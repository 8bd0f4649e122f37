"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into markdown.

Usage: python scripts/prof_summary.py gpurun_out/prof/run_results.db [--title T] [--out profiles/x.md]

Prints per-kernel totals (calls, total/avg/min/max us, share, VGPR/AGPR/SGPR,
LDS, scratch) and, for the last bench round, the per-round kernel timeline
(span from the first to the last kernel of one train->eval round), and the
median inter-round gap on the main stream (verification end -> next
training start).
"""
from __future__ import annotations

import argparse
import sqlite3
import sys


def _short(name: str, n: int = 70) -> str:
    s = name.replace("void ", "")
    s = s.split("(")[0] if "fedmx" in s else s
    return s if len(s) <= n else s[: n - 3] + "..."


POLLING = ("side_wait_kernel",)


def summarize(db: str, title: str) -> str:
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, duration, grid_x, grid_y, workgroup_x, lds_size, scratch_size, "
                     "vgpr_count, accum_vgpr_count, sgpr_count from kernels order by start").fetchall()
    out = [f"# {title}", "", f"source: `{db}` (rocprofv3 --kernel-trace --stats)", ""]
    agg = {}
    for r in rows:
        a = agg.setdefault(r[0], dict(n=0, tot=0.0, mn=1e30, mx=0.0, meta=r[4:]))
        d = r[3] / 1000.0
        a["n"] += 1
        a["tot"] += d
        a["mn"] = min(a["mn"], d)
        a["mx"] = max(a["mx"], d)
    # polling kernels (a lane that sleeps between loads while the round runs,
    # e.g. side_wait_kernel) are not GPU work: kept out of the % column
    polling = [n for n in agg if any(p in n for p in POLLING)]
    total = sum(a["tot"] for n, a in agg.items() if n not in polling) or 1.0
    out += ["| kernel | calls | total us | avg us | min us | max us | % (polling kernels excluded) | grid | VGPR/AGPR/SGPR "
            "| LDS B | scratch B |",
            "|---|---|---|---|---|---|---|---|---|---|---|"]
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["tot"]):
        gx, gy, wg, lds, scr, vg, ag, sg = a["meta"]
        share = "polling" if name in polling else f"{100 * a['tot'] / total:.1f}"
        out.append(f"| `{_short(name)}` | {a['n']} | {a['tot']:.1f} | {a['tot'] / a['n']:.1f} | {a['mn']:.1f} | "
                   f"{a['mx']:.1f} | {share} | {gx // max(wg, 1)}x{gy} | {vg}/{ag}/{sg} | {lds} | {scr} |")
    # last round: from the last train_kernel launch to the end of the next auc kernel
    starts = [i for i, r in enumerate(rows) if "train_kernel" in r[0]]
    if starts:
        i0 = starts[-2] if len(starts) > 1 else starts[-1]
        i1 = starts[-1] if len(starts) > 1 else len(rows)
        seg = rows[i0:i1]
        t0 = seg[0][1]
        out += ["", f"## one round timeline (kernels {i0}..{i1 - 1}, span {(seg[-1][2] - t0) / 1000:.1f} us, "
                f"busy {sum(r[3] for r in seg) / 1000:.1f} us)", "",
                "| t0 us | dur us | gap before us | kernel |", "|---|---|---|---|"]
        prev_end = t0
        for r in seg:
            out.append(f"| {(r[1] - t0) / 1000:.1f} | {r[3] / 1000:.1f} | {(r[1] - prev_end) / 1000:.1f} | `{_short(r[0])}` |")
            prev_end = r[2]
    # the inter-round gap on the main stream: the end of each round's last
    # protocol kernel (verification) to the start of the next training launch
    gaps, last_v = [], None
    for r in rows:
        if "verify" in r[0] or "decide_adopt" in r[0]:
            last_v = r[2]
        elif "train_kernel" in r[0] and last_v is not None:
            gaps.append((r[1] - last_v) / 1000.0)
            last_v = None
    if gaps:
        g = sorted(gaps)
        out += ["", f"inter-round gap (verification end -> next training start): median {g[len(g) // 2]:.1f} us, "
                f"min {g[0]:.1f}, max {g[-1]:.1f} over {len(g)} rounds"]
    return "\n".join(out) + "\n"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    ap.add_argument("--out", default=None)
    ap.add_argument("--pmc", action="store_true", help="the database holds PMC counters")
    ap.add_argument("--kernel", default="", help="only kernels whose name contains this")
    a = ap.parse_args(argv)
    text = (f"# {a.title}\n\nsource: `{a.db}`\n\n" + pmc_summary(a.db, a.kernel)) if a.pmc else summarize(a.db, a.title)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    sys.stdout.write(text)


def pmc_summary(db: str, kernel_substr: str = "") -> str:
    """Per-kernel PMC counter totals (and per-dispatch means) from a --pmc run."""
    c = sqlite3.connect(db)
    cols = [d[0] for d in c.execute("select * from pmc_events limit 1").description or []]
    if "dispatch_id" in cols and "name" in cols:
        # rocpd views that carry the dispatch and kernel name on every counter row
        rows = c.execute("select name, counter_name, sum(counter_value), count(distinct dispatch_id) "
                         "from pmc_events group by name, counter_name").fetchall()
    else:
        rows = c.execute("select k.name, p.counter_name, sum(p.counter_value), count(distinct k.id) "
                         "from pmc_events p join kernels k on p.event_id = k.id "
                         "group by k.name, p.counter_name").fetchall()
    out = ["| kernel | counter | total | per dispatch |", "|---|---|---|---|"]
    for name, cn, v, n in sorted(rows):
        if kernel_substr and kernel_substr not in name:
            continue
        out.append(f"| `{_short(name, 40)}` | {cn} | {v:.0f} | {v / max(n, 1):.0f} |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    main()
