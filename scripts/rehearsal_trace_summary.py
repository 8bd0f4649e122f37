"""Merge the per-rank rocprofv3 kernel traces of a one-GPU multi-rank
rehearsal (scripts/rehearsal_trace.sh) into one device timeline: where a
round's wall time goes when N processes share the GPU -- each rank's own
kernels, the other ranks' kernels (time slicing), the peer-memory exchange's
push / wait kernels, and time with no kernel of any rank running.

    python scripts/rehearsal_trace_summary.py gpurun_out/reh8 [--out summary.md]
"""
from __future__ import annotations

import argparse
import glob
import os
import sqlite3
import sys


def load(d):
    ranks = {}
    for db in sorted(glob.glob(os.path.join(d, "rank*", "**", "*.db"), recursive=True)):
        r = int(db.split("rank")[1].split(os.sep)[0])
        c = sqlite3.connect(db)
        ranks[r] = c.execute("select name, start, end from kernels order by start").fetchall()
    return ranks


def union_len(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def kind(name):
    if "ipc_" in name:
        return "exchange (ipc push / wait)"
    if "train_kernel" in name:
        return "training"
    if any(k in name for k in ("fwd_rows", "score_reduce", "elect", "verify", "decide")):
        return "vote / election / verification"
    if any(k in name for k in ("auc", "cen_score", "copy2", "copy_f64")):
        return "evaluation + copies"
    return "other"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    ranks = load(a.dir)
    if not ranks:
        raise SystemExit("no traces")
    # the timed window: rank 0's last 20 training launches (bench: steps after warm-up)
    tr0 = [k for k in ranks[0] if "train_kernel" in k[0]]
    t_lo, t_hi = tr0[-20][1] if len(tr0) >= 20 else tr0[0][1], ranks[0][-1][2]
    span = t_hi - t_lo
    out = [f"# One-GPU rehearsal, {len(ranks)} ranks: merged kernel trace", "",
           f"source: `{a.dir}/rank*/` (rocprofv3 --kernel-trace per rank); window: rank 0's last 20 training "
           f"launches to its last kernel, {span / 1e6:.2f} ms", ""]
    allk = [(s, e, r, n) for r, ks in ranks.items() for n, s, e in ks if e > t_lo and s < t_hi]
    busy_any = union_len([(max(s, t_lo), min(e, t_hi)) for s, e, _, _ in allk])
    out += [f"* device busy (any rank's kernel running): {busy_any / 1e6:.2f} ms = {100 * busy_any / span:.1f} % "
            f"of the window; idle {(span - busy_any) / 1e6:.2f} ms", ""]
    out += ["| rank | kernels | own busy ms (union) | training ms | exchange ms | vote/elect/verify ms | eval ms |",
            "|---|---|---|---|---|---|---|"]
    for r in sorted(ranks):
        mine = [(max(s, t_lo), min(e, t_hi), n) for s, e, rr, n in allk if rr == r]
        by = {}
        for s, e, n in mine:
            by[kind(n)] = by.get(kind(n), 0) + (e - s)
        out.append(f"| {r} | {len(mine)} | {union_len([(s, e) for s, e, _ in mine]) / 1e6:.2f} | "
                   f"{by.get('training', 0) / 1e6:.2f} | {by.get('exchange (ipc push / wait)', 0) / 1e6:.2f} | "
                   f"{by.get('vote / election / verification', 0) / 1e6:.2f} | "
                   f"{by.get('evaluation + copies', 0) / 1e6:.2f} |")
    # exchange kernels: how much of their duration is spent while OTHER ranks' non-exchange kernels run
    ex = [(max(s, t_lo), min(e, t_hi), r) for s, e, r, n in allk if "ipc_" in n]
    ex_tot = sum(e - s for s, e, _ in ex)
    out += ["", f"* exchange kernels (all ranks, summed durations): {ex_tot / 1e6:.2f} ms; "
            f"training kernels (all ranks): {sum(e - s for s, e, _, n in allk if 'train_kernel' in n) / 1e6:.2f} ms",
            ""]
    text = "\n".join(out) + "\n"
    if a.out:
        open(a.out, "w").write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
