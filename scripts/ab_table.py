"""Markdown table of a scripts/ab_train.sh run (gpurun_out/ab/<lib>.<rep>.log).

  python scripts/ab_table.py gpurun_out/ab [--base libfedmx_hip_base]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
from collections import defaultdict


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--base", default="libfedmx_hip_base")
    a = p.parse_args(argv)
    runs = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(a.dir, "*.log"))):
        name, rep = os.path.basename(f)[:-4].rsplit(".", 1)
        try:
            rec = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        runs[name].append((int(rep), rec))
    if not runs:
        print("no records")
        return 1
    base = runs.get(a.base)
    b_tr = sum(r["train_launch_us"] for _, r in base) / len(base) if base else None
    print("| variant | train launch us (per pass) | vs base | FedProx launch us | 1-client launch us |")
    print("|---|---|---|---|---|")
    for name, rs in sorted(runs.items()):
        rs.sort()
        tr = [r["train_launch_us"] for _, r in rs]
        mean = sum(tr) / len(tr)
        rel = f"{100 * (mean / b_tr - 1):+.1f} %" if b_tr else "-"
        px = " / ".join(f"{r.get('train_launch_fedprox_us', float('nan')):.1f}" for _, r in rs)
        one = " / ".join(f"{r.get('train_launch_1client_us', float('nan')):.1f}" for _, r in rs)
        print(f"| {name.replace('libfedmx_hip_', '')} | {' / '.join(f'{x:.1f}' for x in tr)} | {rel} | {px} | {one} |")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
