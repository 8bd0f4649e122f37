#!/bin/bash
# GPU side of profiles/r4_adoption_ablation.md: adoption vs local-only ablation
# at 10 / 64 / 256 clients, IID and non-IID, 50 rounds (HIP engine), plus the
# relative drift limit.
set -u
OUT=${1:-gpurun_out/r4_adoption}
mkdir -p "$OUT"
rm -f "$OUT/adoption.jsonl"
timeout -k 10 500 python -u scripts/adoption_ablation.py --clients 10 64 256 --rounds 50 \
  --out "$OUT/adoption.jsonl" || exit 1
timeout -k 10 300 python -u scripts/adoption_ablation.py --clients 10 64 256 --rounds 50 --modes aggregate \
  --drift-rel 0.25 --out "$OUT/adoption.jsonl" || exit 1
wc -l "$OUT/adoption.jsonl"
