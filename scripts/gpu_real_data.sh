#!/bin/bash
# Real N-BaIoT IID-10 CSVs (copied into data_cache/, not tracked): the paper
# configuration's six combinations at 50 % participation, then SAE-CEN +
# MSEAvg against the client ratio (50-100 %), HIP engine, compat fixed.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python -u scripts/real_data_paper.py --data-root data_cache/nbaiot_iid10 \
  > "$OUT/real_paper_combos.jsonl" 2> "$OUT/real_paper_combos.err" || { echo "combos rc=$?"; tail "$OUT/real_paper_combos.err"; exit 1; }
cat "$OUT/real_paper_combos.jsonl"
timeout -k 10 600 python -u scripts/real_data_paper.py --data-root data_cache/nbaiot_iid10 --combos hybrid:mse_avg \
  --participation 0.5 0.6 0.7 0.8 0.9 1.0 > "$OUT/real_ratio.jsonl" 2> "$OUT/real_ratio.err" || { echo "ratio rc=$?"; tail "$OUT/real_ratio.err"; exit 1; }
cat "$OUT/real_ratio.jsonl"
