#!/bin/bash
# Round-4 GPU check: the GPU test tier, then the headline bench and the paper
# configuration, each under its own time limit; stops at the first failure.
set -u
OUT=${1:-gpurun_out/r4}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread ${PYTEST_EXTRA:-} \
  > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; tail -n 30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -n 3 "$OUT/pytest_gpu.txt"
timeout -k 10 180 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -n 20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 180 python bench.py --epochs 100 --lr 1e-5 --shrink-lambda 10 --steps 10 --warmup 2 \
  > "$OUT/paper.json" 2>> "$OUT/bench.err" || { echo "paper rc=$?"; exit 1; }
cat "$OUT/paper.json"
