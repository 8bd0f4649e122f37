#!/bin/bash
# Training-kernel iteration on the GPU box: numerics tests of the working-tree
# kernels, same-box A/B of every libfedmx_hip_<name>.so (scripts/ab_train.sh),
# phase stamps of the working tree, then the headline bench.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py -x -q --timeout 200 \
  --timeout-method thread > "$OUT/kernels_tests.log" 2>&1 || { echo "tests rc=$?"; tail -20 "$OUT/kernels_tests.log"; exit 1; }
tail -2 "$OUT/kernels_tests.log"
bash scripts/ab_train.sh || exit $?
timeout -k 10 300 python scripts/train_stamps.py --json "$OUT/stamps.json" > "$OUT/stamps.log" 2>&1 || exit $?
head -22 "$OUT/stamps.log"
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log"
