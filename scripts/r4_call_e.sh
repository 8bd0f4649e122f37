#!/bin/bash
# Round-4: helper-wave kernel for batches over 12 rows (16-row chunks):
# the training-kernel GPU tests, then launch timing incl. batch 64.
set -u
mkdir -p gpurun_out/r4e
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4e/pytest_kernels.txt 2>&1 || { echo "pytest rc=$?"; tail -n 40 gpurun_out/r4e/pytest_kernels.txt; exit 1; }
tail -n 2 gpurun_out/r4e/pytest_kernels.txt
for rep in 1 2; do
  timeout -k 10 120 python scripts/bench_kernels.py --train-only --reps 15 > gpurun_out/r4e/train_kernel.$rep.json \
    2> gpurun_out/r4e/train_kernel.err || { echo "bench_kernels rc=$?"; tail -n 20 gpurun_out/r4e/train_kernel.err; exit 1; }
  cat gpurun_out/r4e/train_kernel.$rep.json
done
rm -rf gpurun_out/ab
AB_REPS=2 AB_CHECK="noiglp iglp1" bash scripts/r4_ab.sh || exit 1
