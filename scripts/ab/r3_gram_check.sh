#!/bin/bash
# Round 3: Gram-form training step -- training-kernel GPU tests, the A/B
# timing of gram0 (round-2 step) vs gram1 (Gram form) via scripts/ab_train.sh,
# then the Gram form's per-stage stamps.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "train" \
  > gpurun_out/gram_kt.log 2>&1
rc=$?
tail -n 22 gpurun_out/gram_kt.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 bash scripts/ab_train.sh || exit $?
timeout -k 10 120 python -u scripts/train_stamps.py --lib libfedmx_hip_stamps_gram1.so --gram > gpurun_out/stamps_gram1.log 2>&1 || exit $?
head -n 24 gpurun_out/stamps_gram1.log
