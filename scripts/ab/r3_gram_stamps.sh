#!/bin/bash
# Round 3: per-stage s_memtime stamps of the Gram-form and round-2 helper-wave steps.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/train_stamps.py --lib libfedmx_hip_stamps_gram1.so --gram > gpurun_out/stamps_gram1.log 2>&1 || exit $?
head -n 24 gpurun_out/stamps_gram1.log
timeout -k 10 120 python -u scripts/train_stamps.py --lib libfedmx_hip_stamps_gram0.so > gpurun_out/stamps_gram0.log 2>&1 || exit $?
head -n 24 gpurun_out/stamps_gram0.log
