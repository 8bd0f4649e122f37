#!/bin/bash
# Round-4 GPU call A: MFMA chain probe, GPU test tier + bench + paper config,
# then the kernel A/B (HW_SPLIT / RED8 bit-identity, train-launch timing).
set -u
mkdir -p gpurun_out/r4b
timeout -k 10 60 scripts/probes/mfma_chain > gpurun_out/r4b/mfma_chain.json || { echo "probe rc=$?"; exit 1; }
cat gpurun_out/r4b/mfma_chain.json
bash scripts/r4_exact_diag.sh || exit 1
PYTEST_EXTRA="--deselect tests/test_long_horizon_gpu.py::test_exact_adam_build_matches_torch_oracle" \
  bash scripts/r4_gpu_check.sh gpurun_out/r4b || exit 1
# (the hwsplit / red8 A/B variants of this call were removed from the kernel after it; profiles/r4_ab_logs2)
