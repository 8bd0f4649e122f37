#!/bin/bash
# A/B of the built variant libraries (scripts/ab_variants.py build ...): the
# helper-vs-4-wave bit-identity and torch-parity kernel tests under each
# numerics-preserving variant, then train-launch timing (scripts/ab_train.sh).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/ab
mkdir -p "$OUT"
for v in ${AB_CHECK:-flags}; do
  FEDMX_HIP_LIB=$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip_$v.so timeout -k 10 300 \
    python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "helper_waves or matches_torch_engine or single_step" > "$OUT/check_$v.txt" 2>&1 \
    || { echo "check $v failed"; tail -n 30 "$OUT/check_$v.txt"; exit 1; }
  echo "check $v: $(tail -n 1 "$OUT/check_$v.txt")"
done
bash scripts/ab_train.sh
