#!/bin/bash
# A/B two builds of the HIP library on the training-kernel microbenchmark:
#   bash scripts/ab/ab_lib.sh <alt .so path>
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
python -c "import fedmse_decentralized_amd.ops.build as b; b.build_all()" || exit 3
timeout -k 10 300 python scripts/bench_kernels.py > "$OUT/bk_default.log" 2>&1 || exit $?
FEDMX_HIP_LIB=$1 timeout -k 10 300 python scripts/bench_kernels.py > "$OUT/bk_alt.log" 2>&1 || exit $?
tail -n 1 "$OUT/bk_default.log" | cut -c1-120
tail -n 1 "$OUT/bk_alt.log" | cut -c1-120
