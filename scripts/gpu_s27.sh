#!/bin/bash
# Round-6 epoch-end publication without thread 0's second drain (FedProx
# partials drained with the payload): the async-validation and FedProx
# numerics tests, then an A/B of the training launches and the bench against
# the previous library (libfedmx_hip_prev.so, built from the previous commit).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/${TAG:-s27}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_async_validation_gpu.py \
  tests/test_train_failure_gpu.py tests/test_kernels_gpu.py > $OUT/pytest.log 2>&1 \
  || { echo tests failed; tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
OUTAB=$OUT/ab AB_LIBS="main prev" AB_REPS=2 bash scripts/ab_train.sh > $OUT/ab_train.log 2>&1 || { echo ab_train failed; tail $OUT/ab_train.log; exit 1; }
grep -E "^[12] " $OUT/ab_train.log | cut -c1-150
TAG=$(basename $OUT)/bench_ab AB_LIBS="main prev" REPS=2 LONG=200 bash scripts/bench_ab.sh
