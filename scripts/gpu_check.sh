#!/bin/bash
# One GPU-box call: the GPU tests named in $TESTS (default: the kernel and
# long-horizon numerics), then the train-kernel A/B of $AB_LIBS
# (scripts/ab_train.sh).  Logs under gpurun_out/$TAG/.  A test run that ends
# in anything but pass (0) or test failure (1) -- a fault, abort or time
# limit -- ends the call before the timing starts.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${TAG:-check}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
TESTS=${TESTS:-"tests/test_kernels_gpu.py tests/test_long_horizon_gpu.py"}
if [ "$TESTS" != none ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${PYTEST_X--x} -v --timeout 600 --timeout-method thread $TESTS \
    > "$OUT/tests.log" 2>&1
  rc=$?
  tail -n 5 "$OUT/tests.log"
  grep -h "long-horizon\|exact-adam" "$OUT/tests.log" | cut -c1-600 > "$OUT/long_horizon.txt" || true
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
  echo "tests rc=$rc"
fi
if [ -n "${AB_LIBS:-}" ]; then
  OUTAB=$OUT AB_LIBS="$AB_LIBS" AB_REPS=${AB_REPS:-2} bash scripts/ab_train.sh
fi
