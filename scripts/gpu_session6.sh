#!/bin/bash
# Round-6 GPU session: the GPU test suite, then (if it did not crash) the
# headline bench twice, the training-kernel A/B of $AB_LIBS and the paper
# configuration.  Every GPU step has its own time limit; a fault, abort or
# time limit ends the call.  Output: gpurun_out/$TAG/.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${TAG:-s6}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${TESTS:-all}" != none ]; then
  T=${TESTS:-tests}
  [ "$T" = all ] && T=tests
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $T -m gpu -v --maxfail=5 --timeout 300 \
    --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?
  tail -n 8 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
if [ "${BENCH:-1}" = 1 ]; then
  for i in 1 2; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench_$i.json > $OUT/bench_$i.log 2>&1 \
      || { echo "bench $i failed"; tail -n 20 $OUT/bench_$i.log; exit 1; }
    tail -n 1 $OUT/bench_$i.log | cut -c1-220
  done
fi
if [ -n "${AB_LIBS:-}" ]; then
  OUTAB=$OUT/ab AB_LIBS="$AB_LIBS" AB_REPS=${AB_REPS:-2} bash scripts/ab_train.sh || exit 1
fi
if [ "${PAPER:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 2 --epochs 100 --lr 1e-5 --shrink-lambda 10 \
    --out $OUT/paper_config.json > $OUT/paper_config.log 2>&1 || { echo "paper config failed"; exit 1; }
  tail -n 1 $OUT/paper_config.log | cut -c1-220
fi
echo done
