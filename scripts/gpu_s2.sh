set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/s2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_train_failure_gpu.py tests/test_async_validation_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_new.log 2>&1; rc=$?
tail -n 5 $OUT/pytest_new.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python scripts/train_stamps.py --json $OUT/stamps.json > $OUT/stamps.log 2>&1 || { echo stamps failed; tail $OUT/stamps.log; exit 1; }
tail -n 30 $OUT/stamps.log
OUTAB=$OUT/ab AB_LIBS="main bu7vm7 pp7 all7 w4flag3" AB_REPS=2 bash scripts/ab_train.sh
