set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/s3; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ipc_gpu.py tests/test_device_protocol_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_ipc.log 2>&1; rc=$?
tail -n 4 $OUT/pytest_ipc.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
OUTAB=$OUT/ab AB_LIBS="main av3" AB_REPS=2 bash scripts/ab_train.sh || exit 1
TAG=s3/reh8 EXTRA="" bash scripts/rehearsal_trace.sh
