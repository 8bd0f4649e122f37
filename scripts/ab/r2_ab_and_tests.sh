# A/B the built variant libraries on the training-kernel microbenchmark, then
# the GPU test suite on the default library (stops at the first failure).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/ab_train.sh || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -n 15 gpurun_out/pytest_gpu.log
exit $rc
