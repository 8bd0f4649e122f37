# helper-wave kernel: parity test first (short limit), then A/B timing, then the GPU suite
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -x -q -k helper_waves --timeout 100 --timeout-method thread > gpurun_out/pytest_hw.log 2>&1
rc=$?; tail -n 25 gpurun_out/pytest_hw.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_train.sh || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_gpu.log; exit $rc
