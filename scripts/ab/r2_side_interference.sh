# training-kernel durations with and without the concurrent side-stream evaluation
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p "$ROOT/gpurun_out/si"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/si/eval" -o run -- python3 "$ROOT/scripts/diag_side_interference.py" --rounds 30 > "$ROOT/gpurun_out/si/eval.log" 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/si/noeval" -o run -- python3 "$ROOT/scripts/diag_side_interference.py" --rounds 30 --no-eval > "$ROOT/gpurun_out/si/noeval.log" 2>&1 || exit $?
if [ -f "$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip_prev.so" ]; then
  FEDMX_HIP_LIB="$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip_prev.so" timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/si/prev" -o run -- python3 "$ROOT/scripts/diag_side_interference.py" --rounds 30 > "$ROOT/gpurun_out/si/prev.log" 2>&1 || exit $?
fi
