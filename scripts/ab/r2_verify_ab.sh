# fused verification kernel with the drift loads batched (one round trip)
# vs the previous kernel
# (libfedmx_hip_oldverify.so): GPU suite, alternating bench arms, profile
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/vf
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vf/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/vf/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
OLD="$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip_oldverify.so"
for i in 1 2; do
  FEDMX_HIP_LIB=$OLD timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out gpurun_out/vf/old_$i.json > /dev/null 2> gpurun_out/vf/old_$i.err || exit $?
  timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out gpurun_out/vf/new_$i.json > /dev/null 2> gpurun_out/vf/new_$i.err || exit $?
  for m in old new; do python -c "import json; r=json.load(open('gpurun_out/vf/${m}_$i.json')); print('$m run $i', r['ms_per_step'], r['value'], r['detection_auc_mean'])"; done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/vf/prof" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/vf/prof.log" 2>&1 || exit $?
