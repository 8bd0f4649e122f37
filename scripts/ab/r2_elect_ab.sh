# weighted sum of the election kernel: one element per thread, every selected
# row's load in flight (new) vs float4 with 8 loads in flight (old,
# libfedmx_hip_oldelect.so); 1 GPU headline and the 8-rank phantom projection
# (k = 40 selections), with kernel profiles
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/el
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/el/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/el/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
OLD="$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip_oldelect.so"
for i in 1 2; do
  FEDMX_HIP_LIB=$OLD timeout -k 10 120 python bench.py --phantom-ranks 8 --steps 200 --warmup 20 --out gpurun_out/el/p8old_$i.json > /dev/null 2> gpurun_out/el/p8old_$i.err || exit $?
  timeout -k 10 120 python bench.py --phantom-ranks 8 --steps 200 --warmup 20 --out gpurun_out/el/p8new_$i.json > /dev/null 2> gpurun_out/el/p8new_$i.err || exit $?
  for m in p8old p8new; do python -c "import json; r=json.load(open('gpurun_out/el/${m}_$i.json')); print('$m run $i', r['ms_per_step'], r['projected_value'])"; done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/el/prof8" -o run -- python3 "$ROOT/bench.py" --phantom-ranks 8 --steps 5 --warmup 2 > "$ROOT/gpurun_out/el/prof8.log" 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/el/prof1" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/el/prof1.log" 2>&1 || exit $?
