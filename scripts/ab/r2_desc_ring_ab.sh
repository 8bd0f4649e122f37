# descriptor ring in fine-grained device memory vs mapped host memory:
# GPU suite, then bench A/B (alternating, same box), then a kernel profile
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/dr
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dr/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/dr/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in host device; do
    FEDMX_DESC_RING=$m timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out gpurun_out/dr/b_${m}_$i.json > /dev/null 2> gpurun_out/dr/b_${m}_$i.err || exit $?
    python -c "import json; r=json.load(open('gpurun_out/dr/b_${m}_$i.json')); print('$m', $i, r['ms_per_step'], r['value'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/dr/prof" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/dr/prof.log" 2>&1 || exit $?
