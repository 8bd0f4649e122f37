# forward staging in one load round: GPU suite, 1-GPU kernel profile, and
# rows-per-block 64 (default at N=1) vs 128 vs 256 on the headline bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/fs
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fs/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/fs/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for r in 0 128 256; do
    FEDMX_FWD_ROWS_PER_BLOCK=$r timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out gpurun_out/fs/n1_${r}_$i.json > /dev/null 2>&1 || exit $?
    python -c "import json; r=json.load(open('gpurun_out/fs/n1_${r}_$i.json')); print('rpb=$r run $i', r['ms_per_step'], r['value'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/fs/prof1" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/fs/prof1.log" 2>&1 || exit $?
