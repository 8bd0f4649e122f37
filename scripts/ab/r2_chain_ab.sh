# post-training chain changes A/B: per-client vote-data cache (FEDMX_VOTE_CACHE_MB)
# and split verification (FEDMX_VERIFY_SPLIT): GPU suite, alternating bench
# arms on one box, then a kernel profile of the default build
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ch
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ch/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/ch/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for arm in "0 0" "2048 0" "2048 1"; do
    set -- $arm
    FEDMX_VOTE_CACHE_MB=$1 FEDMX_VERIFY_SPLIT=$2 timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out gpurun_out/ch/b_$1_$2_$i.json > /dev/null 2> gpurun_out/ch/b_$1_$2_$i.err || exit $?
    python -c "import json; r=json.load(open('gpurun_out/ch/b_$1_$2_$i.json')); print('cache_mb=$1 split=$2 run $i', r['ms_per_step'], r['value'], r['detection_auc_mean'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/ch/prof" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/ch/prof.log" 2>&1 || exit $?
