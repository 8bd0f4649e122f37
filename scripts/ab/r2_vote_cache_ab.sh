# per-client standardised vote data computed once (no per-round side-stream
# standardisation + cross-stream wait) vs per round: GPU suite, bench A/B
# (alternating, same box), kernel profile
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/vc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vc/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/vc/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in 0 2048; do
    FEDMX_VOTE_CACHE_MB=$m timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out gpurun_out/vc/b_${m}_$i.json > /dev/null 2> gpurun_out/vc/b_${m}_$i.err || exit $?
    python -c "import json; r=json.load(open('gpurun_out/vc/b_${m}_$i.json')); print('cache_mb=$m', $i, r['ms_per_step'], r['value'], r['detection_auc_mean'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/vc/prof" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/vc/prof.log" 2>&1 || exit $?
