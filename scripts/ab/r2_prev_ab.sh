# current build vs the previous commit's library (libfedmx_hip_prev.so):
# GPU suite, alternating headline bench arms, kernel profile of the current
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/${AB_TAG:-ab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
PREV="$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip_prev.so"
for i in 1 2; do
  FEDMX_HIP_LIB=$PREV timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out $OUT/prev_$i.json > /dev/null 2>&1 || exit $?
  timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out $OUT/cur_$i.json > /dev/null 2>&1 || exit $?
  for m in prev cur; do python -c "import json; r=json.load(open('$OUT/${m}_$i.json')); print('$m run $i', r['ms_per_step'], r['value'], r['detection_auc_mean'])"; done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 > "$ROOT/$OUT/prof.log" 2>&1 || exit $?
