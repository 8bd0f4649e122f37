# compact-order forward (125 instead of 144 MFMAs per 16-row tile): GPU suite,
# headline + 8-rank phantom + 64-client benches, kernel profiles
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/fc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fc/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/fc/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out gpurun_out/fc/n1.json > /dev/null 2> gpurun_out/fc/n1.err || exit $?
timeout -k 10 120 python bench.py --phantom-ranks 8 --steps 200 --warmup 20 --out gpurun_out/fc/p8.json > /dev/null 2> gpurun_out/fc/p8.err || exit $?
timeout -k 10 180 python bench.py --clients 256 --steps 20 --warmup 5 --out gpurun_out/fc/c256.json > /dev/null 2> gpurun_out/fc/c256.err || exit $?
for f in n1 p8 c256; do python -c "import json; r=json.load(open('gpurun_out/fc/$f.json')); print('$f', r['ms_per_step'], r['value'], r.get('projected_value'), r['detection_auc_mean'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/fc/prof8" -o run -- python3 "$ROOT/bench.py" --phantom-ranks 8 --steps 5 --warmup 2 > "$ROOT/gpurun_out/fc/prof8.log" 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/fc/prof1" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/gpurun_out/fc/prof1.log" 2>&1 || exit $?
