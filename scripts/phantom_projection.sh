set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ph
for W in 2 4 8; do
  timeout -k 10 240 python bench.py --phantom-ranks $W --steps 300 --warmup 20 --out gpurun_out/ph/ph$W.json > gpurun_out/ph/ph$W.log 2>&1 || exit $?
  tail -c 300 gpurun_out/ph/ph$W.json; echo
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/ph/prof8" -o run -- python3 "$ROOT/bench.py" --phantom-ranks 8 --steps 20 --warmup 5 > "$ROOT/gpurun_out/ph/prof8.log" 2>&1
