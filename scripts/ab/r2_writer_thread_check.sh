# C++ writer thread owns the artefact files: GPU suite (device vs host artefact
# bytes), 64-client round time series (first-round stall), benches with writer stats
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/wt
for v in "--gpu --hold" "--gpu --hold --reserve"; do
  timeout -k 10 120 python scripts/open_probe.py $v >> gpurun_out/wt/open_probe.jsonl 2>/dev/null || exit $?
done
cat gpurun_out/wt/open_probe.jsonl
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wt/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/wt/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u scripts/round_time_series.py --clients 64 --rounds 60 --block 5 --non-iid > gpurun_out/wt/ts64.log 2>&1 || exit $?
tail -n 20 gpurun_out/wt/ts64.log
FEDMX_WRITER_STATS=1 timeout -k 10 180 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 5 --out gpurun_out/wt/kitsune64.json > gpurun_out/wt/kitsune64.log 2> gpurun_out/wt/kitsune64.err || exit $?
tail -n 2 gpurun_out/wt/kitsune64.err
FEDMX_WRITER_STATS=1 timeout -k 10 180 python bench.py --steps 200 --warmup 20 --out gpurun_out/wt/n10.json > gpurun_out/wt/n10.log 2> gpurun_out/wt/n10.err || exit $?
for f in kitsune64 n10; do python -c "
import json; r=json.load(open('gpurun_out/wt/$f.json')); print('$f', r['ms_per_step'], r['federation_rounds_per_sec'], r.get('writer_busy_ms_per_round'), r['phase_ms_total'])"; done
