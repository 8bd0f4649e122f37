# native checkpoint writer: GPU suite, then the 64-client and 10-client benches with writer stats
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/cfg
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
FEDMX_WRITER_STATS=1 timeout -k 10 180 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 5 --out gpurun_out/cfg/kitsune64.json > gpurun_out/cfg/kitsune64.log 2> gpurun_out/cfg/kitsune64.err || exit $?
FEDMX_WRITER_STATS=1 timeout -k 10 180 python bench.py --steps 50 --warmup 5 --out gpurun_out/cfg/n10.json > gpurun_out/cfg/n10.log 2> gpurun_out/cfg/n10.err || exit $?
for f in kitsune64 n10; do python -c "
import json; r=json.load(open('gpurun_out/cfg/$f.json')); print('$f', r['ms_per_step'], r['federation_rounds_per_sec'], r['writer_busy_ms_per_round'], r['phase_ms_total'])"; done
