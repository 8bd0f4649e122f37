# where the writer thread's first-round time goes: its own per-phase clock in
# the 64-client bench, and file creation with / without the GPU held
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ws
timeout -k 10 60 python scripts/open_probe.py > gpurun_out/ws/open_cpu.json 2>&1 || exit $?
timeout -k 10 120 python scripts/open_probe.py --gpu > gpurun_out/ws/open_gpu.json 2>&1 || exit $?
FEDMX_WRITER_STATS=1 timeout -k 10 180 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 5 --out gpurun_out/ws/kitsune64.json > gpurun_out/ws/kitsune64.log 2> gpurun_out/ws/kitsune64.err || exit $?
cat gpurun_out/ws/open_cpu.json gpurun_out/ws/open_gpu.json; tail -n 4 gpurun_out/ws/kitsune64.err
df -T /tmp . | tail -n 2
