# many clients on one GPU: BASELINE config 5 (64 Kitsune-shaped non-IID clients) with a
# warm-up long enough that every client's artefact files exist (first creation costs
# ~1.4 ms per file on the GPU hosts' /tmp), and 256 N-BaIoT-shaped clients
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/mc
timeout -k 10 200 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 20 --out gpurun_out/mc/k64_w20.json > gpurun_out/mc/k64_w20.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 5 --out gpurun_out/mc/k64_w5.json > gpurun_out/mc/k64_w5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --clients 256 --steps 10 --warmup 10 --out gpurun_out/mc/n256.json > gpurun_out/mc/n256.log 2>&1 || exit $?
