# 64-client Kitsune non-IID federation: kernel timeline (rocprofv3) and host cProfile
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/k64
timeout -k 10 180 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 30 --warmup 5 --profile gpurun_out/k64/cprofile.txt --out gpurun_out/k64/bench_prof.json > gpurun_out/k64/bench_prof.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/k64/prof" -o run -- python3 "$ROOT/bench.py" --clients 64 --data-kind kitsune --non-iid --steps 10 --warmup 3 > "$ROOT/gpurun_out/k64/prof.log" 2>&1
