# batched-forward kernel at scale: kernel statistics and PMC counters of the 256-client round
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p "$ROOT/gpurun_out/fwd"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/fwd/prof256" -o run -- python3 "$ROOT/bench.py" --clients 256 --steps 4 --warmup 3 > "$ROOT/gpurun_out/fwd/prof256.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES -d "$ROOT/gpurun_out/fwd/pmc256" -o pmc -- python3 "$ROOT/bench.py" --clients 256 --steps 2 --warmup 1 > "$ROOT/gpurun_out/fwd/pmc256.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d "$ROOT/gpurun_out/fwd/pmc256b" -o pmc -- python3 "$ROOT/bench.py" --clients 256 --steps 2 --warmup 1 > "$ROOT/gpurun_out/fwd/pmc256b.log" 2>&1
