# PMC counters of fwd_rows_kernel at the 8-rank phantom (dev set of 80 clients)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p "$ROOT/gpurun_out/pf"
timeout -s KILL 120 rocprofv3 --kernel-include-regex fwd_rows --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY -d "$ROOT/gpurun_out/pf/p1" -o run -- python3 "$ROOT/bench.py" --phantom-ranks 8 --steps 10 --warmup 3 > "$ROOT/gpurun_out/pf/p1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-include-regex fwd_rows --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -d "$ROOT/gpurun_out/pf/p2" -o run -- python3 "$ROOT/bench.py" --phantom-ranks 8 --steps 10 --warmup 3 > "$ROOT/gpurun_out/pf/p2.log" 2>&1 || exit $?
