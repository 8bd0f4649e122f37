# r2 end: PMC counters of the helper-wave training launch at HEAD (two passes
# within the counter-block limits; --pmc runs carry no trace domains)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d "$ROOT/gpurun_out/pmc_end1" -o pmc -- python3 "$ROOT/scripts/train_stamps.py" --plain > "$ROOT/gpurun_out/pmc_end1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVES -d "$ROOT/gpurun_out/pmc_end2" -o pmc -- python3 "$ROOT/scripts/train_stamps.py" --plain > "$ROOT/gpurun_out/pmc_end2.log" 2>&1 || exit $?
