#!/bin/bash
# One GPU session on the MI355X box: kernel numerics tests, smoke, bench,
# rocprofv3 kernel statistics.  Every GPU step has its own time limit; the
# script stops at the first fault / abort / timeout (rc not in {0,1}).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
python -c "import fedmse_decentralized_amd.ops.build as b; b.build_all()" || exit 3
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = kernels ]; then
  step bench_kernels 300 python scripts/bench_kernels.py
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 300 python bench.py --steps 50 --warmup 5 --out "$OUT/bench.json"
  step bench_cprofile 300 python bench.py --steps 20 --warmup 3 --out "$OUT/bench_cprofile.json" --profile "$OUT/bench_profile.txt"
fi
if [ "$MODE" = all ] || [ "$MODE" = rccl1 ]; then
  # the multi-GPU code path over a real one-rank RCCL group (prints the collective self-test)
  step rccl1 300 env FEDMX_FORCE_COLLECTIVES=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 50 --warmup 5 --out "$OUT/bench_rccl1.json"
fi
if [ "$MODE" = stamps ]; then
  step train_stamps 300 python scripts/train_stamps.py
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  cd /tmp && export TMPDIR=/tmp
  step rocprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2
  cd "$ROOT"
fi
if [ "$MODE" = pmc ]; then
  cd /tmp && export TMPDIR=/tmp
  rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
  step pmc 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d "$OUT/pmc" -o pmc -- python3 "$ROOT/scripts/bench_kernels.py" --reps 3
  cd "$ROOT"
fi
if [ "$MODE" = pmctrain ]; then
  cd /tmp && export TMPDIR=/tmp
  step pmc_train1 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d "$OUT/pmc_train1" -o pmc -- python3 "$ROOT/scripts/train_stamps.py" --plain
  step pmc_train2 300 rocprofv3 --kernel-trace --stats --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC -d "$OUT/pmc_train2" -o pmc -- python3 "$ROOT/scripts/train_stamps.py" --plain
  cd "$ROOT"
fi
echo "=== done"
