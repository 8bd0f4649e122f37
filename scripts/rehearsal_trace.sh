#!/bin/bash
# Kernel trace of the 8-process one-GPU rehearsal (VERDICT r5 Next #4c): NR
# ranks of bench.py share cuda:0 (gloo bring-up, FEDMX_DEVICE_INDEX=0), each
# started by rocprofv3 --kernel-trace directly (no launcher in between: the
# profiler must start the program itself), with the env rendezvous torchrun
# would give them.  scripts/rehearsal_trace_summary.py merges the per-rank
# traces into one device timeline.  Output: gpurun_out/$TAG/.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${TAG:-reh8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
NR=${NRANKS:-8}
COMM=${COMM:-ipc}
export FEDMX_DEVICE_INDEX=0 FEDMX_DIST_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0
export MASTER_ADDR=127.0.0.1 MASTER_PORT=${MASTER_PORT:-29541} WORLD_SIZE=$NR LOCAL_WORLD_SIZE=$NR
export FEDMX_BENCH_EXTRA_TIMEOUT_S=${FEDMX_BENCH_EXTRA_TIMEOUT_S:-150}
CARG=""
[ "$COMM" = ipc ] && CARG="--comm ipc"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
# the per-rank traces stay outside gpurun_out (8 databases exceed what a call
# copies back); the merged summary and the rank logs are kept
TR=/tmp/fedmx_reh_$$
mkdir -p $TR
pids=""
for r in $(seq 0 $((NR - 1))); do
  RANK=$r LOCAL_RANK=$r timeout -k 10 400 rocprofv3 --kernel-trace -d $TR/rank$r -o run \
    -- python3 bench.py --gpus $NR --steps ${STEPS:-20} --warmup 5 $CARG ${EXTRA---no-extra} \
    --out $OUT/bench_rank$r.json > $OUT/rank$r.log 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
echo "ranks done rc=$rc"
tail -n 2 $OUT/rank0.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
grep -h "peer-memory\|transport\|self-test\|fallback\|Traceback\|Error" $OUT/rank*.log | sort | uniq -c | head -n 20
python3 scripts/rehearsal_trace_summary.py $TR --out $OUT/summary.md > /dev/null && tail -n 30 $OUT/summary.md
rm -rf $TR
