#!/bin/bash
# Multi-rank rehearsal of bench.py / main.py on a ONE-GPU box: NRANKS ranks
# (default 2, at most 8 here) share cuda:0 (RCCL refuses duplicate GPUs):
# COMM=gloo (default) runs the round's collectives over gloo, COMM=ipc over
# the peer-memory kernels (parallel/ipc.py; gloo only for bring-up), the
# transport of the 8-GPU job's fallback (parallel/probe.py), which probes it
# first here too.  Exercises the sharded federation, the device-resident
# protocol's collectives and the bench JSON contract (max over ranks) end to
# end; the bench record lands in gpurun_out/rehearsal_bench$NRANKS_$COMM.json.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
NR=${NRANKS:-2}
[ "$NR" -ge 2 ] && [ "$NR" -le 8 ] || { echo "NRANKS must be 2..8"; exit 2; }
export FEDMX_DEVICE_INDEX=0 FEDMX_DIST_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0
# the extras' watchdog well inside gpurun's 180 s silence limit
export FEDMX_BENCH_EXTRA_TIMEOUT_S=${FEDMX_BENCH_EXTRA_TIMEOUT_S:-150}
COMM=${COMM:-gloo}
CARG=""
[ "$COMM" = ipc ] && CARG="--comm ipc"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NR --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus $NR --steps ${STEPS:-20} --warmup 5 $CARG \
  --out "$OUT/rehearsal_bench${NR}_$COMM.json" > "$OUT/rehearsal_bench$NR.log" 2>&1
rc=$?
echo "bench $NR ranks rc=$rc"; tail -n 3 "$OUT/rehearsal_bench$NR.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NR --master-addr 127.0.0.1 \
  --master-port 29518 main.py --synthetic nbaiot --num-rounds 2 --epoch 1 --model-types hybrid \
  --update-types mse_avg --compat fixed --output-root "$OUT/rehearsal_main" --log-level WARNING > "$OUT/rehearsal_main$NR.log" 2>&1
rc=$?
echo "main $NR ranks rc=$rc"; tail -n 3 "$OUT/rehearsal_main$NR.log"
exit $rc
