#!/bin/bash
# BASELINE.json configs 3 and 5 (8 ranks) rehearsed on a ONE-GPU box: 8 gloo
# ranks share cuda:0 (RCCL refuses duplicate GPUs), so this checks the code
# path and the bench contract, not the timing.
#   config 3: 8-client SAE, one client per GPU            (--clients-per-gpu 1)
#   config 5: 64-client non-IID Kitsune-shaped, 8 per GPU (--clients-per-gpu 8 --data-kind kitsune --non-iid)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export FEDMX_DEVICE_INDEX=0 FEDMX_DIST_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name port args...
  local name=$1 port=$2; shift 2
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port "$port" bench.py --gpus 8 --steps 6 --warmup 2 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  grep '^{' "$OUT/$name.log" | tail -n 1
  return $rc
}
run config3_8x1 29531 --clients-per-gpu 1 && \
run config5_8x8_kitsune 29532 --clients-per-gpu 8 --data-kind kitsune --non-iid
