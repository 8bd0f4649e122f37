#!/bin/bash
# One-rank RCCL run (FEDMX_FORCE_COLLECTIVES=1: the multi-rank code path's
# collectives through a real one-rank NCCL/RCCL process group) of the bench.
set -u
mkdir -p gpurun_out/r4rccl
FEDMX_FORCE_COLLECTIVES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --steps 50 --warmup 5 \
  > gpurun_out/r4rccl/bench.json 2> gpurun_out/r4rccl/bench.err || { echo "rc=$?"; tail -n 30 gpurun_out/r4rccl/bench.err; exit 1; }
grep '^{' gpurun_out/r4rccl/bench.json | tail -1
grep -i "self-test" gpurun_out/r4rccl/bench.err | head -2
