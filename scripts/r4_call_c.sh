#!/bin/bash
# Round-4 final GPU check on the committed tree: the whole GPU test tier, the
# headline bench and the paper configuration (scripts/r4_gpu_check.sh), and
# the training-kernel launch timing of the production build.
set -u
bash scripts/r4_gpu_check.sh ${OUT:-gpurun_out/r4c} || exit 1
timeout -k 10 120 python scripts/bench_kernels.py --train-only --reps 15 > ${OUT:-gpurun_out/r4c}/train_kernel.json 2> ${OUT:-gpurun_out/r4c}/train_kernel.err \
  || { echo "bench_kernels rc=$?"; tail -n 20 ${OUT:-gpurun_out/r4c}/train_kernel.err; exit 1; }
cat ${OUT:-gpurun_out/r4c}/train_kernel.json
