#!/bin/bash
# GPU test tier + bench + paper config, the adoption ablation, a kernel-trace
# profile of the bench; stops at the first failure.
set -u
bash scripts/r4_gpu_check.sh gpurun_out/r4b || exit 1
bash scripts/r4_adoption.sh gpurun_out/r4_adoption || exit 1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b/prof -o run -- python3 bench.py --steps 20 --warmup 3 \
  > gpurun_out/r4b/prof_bench.json 2> gpurun_out/r4b/prof.err || { echo "rocprof rc=$?"; tail -n 20 gpurun_out/r4b/prof.err; exit 1; }
echo "profile ok"
