#!/bin/bash
# Round-4 GPU call B: the adoption ablation (HIP engine) and a kernel-trace
# profile of the headline bench.
set -u
mkdir -p gpurun_out/r4b
bash scripts/r4_adoption.sh gpurun_out/r4_adoption || exit 1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b/prof -o run -- python3 bench.py --steps 20 --warmup 3 \
  > gpurun_out/r4b/prof_bench.json 2> gpurun_out/r4b/prof.err || { echo "rocprof rc=$?"; tail -n 20 gpurun_out/r4b/prof.err; exit 1; }
echo "profile ok"
