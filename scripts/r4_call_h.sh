#!/bin/bash
# Round-4 closing call: the driver's smoke(), and a kernel-trace profile of
# the headline bench on the final tree.
set -u
mkdir -p gpurun_out/r4h
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4h/smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -n 20 gpurun_out/r4h/smoke.txt; exit 1; }
tail -n 1 gpurun_out/r4h/smoke.txt
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4h/prof -o run -- python3 bench.py --steps 20 --warmup 3 \
  > gpurun_out/r4h/prof_bench.json 2> gpurun_out/r4h/prof.err || { echo "rocprof rc=$?"; tail -n 20 gpurun_out/r4h/prof.err; exit 1; }
echo "profile ok"
