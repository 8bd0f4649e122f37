#!/bin/bash
# End-of-round measurements on one MI355X, every GPU step under its own time
# limit, stopping at the first failure: the driver's headline command three
# times (bench.py --gpus 1 --steps 20 --warmup 5), the paper configuration
# (100 epochs, lr 1e-5, lambda 10; 10 rounds after 2), the training-kernel
# timing (bench_kernels --train-only), a rocprofv3 kernel trace of the
# headline bench summarised by scripts/prof_summary.py, and the PMC passes of
# the training kernel (scripts/pmc_passes.sh).  Output: gpurun_out/$TAG/.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${TAG:-measure}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench_$i.json > $OUT/bench_$i.log 2>&1 \
    || { echo "bench $i failed"; tail -n 20 $OUT/bench_$i.log; exit 1; }
  tail -n 1 $OUT/bench_$i.log | cut -c1-200
done
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --epochs 100 --lr 1e-5 --shrink-lambda 10 \
  --out $OUT/paper_config.json > $OUT/paper_config.log 2>&1 || { echo "paper config failed"; exit 1; }
tail -n 1 $OUT/paper_config.log | cut -c1-200
timeout -k 10 300 python scripts/bench_kernels.py > $OUT/kernels.json 2> $OUT/kernels.err || { echo "bench_kernels failed"; exit 1; }
tail -n 1 $OUT/kernels.json | cut -c1-300
( cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof.log 2>&1 ) || { echo "rocprofv3 failed"; exit 1; }
db=$(find $OUT/prof -name "*.db" | head -n 1)
python3 scripts/prof_summary.py "$db" --title "round 5: bench.py --gpus 1 --steps 20 --warmup 5, 1x MI355X" \
  --out $OUT/bench_kernels.md > /dev/null && echo "kernel trace summarised"
TAG=$TAG LIBS=${PMC_LIBS:-main} bash scripts/pmc_passes.sh
