#!/bin/bash
# Round-6 end-of-round measurements on one MI355X (every GPU step under its
# own time limit; a fault, abort or time limit ends the call): smoke, the GPU
# test suite, the driver's headline command three times, the paper
# configuration, the training-kernel launch times, a rocprofv3 kernel trace of
# the headline, the FedProx variants' A/B and the training kernel's PMC passes.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
TAG=${TAG:-final}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -n 4 $OUT/pytest_gpu.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench_$i.json > $OUT/bench_$i.log 2>&1 || { echo bench failed; tail $OUT/bench_$i.log; exit 1; }
  tail -n 1 $OUT/bench_$i.log | cut -c1-160
done
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --epochs 100 --lr 1e-5 --shrink-lambda 10 --out $OUT/paper_config.json > $OUT/paper_config.log 2>&1 || { echo paper failed; exit 1; }
tail -n 1 $OUT/paper_config.log | cut -c1-160
timeout -k 10 300 python scripts/bench_kernels.py > $OUT/kernels.json 2> $OUT/kernels.err || { echo bench_kernels failed; exit 1; }
tail -n 1 $OUT/kernels.json | cut -c1-400
( cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof.log 2>&1 ) || { echo "rocprofv3 failed"; exit 1; }
db=$(find $OUT/prof -name "*.db" | head -n 1)
python3 scripts/prof_summary.py "$db" --title "round 6 (end): bench.py --gpus 1 --steps 20 --warmup 5, 1x MI355X" --out $OUT/bench_kernels.md > /dev/null && echo "trace summarised"
rm -rf $OUT/prof
if [ -n "${AB_LIBS:-}" ]; then OUTAB=$OUT/ab AB_LIBS="$AB_LIBS" AB_REPS=2 bash scripts/ab_train.sh || exit 1; fi
TAG=$TAG/pmc LIBS=main bash scripts/pmc_passes.sh && rm -rf $OUT/pmc/main_p1 $OUT/pmc/main_p2
echo done
