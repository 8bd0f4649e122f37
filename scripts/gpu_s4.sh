set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/s4; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_ipc_gpu.py tests/test_device_protocol_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_ipc.log 2>&1; rc=$?
tail -n 4 $OUT/pytest_ipc.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench_$i.json > $OUT/bench_$i.log 2>&1 || { echo bench failed; tail $OUT/bench_$i.log; exit 1; }
  tail -n 1 $OUT/bench_$i.log | cut -c1-200
  FEDMX_VERIFY_SPLIT=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --out $OUT/bench_fused_$i.json > $OUT/bench_fused_$i.log 2>&1 || exit 1
  tail -n 1 $OUT/bench_fused_$i.log | cut -c1-200
done
( cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof.log 2>&1 ) || { echo "rocprofv3 failed"; exit 1; }
db=$(find $OUT/prof -name "*.db" | head -n 1)
python3 scripts/prof_summary.py "$db" --title "round 6: bench.py --gpus 1 --steps 20 --warmup 5, 1x MI355X" --out $OUT/bench_kernels.md > /dev/null && sed -n '/one round timeline/,$p' $OUT/bench_kernels.md
OUTAB=$OUT/ab AB_LIBS="main av3" AB_REPS=2 bash scripts/ab_train.sh || exit 1
TAG=s4/reh8 EXTRA="" bash scripts/rehearsal_trace.sh
