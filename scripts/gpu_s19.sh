#!/bin/bash
# Round-6 side-stream hand-off (verify_split_kernel's hand-off word +
# side_wait_kernel instead of an event between the verification and the next
# training launch): kernel and device-round suites, 200-round device-vs-host
# parity, an end-to-end A/B against the device event (FEDMX_SIDE_FLAG=0;
# identical numerics in both arms) and a kernel trace with the gap statistic.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/${TAG:-s19}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_device_protocol_gpu.py tests/test_async_validation_gpu.py tests/test_train_failure_gpu.py \
  > $OUT/pytest.log 2>&1 || { echo tests failed; tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 400 python scripts/device_vs_host_long.py --rounds 200 --out $OUT/dvh_mse_avg_200.json > $OUT/dvh.log 2>&1 \
  || { echo parity failed; tail -n 3 $OUT/dvh.log | cut -c1-300; exit 1; }
tail -n 1 $OUT/dvh.log | cut -c1-160
for rep in 1 2 3; do
  for f in 1 0; do
    FEDMX_SIDE_FLAG=$f timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --out $OUT/ab_f$f.$rep.json \
      > $OUT/ab_f$f.$rep.log 2>&1 || { echo bench failed; tail $OUT/ab_f$f.$rep.log; exit 1; }
    echo "side_flag=$f rep=$rep $(tail -n 1 $OUT/ab_f$f.$rep.log | cut -c1-140)"
  done
done
( cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof.log 2>&1 ) || { echo "rocprofv3 failed"; exit 1; }
db=$(find $OUT/prof -name "*.db" | head -n 1)
python3 scripts/prof_summary.py "$db" --title "round 6: bench.py --gpus 1 --steps 20 --warmup 5 with the side-stream hand-off word, 1x MI355X" \
  --out $OUT/bench_kernels.md > /dev/null && echo "trace summarised"
rm -rf $OUT/prof
