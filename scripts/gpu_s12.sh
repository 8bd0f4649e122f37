#!/bin/bash
# Round-6 fence-less device events (VERDICT r5 Next #7, second item): the
# device-round suites that compare the device path with the host path
# bit for bit, then an end-to-end A/B against torch events
# (FEDMX_DEVICE_EVENTS=0; identical numerics in both arms) and a kernel
# trace of the headline with the device events.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/${TAG:-s12}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_device_protocol_gpu.py \
  tests/test_async_validation_gpu.py tests/test_train_failure_gpu.py > $OUT/pytest.log 2>&1 \
  || { echo tests failed; tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
for rep in 1 2 3; do
  for f in 1 0; do
    FEDMX_DEVICE_EVENTS=$f timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --out $OUT/ab_e$f.$rep.json \
      > $OUT/ab_e$f.$rep.log 2>&1 || { echo bench failed; tail $OUT/ab_e$f.$rep.log; exit 1; }
    echo "device_events=$f rep=$rep $(tail -n 1 $OUT/ab_e$f.$rep.log | cut -c1-140)"
  done
done
( cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run \
    -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof.log 2>&1 ) || { echo "rocprofv3 failed"; exit 1; }
db=$(find $OUT/prof -name "*.db" | head -n 1)
python3 scripts/prof_summary.py "$db" --title "round 6: bench.py --gpus 1 --steps 20 --warmup 5 with fence-less device events, 1x MI355X" \
  --out $OUT/bench_kernels.md > /dev/null && echo "trace summarised"
rm -rf $OUT/prof
