#!/bin/bash
# Early scoring on the GPU: its tests, then bench.py with it on / off
# (alternating, one box) at 1 and phantom 4 / 8 ranks.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_device_protocol_gpu.py \
  -k "early" > "$OUT/early_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/early_tests.log"; exit 1; }
grep "ticks/us" "$OUT/early_tests.log"; tail -1 "$OUT/early_tests.log"
for pass in 1 2; do
  for ph in 8 4 1; do
    for e in 1 0; do
      f="$OUT/bench_ph${ph}_early${e}_p${pass}"
      FEDMX_EARLY_SCORE=$e timeout -k 10 180 python -u bench.py --steps 300 --warmup 20 --phantom-ranks $ph > "$f.json" \
        2> "$f.err" || { echo "bench rc=$?"; tail "$f.err"; exit 1; }
      echo "ph=$ph early=$e pass=$pass $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d.get('value'), d.get('projected_value'), d['detection_auc_mean'])" "$f.json")"
    done
  done
done
