#!/bin/bash
# Early scoring: kernel durations with it on / off (rocprofv3 --stats), and
# bench.py with a 16x longer poll period (libfedmx_hip_poll16.so) against off.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
for pass in 1 2; do
  for v in poll16 off default; do
    f="$OUT/bench_e2_${v}_p${pass}"
    case $v in
      poll16) env_="FEDMX_EARLY_SCORE=1 FEDMX_HIP_LIB=$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip_poll16.so" ;;
      off) env_="FEDMX_EARLY_SCORE=0" ;;
      default) env_="FEDMX_EARLY_SCORE=1" ;;
    esac
    env $env_ timeout -k 10 180 python -u bench.py --steps 300 --warmup 20 > "$f.json" 2> "$f.err" || { echo "bench rc=$?"; tail "$f.err"; exit 1; }
    echo "$v pass=$pass $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d.get('value'), d['detection_auc_mean'])" "$f.json")"
  done
done
cd /tmp && export TMPDIR=/tmp
for e in 1 0; do
  FEDMX_EARLY_SCORE=$e timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_e$e" -o run -- python3 "$ROOT/bench.py" --steps 30 --warmup 3 \
    > "$OUT/prof_e$e.log" 2>&1 || { echo "rocprof rc=$?"; tail "$OUT/prof_e$e.log"; exit 1; }
done
echo profiled
