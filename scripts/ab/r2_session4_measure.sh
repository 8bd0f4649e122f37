# HEAD measurement set (session 4 of round 2): GPU suite, smoke, headline
# bench x3 (driver defaults), 300-round runs, phantom 2/4/8 projection,
# kernel profile of the headline bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${MEASURE_DIR:-s4}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --out $O/n1_default_$i.json > /dev/null 2> $O/n1_default_$i.err || exit $?
done
timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out $O/n1_300.json > /dev/null 2>&1 || exit $?
for W in 2 4 8; do
  timeout -k 10 240 python bench.py --phantom-ranks $W --steps 300 --warmup 20 --out $O/ph$W.json > /dev/null 2>&1 || exit $?
done
for f in $O/*.json; do python -c "import json; r=json.load(open('$f')); print('$f', r['ms_per_step'], r['value'], r.get('projected_value'), r.get('detection_auc_mean'))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/prof1" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 > "$ROOT/$O/prof1.log" 2>&1 || exit $?
