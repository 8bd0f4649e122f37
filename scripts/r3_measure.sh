# end-of-round measurement set (round 3): GPU suite, smoke, headline bench x3 (+300-round),
# config, phantom 2/4/8 projection, many clients (64 Kitsune non-IID with 5 and
# 20 warm-up rounds, 256 N-BaIoT), kernel profiles (headline, 8-rank phantom)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${MEASURE_DIR:-r3}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --out $O/n1_default_$i.json > $O/n1_default_$i.stdout 2> $O/n1_default_$i.err || exit $?
  timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out $O/n1_300_$i.json > /dev/null 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --epochs 100 --lr 1e-5 --shrink-lambda 10 --steps 20 --warmup 3 --out $O/paper.json > /dev/null 2>&1 || exit $?
for W in 2 4 8; do
  timeout -k 10 240 python bench.py --phantom-ranks $W --steps 300 --warmup 20 --out $O/ph$W.json > /dev/null 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 20 --out $O/k64_w20.json > /dev/null 2>&1 || exit $?
timeout -k 10 200 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 5 --out $O/k64_w5.json > /dev/null 2>&1 || exit $?
timeout -k 10 300 python bench.py --clients 256 --steps 10 --warmup 10 --out $O/n256.json > /dev/null 2>&1 || exit $?
for f in $O/*.json; do python -c "import json; r=json.load(open('$f')); print('$f', r['ms_per_step'], r['value'], r.get('projected_value'), r.get('detection_auc_mean'))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/prof1" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 > "$ROOT/$O/prof1.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/prof8" -o run -- python3 "$ROOT/bench.py" --phantom-ranks 8 --steps 20 --warmup 5 > "$ROOT/$O/prof8.log" 2>&1 || exit $?
python "$ROOT/scripts/prof_summary.py" "$ROOT/$O/prof1/run_results.db" --title "round 3: bench.py --steps 20 --warmup 3, 1x MI355X" --out "$ROOT/$O/prof1.md" > /dev/null
python "$ROOT/scripts/prof_summary.py" "$ROOT/$O/prof8/run_results.db" --title "round 3: bench.py --phantom-ranks 8 (rank 0 of the 8-GPU job, collectives stubbed)" --out "$ROOT/$O/prof8.md" > /dev/null
echo done
