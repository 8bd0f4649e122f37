# quick HEAD check (round 3): GPU suite, smoke, headline bench x2, kernel profile
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${MEASURE_DIR:-r3q}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python bench.py --out $O/n1_default_$i.json > $O/n1_default_$i.stdout 2> $O/n1_default_$i.err || exit $?
  tail -n 1 $O/n1_default_$i.stdout | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/prof1" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 > "$ROOT/$O/prof1.log" 2>&1 || exit $?
python "$ROOT/scripts/prof_summary.py" "$ROOT/$O/prof1/run_results.db" --title "round 3: bench.py --steps 20 --warmup 3, 1x MI355X" --out "$ROOT/$O/prof1.md" > /dev/null
echo done
