# re-entry check of HEAD on a fresh box: GPU suite, smoke, headline bench x2
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/re
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python bench.py --out $O/n1_default_$i.json > $O/n1_default_$i.stdout 2> $O/n1_default_$i.err || exit $?
  cat $O/n1_default_$i.stdout
done
