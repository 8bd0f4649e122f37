set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/s7; mkdir -p $OUT
NRANKS=8 COMM=ipc bash scripts/multirank_rehearsal.sh; rc=$?
grep -h "peer-memory\|transport\|fallback\|Traceback" gpurun_out/rehearsal_bench8.log | sort | uniq -c | head -n 20
cp gpurun_out/rehearsal_bench8_ipc.json $OUT/ 2>/dev/null; cp gpurun_out/rehearsal_bench8.log $OUT/ 2>/dev/null
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_ipc_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_ipc.log 2>&1; rc=$?
tail -n 3 $OUT/pytest_ipc.log; exit $rc
