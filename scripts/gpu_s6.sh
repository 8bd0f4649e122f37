set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/s6; mkdir -p $OUT
TAG=s6/reh8 bash scripts/rehearsal_trace.sh || exit 1
NRANKS=8 COMM=ipc bash scripts/multirank_rehearsal.sh; rc=$?
grep -h "peer-memory\|transport\|fallback\|self-test\|Traceback" gpurun_out/rehearsal_bench8.log | sort | uniq -c | head -n 20
cp gpurun_out/rehearsal_bench8_ipc.json $OUT/ 2>/dev/null; cp gpurun_out/rehearsal_bench8.log $OUT/ 2>/dev/null
exit $rc
