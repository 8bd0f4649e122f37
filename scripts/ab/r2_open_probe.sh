# file creation cost on the GPU box under bench-like process conditions
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/op
for v in "" "--hold" "--threads 24" "--gpu" "--gpu --hold"; do
  timeout -k 10 120 python scripts/open_probe.py $v >> gpurun_out/op/probe.jsonl 2>/dev/null || exit $?
done
cat gpurun_out/op/probe.jsonl
