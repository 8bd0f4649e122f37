set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/auc
timeout -k 10 200 python scripts/auc_trajectory.py --clients 64 --data-kind kitsune --non-iid --rounds 60 --episode 20 --out gpurun_out/auc/k64_ep20.jsonl > gpurun_out/auc/k64_ep20.log 2>&1 || exit $?
timeout -k 10 200 python scripts/auc_trajectory.py --clients 64 --data-kind kitsune --non-iid --rounds 60 --episode 0 --out gpurun_out/auc/k64_ep0.jsonl > gpurun_out/auc/k64_ep0.log 2>&1 || exit $?
timeout -k 10 200 python scripts/auc_trajectory.py --clients 64 --data-kind kitsune --non-iid --rounds 60 --episode 20 --shrink-lambda 1 --out gpurun_out/auc/k64_lam1.jsonl > gpurun_out/auc/k64_lam1.log 2>&1 || exit $?
timeout -k 10 200 python scripts/auc_trajectory.py --clients 10 --data-kind nbaiot --rounds 60 --episode 20 --out gpurun_out/auc/n10_ep20.jsonl > gpurun_out/auc/n10_ep20.log 2>&1 || exit $?
bash scripts/phantom_projection.sh
