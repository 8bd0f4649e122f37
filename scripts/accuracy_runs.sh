#!/bin/bash
# GPU side of the non-IID accuracy records (VERDICT r4 Next #2b/#2c):
# the six model x aggregation combinations at the paper's hyper-parameters
# (100 local epochs, 20 rounds, lr 1e-5, shrink lambda 10, 50 % of 10 clients)
# on synthetic N-BaIoT-shaped NON-IID clients (Dirichlet alpha 0.5 = the
# generator's non-IID default), 3 runs; then the settings that could separate
# the aggregation rules: stronger heterogeneity (alpha 0.05) and one poisoned
# client (fault injection: client 3's update scaled x10 every round it trains).
# Report trees under gpurun_out/$TAG/<setting>/; tables: scripts/results_table.py.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${TAG:-acc}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
COMMON="--synthetic nbaiot --synthetic-iid False --epoch 100 --num-rounds 20 --lr-rate 1e-5 --shrink-lambda 10
        --num-runs ${RUNS:-3} --compat fixed --global-early-stop False --save-checkpoints False --log-level WARNING
        --backend hip"
run() {
  name=$1; shift
  timeout -k 10 ${STEP_TIMEOUT:-300} python main.py $COMMON --output-root "$OUT/$name" --no-exp "$name" "$@" \
    > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc $(tail -n 1 "$OUT/$name.log" | cut -c1-200)"
  return $rc
}
# SETTINGS="tableA_noniid noniid_a005 noniid_poison3" (default: all three)
for s in ${SETTINGS:-tableA_noniid noniid_a005 noniid_poison3}; do
  case $s in
    tableA_noniid) run tableA_noniid || exit $? ;;
    noniid_a005) run noniid_a005 --synthetic-alpha 0.05 || exit $? ;;
    noniid_poison3) run noniid_poison3 --malicious-clients 3 --malicious-scale 10 || exit $? ;;
  esac
done
