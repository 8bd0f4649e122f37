#!/bin/bash
# Wall clock of the reference-default sweep (python main.py: 6 model x update
# combinations x 3 rounds x 5 epochs, 10 clients, every artefact) on one GPU,
# reference-compat and fixed-compat, plus a cProfile of the fixed run.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/sweep
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
run_main() {  # label extra-args...
  local label=$1; shift
  d=$(mktemp -d)
  s=$(date +%s.%N)
  timeout -k 10 300 python main.py --synthetic nbaiot --output-root "$d" --log-level WARNING "$@" \
    > "$OUT/main_$label.log" 2>&1 || { echo "main $label rc=$?"; tail -5 "$OUT/main_$label.log"; exit 1; }
  e=$(date +%s.%N)
  echo "main.py $* wall_s=$(python -c "print(round($e-$s,3))") summary_sha=$(sha256sum "$d"/Checkpoint/Results/Update/10/*/training_summary.json | cut -c1-16) reports_sha=$(find "$d"/Checkpoint/Results -name '*.json' | sort | xargs cat | sha256sum | cut -c1-16)"
  rm -rf "$d"
}
run_main fixed --compat fixed
run_main reference --compat reference
run_main fixed_conc --compat fixed --concurrent-combos true
run_main fixed2 --compat fixed
run_main fixed_conc2 --compat fixed --concurrent-combos true
# paper configuration sweep (100 epochs, 20 rounds, lr 1e-5, lambda 10): sequential vs concurrent
run_main paper --compat fixed --epoch 100 --num-rounds 20 --lr-rate 1e-5 --shrink-lambda 10
run_main paper_conc --compat fixed --epoch 100 --num-rounds 20 --lr-rate 1e-5 --shrink-lambda 10 --concurrent-combos true
d=$(mktemp -d)
timeout -k 10 300 python -m cProfile -o "$OUT/main_fixed.prof" main.py --synthetic nbaiot --compat fixed --output-root "$d" \
  --log-level WARNING > /dev/null 2>&1 || exit 1
python -c "
import pstats; s = pstats.Stats('$OUT/main_fixed.prof'); s.sort_stats('cumulative').print_stats(45)" > "$OUT/main_fixed_prof.txt"
head -70 "$OUT/main_fixed_prof.txt" | tail -55
