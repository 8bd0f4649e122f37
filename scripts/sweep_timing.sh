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
for compat in fixed reference fixed; do
  d=$(mktemp -d)
  s=$(date +%s.%N)
  timeout -k 10 300 python main.py --synthetic nbaiot --compat $compat --output-root "$d" --log-level WARNING \
    > "$OUT/main_$compat.log" 2>&1 || { echo "main $compat rc=$?"; tail -5 "$OUT/main_$compat.log"; exit 1; }
  e=$(date +%s.%N)
  echo "main.py --compat $compat wall_s=$(python -c "print(round($e-$s,3))") summary=$(tr -d '\n ' < "$d"/Checkpoint/Results/Update/10/*/training_summary.json)"
  rm -rf "$d"
done
d=$(mktemp -d)
timeout -k 10 300 python -m cProfile -o "$OUT/main_fixed.prof" main.py --synthetic nbaiot --compat fixed --output-root "$d" \
  --log-level WARNING > /dev/null 2>&1 || exit 1
python -c "
import pstats; s = pstats.Stats('$OUT/main_fixed.prof'); s.sort_stats('cumulative').print_stats(45)" > "$OUT/main_fixed_prof.txt"
head -70 "$OUT/main_fixed_prof.txt" | tail -55
