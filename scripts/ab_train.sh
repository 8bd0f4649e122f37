#!/bin/bash
# GPU side of scripts/ab_variants.py: train-kernel timing of every built
# variant library, each in its own process with its own time limit, twice
# in alternating order (clock drift shows up as a base/base difference).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=${OUTAB:-$ROOT/gpurun_out/ab}
mkdir -p "$OUT"
# AB_LIBS="base hwscaled0 ...": only these variants ("main" = the production libfedmx_hip.so)
if [ -n "${AB_LIBS:-}" ]; then
  LIBS=""
  for n in $AB_LIBS; do
    if [ "$n" = main ]; then LIBS="$LIBS fedmse_decentralized_amd/ops/lib/libfedmx_hip.so";
    else LIBS="$LIBS fedmse_decentralized_amd/ops/lib/libfedmx_hip_$n.so"; fi
  done
else
  LIBS=$(ls fedmse_decentralized_amd/ops/lib/libfedmx_hip_*.so | grep -v stamps)
fi
for rep in $(seq 1 ${AB_REPS:-3}); do
  for lib in $LIBS; do
    name=$(basename "$lib" .so)
    FEDMX_HIP_LIB=$ROOT/$lib timeout -k 10 120 python scripts/bench_kernels.py --train-only --reps 15 \
      > "$OUT/$name.$rep.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -n 5 "$OUT/$name.$rep.log"; exit $rc; fi
    echo "$rep $name $(tail -n 1 "$OUT/$name.$rep.log")"
  done
done
