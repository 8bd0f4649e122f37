#!/bin/bash
# End-to-end A/B of kernel-library variants on one GPU box: for each of $REPS
# alternating passes, every library in $AB_LIBS ("main" = the production
# build, NAME = fedmse_decentralized_amd/ops/lib/libfedmx_hip_NAME.so from
# scripts/ab_variants.py) runs `python bench.py` at the driver's defaults and
# at $LONG timed rounds (or with $LONG_ARGS instead, e.g. the paper
# configuration: LONG_ARGS="--steps 10 --warmup 2 --epochs 100 --lr 1e-5
# --shrink-lambda 10").  A library that changes the fp32 rounding also
# changes the clients' early-stopping pattern, so the short run alone can move
# either way; the long run averages that out.  Records under
# gpurun_out/$TAG/, one summary line per run on stdout.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${TAG:-bench_ab}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
L=$ROOT/fedmse_decentralized_amd/ops/lib
LONG=${LONG:-200}
LONG_ARGS=${LONG_ARGS:-"--steps $LONG --warmup 5"}
for rep in $(seq 1 ${REPS:-3}); do
  for v in ${AB_LIBS:-main}; do
    if [ "$v" = main ]; then lib=$L/libfedmx_hip.so; else lib=$L/libfedmx_hip_$v.so; fi
    FEDMX_HIP_LIB=$lib timeout -k 10 300 python bench.py > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || exit $?
    FEDMX_HIP_LIB=$lib timeout -k 10 600 python bench.py $LONG_ARGS > "$OUT/$v.long.$rep.json" \
      2>> "$OUT/$v.$rep.err" || exit $?
    python - "$OUT/$v.$rep.json" "$OUT/$v.long.$rep.json" "$rep" "$v" <<'EOF'
import json, sys
recs = [json.loads(open(p).read().strip().splitlines()[-1]) for p in sys.argv[1:3]]
print(sys.argv[3], sys.argv[4], " | ".join(f"{r['steps']} rounds: {r['value']} rounds/s, {r['local_epochs_run_mean']} epochs,"
                                          f" AUC {r.get('detection_auc_mean')}" for r in recs), flush=True)
EOF
  done
done
