#!/bin/bash
# Round-6 re-check of the scoring forward's rows per workgroup on the final
# build (FEDMX_FWD_ROWS_PER_BLOCK overrides fwd_rows_per_block: 0 = the
# heuristic, 128 rows at the headline): end-to-end A/B, alternating passes.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/${TAG:-s15}; mkdir -p $OUT
for rep in 1 2; do
  for r in 0 64 192 256; do
    FEDMX_FWD_ROWS_PER_BLOCK=$r timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --out $OUT/rpb$r.$rep.json \
      > $OUT/rpb$r.$rep.log 2>&1 || { echo bench failed; tail $OUT/rpb$r.$rep.log; exit 1; }
    echo "rows_per_block=$r rep=$rep $(tail -n 1 $OUT/rpb$r.$rep.log | cut -c1-120)"
  done
done
