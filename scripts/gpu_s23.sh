#!/bin/bash
# Round-6 FedProx instantiation in its own translation unit with memory
# clustering off (build.SOURCE_FLAGS): the GPU suite, the training launches
# (scripts/bench_kernels.py, twice) and FedProx federations end to end.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/${TAG:-s23}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { echo tests failed; tail -n 30 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 200 python scripts/bench_kernels.py > $OUT/kernels.$r.json 2> $OUT/kernels.$r.err || { echo bench_kernels failed; exit 1; }
  tail -n 1 $OUT/kernels.$r.json | cut -c1-240
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --update-type fedprox --out $OUT/fedprox200.$r.json \
    > $OUT/fedprox200.$r.log 2>&1 || { echo bench failed; tail $OUT/fedprox200.$r.log; exit 1; }
  tail -n 1 $OUT/fedprox200.$r.log | cut -c1-160
done
