#!/bin/bash
# Round-6 FedProx: the main waves' anchor slabs in LDS (fedmx_train_hw.hip
# L_AN) -- the FedProx numerics tests, then the training launches.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/${TAG:-s25}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_long_horizon_gpu.py tests/test_engine_parity_gpu.py > $OUT/pytest.log 2>&1 \
  || { echo tests failed; tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
for r in 1 2 3; do
  timeout -k 10 200 python scripts/bench_kernels.py > $OUT/kernels.$r.json 2> $OUT/kernels.$r.err || { echo bench_kernels failed; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['train_launch_us'], d['train_launch_fedprox_us'], d['train_launch_b64_us'])" $OUT/kernels.$r.json
done
