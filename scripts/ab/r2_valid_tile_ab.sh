# A/B of the helper-wave kernel's validation: 16-row tiles (HEAD) vs the
# previous batch-of-12 chunks (libfedmx_hip_v12.so), interleaved, then the
# kernel numerics tests and the headline bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/vt
mkdir -p $O
L=fedmse_decentralized_amd/ops/lib
for i in 1 2 3; do
  for v in v12 main; do
    if [ $v = main ]; then lib=$L/libfedmx_hip.so; else lib=$L/libfedmx_hip_$v.so; fi
    FEDMX_HIP_LIB=$ROOT/$lib timeout -k 10 120 python scripts/bench_kernels.py --train-only --reps 15 > $O/${v}_$i.json 2> $O/${v}_$i.err || exit $?
    echo "$v.$i: $(cat $O/${v}_$i.json)"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 250 --timeout-method thread > $O/pytest_kernels.log 2>&1
rc=$?; tail -n 2 $O/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in v12 main; do
    if [ $v = main ]; then lib=$L/libfedmx_hip.so; else lib=$L/libfedmx_hip_$v.so; fi
    FEDMX_HIP_LIB=$ROOT/$lib timeout -k 10 120 python bench.py --steps 100 --warmup 10 --out $O/bench_${v}_$i.json > /dev/null 2>&1 || exit $?
    python -c "import json; r=json.load(open('$O/bench_${v}_$i.json')); print('bench $v.$i', r['ms_per_step'], r['detection_auc_mean'])"
  done
done
