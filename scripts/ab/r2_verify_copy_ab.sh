# A/B: best -> best_stage snapshot copy in extra workgroups of the fused
# verification launch (HEAD) vs in its adoption pass (libfedmx_hip_vb.so);
# kernel time from rocprofv3 kernel traces, then the bench, interleaved
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/vc
mkdir -p $O
L=$ROOT/fedmse_decentralized_amd/ops/lib
cd /tmp && export TMPDIR=/tmp
for v in vb main; do
  if [ $v = main ]; then lib=$L/libfedmx_hip.so; else lib=$L/libfedmx_hip_$v.so; fi
  FEDMX_HIP_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/prof_$v" -o run -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 > "$ROOT/$O/prof_$v.log" 2>&1 || exit $?
done
cd "$ROOT"
for i in 1 2; do
  for v in vb main; do
    if [ $v = main ]; then lib=$L/libfedmx_hip.so; else lib=$L/libfedmx_hip_$v.so; fi
    FEDMX_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 100 --warmup 10 --out $O/bench_${v}_$i.json > /dev/null 2>&1 || exit $?
    python -c "import json; r=json.load(open('$O/bench_${v}_$i.json')); print('bench $v.$i', r['ms_per_step'], r['detection_auc_mean'])"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_device_protocol_gpu.py -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 1 $O/pytest.log; exit $rc
