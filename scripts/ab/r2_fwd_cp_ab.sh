# compact-order forward vs identity-order forward (libfedmx_hip_idfwd.so):
# alternating 1-GPU headline and 64-client benches on one box
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/cpab
OLD="$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip_idfwd.so"
for i in 1 2; do
  FEDMX_HIP_LIB=$OLD timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out gpurun_out/cpab/n1_id_$i.json > /dev/null 2>&1 || exit $?
  timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out gpurun_out/cpab/n1_cp_$i.json > /dev/null 2>&1 || exit $?
  FEDMX_HIP_LIB=$OLD timeout -k 10 120 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 100 --warmup 20 --no-artifacts --out gpurun_out/cpab/c64_id_$i.json > /dev/null 2>&1 || exit $?
  timeout -k 10 120 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 100 --warmup 20 --no-artifacts --out gpurun_out/cpab/c64_cp_$i.json > /dev/null 2>&1 || exit $?
done
for f in gpurun_out/cpab/*.json; do python -c "import json; r=json.load(open('$f')); print('$f', r['ms_per_step'], r['value'], r['detection_auc_mean'])"; done
