# timing-only ablations of the fused verification kernel (wrong numerics,
# never shipped): kernel time without the forward / drift / adoption pass
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p "$ROOT/gpurun_out/va"
for v in base vabl1 vabl2 vabl4; do
  if [ $v = base ]; then L="$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip.so"; else L="$ROOT/fedmse_decentralized_amd/ops/lib/libfedmx_hip_$v.so"; fi
  FEDMX_HIP_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/va/$v" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 > "$ROOT/gpurun_out/va/$v.log" 2>&1 || exit $?
done
