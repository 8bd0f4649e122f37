# fwd_rows rows-per-block sweep at the 8-rank phantom (dev set 80 clients):
# workgroup residency is 2 per CU at the kernel's VGPR count, not the 4 the
# LDS allows; kernel time per setting from rocprofv3 stats
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p "$ROOT/gpurun_out/rpb"
for r in 0 128 192 448 576 704; do
  FEDMX_FWD_ROWS_PER_BLOCK=$r timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/rpb/p8_$r" -o run -- python3 "$ROOT/bench.py" --phantom-ranks 8 --steps 10 --warmup 3 > "$ROOT/gpurun_out/rpb/p8_$r.log" 2>&1 || exit $?
done
for r in 0 128 192 448 576 704; do
  FEDMX_FWD_ROWS_PER_BLOCK=$r timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/rpb/c64_$r" -o run -- python3 "$ROOT/bench.py" --clients 64 --data-kind kitsune --non-iid --steps 10 --warmup 3 --no-artifacts > "$ROOT/gpurun_out/rpb/c64_$r.log" 2>&1 || exit $?
done
