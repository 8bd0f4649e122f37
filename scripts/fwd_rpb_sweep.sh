# A/B of the fwd_rows block length on the 8-rank projection (rank 0 of the 80-client job).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/rpb
for R in 0 128 256 512 0; do
  FEDMX_FWD_ROWS_PER_BLOCK=$R timeout -k 10 120 python bench.py --phantom-ranks 8 --steps 300 --warmup 20 --out gpurun_out/rpb/r$R.json > gpurun_out/rpb/r$R.log 2>&1 || exit $?
  python -c "import json;r=json.load(open('gpurun_out/rpb/r$R.json'));print('rpb=$R', r['ms_per_step'])"
done
