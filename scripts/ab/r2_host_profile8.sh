# host-side cost per round of rank 0 at 8 ranks (phantom): bench timing and a
# cProfile of the timed rounds
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/hp
timeout -k 10 200 python bench.py --phantom-ranks 8 --steps 300 --warmup 20 --out gpurun_out/hp/ph8.json > /dev/null 2>&1 || exit $?
timeout -k 10 200 python bench.py --phantom-ranks 8 --steps 100 --warmup 20 --profile gpurun_out/hp/ph8.prof --out gpurun_out/hp/ph8p.json > /dev/null 2>&1 || exit $?
python -c "
import pstats; p = pstats.Stats('gpurun_out/hp/ph8.prof'); p.sort_stats('tottime').print_stats(25)" > gpurun_out/hp/top.txt
python -c "
import json; r=json.load(open('gpurun_out/hp/ph8.json')); t=r['phase_ms_total']; n=r['steps']
print(r['ms_per_step'], {k: round(v/n,3) for k,v in t.items()})"
