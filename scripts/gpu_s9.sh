set -u
# Round-6 soak and scale records on the final build: 10,000 headline rounds in
# one process (no failed launch, AUC steady), the 256-client federation
# (validators for 128 trainers, split verification over 256 receivers) and
# the 64-client non-IID Kitsune-shaped configuration of BASELINE.json.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; OUT=gpurun_out/s9; mkdir -p $OUT
timeout -k 10 300 python bench.py --gpus 1 --steps 10000 --warmup 5 --out $OUT/soak_10000.json > $OUT/soak.log 2>&1 || { echo soak failed; tail $OUT/soak.log; exit 1; }
tail -n 1 $OUT/soak.log | cut -c1-200
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 3 --clients 256 --out $OUT/clients256.json > $OUT/c256.log 2>&1 || { echo c256 failed; tail $OUT/c256.log; exit 1; }
tail -n 1 $OUT/c256.log | cut -c1-200
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 3 --clients 64 --data-kind kitsune --non-iid --out $OUT/kitsune64_noniid.json > $OUT/k64.log 2>&1 || { echo k64 failed; tail $OUT/k64.log; exit 1; }
tail -n 1 $OUT/k64.log | cut -c1-200
