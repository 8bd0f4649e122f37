# r2 end: paper configuration, BASELINE config 5 (64 Kitsune-shaped non-IID
# clients) and a 256-client federation on one GPU at HEAD
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/cfg
mkdir -p $O
timeout -k 10 200 python bench.py --epochs 100 --lr 1e-5 --shrink-lambda 10 --steps 20 --warmup 3 --out $O/paper.json > /dev/null 2>&1 || exit $?
timeout -k 10 200 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 20 --out $O/k64_w20.json > /dev/null 2>&1 || exit $?
timeout -k 10 300 python bench.py --clients 256 --steps 10 --warmup 10 --out $O/n256.json > /dev/null 2>&1 || exit $?
for f in $O/*.json; do python -c "import json; r=json.load(open('$f')); print('$f', r['ms_per_step'], r['value'], r['federation_rounds_per_sec'], r.get('detection_auc_mean'))"; done
