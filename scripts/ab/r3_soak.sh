# round-3 soak: full GPU suite, 5,000 headline rounds with every artefact, 1,000 rounds of 64 Kitsune clients
set -u
O=gpurun_out/soak; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5000 --warmup 20 --out $O/soak5000.json > /dev/null 2> $O/soak5000.err || exit $?
timeout -k 10 300 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 1000 --warmup 20 --out $O/k64_1000.json > /dev/null 2> $O/k64.err || exit $?
for f in $O/*.json; do python -c "import json; r=json.load(open('$f')); print('$f', r['ms_per_step'], r['value'], r['local_epochs_run_mean'], r['detection_auc_mean'])"; done
