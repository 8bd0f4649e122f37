#!/bin/bash
# Round-4 soak on the final tree: 3,000 headline rounds, the thesis's batch-64
# configuration (the helper-wave kernel's 16-row-chunk path) plain and
# FedProx, 1,000 rounds of 64 Kitsune-shaped non-IID clients, 100 paper-config
# rounds; every run writes its reports / checkpoints.
set -u
O=gpurun_out/r4soak; mkdir -p $O
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" --out $O/$n.json > /dev/null 2> $O/$n.err || { echo "$n rc=$?"; tail -n 20 $O/$n.err; exit 1; }; echo "$n ok"; }
run headline3000 --steps 3000 --warmup 20
run b64_2000 --batch-size 64 --steps 2000 --warmup 20
run b64_prox_1000 --batch-size 64 --update-type fedprox --steps 1000 --warmup 20
run k64_1000 --clients 64 --data-kind kitsune --non-iid --steps 1000 --warmup 20
run paper100 --epochs 100 --lr 1e-5 --shrink-lambda 10 --steps 100 --warmup 5
for f in $O/*.json; do python -c "import json; r=json.load(open('$f')); print('$f', r['ms_per_step'], r['value'], r['local_epochs_run_mean'], r['detection_auc_mean'], r['detection_auc_min'])"; done
