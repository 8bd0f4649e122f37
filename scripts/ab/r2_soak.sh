# r2 end: soak runs (ring wrap-around, writer backlog, episode resets, long
# run-ahead): 5,000 rounds of the headline config with every artefact, 1,000
# rounds of 64 Kitsune-shaped non-IID clients, the full reference sweep
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/soak
mkdir -p $O
timeout -k 10 300 python bench.py --steps 5000 --warmup 20 --out $O/n1_5000.json > /dev/null 2> $O/n1_5000.err || exit $?
timeout -k 10 300 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 1000 --warmup 20 --out $O/k64_1000.json > /dev/null 2> $O/k64_1000.err || exit $?
timeout -k 10 300 python main.py --synthetic nbaiot --num-rounds 20 --epoch 5 --compat fixed --output-root $O/sweep --log-level WARNING > $O/sweep.log 2>&1 || exit $?
for f in $O/*.json; do python -c "import json; r=json.load(open('$f')); print('$f', r['steps'], r['ms_per_step'], r['federation_rounds_per_sec'], r['detection_auc_mean'], r['writer_busy_ms_per_round'])"; done
python -c "import json; print(open('$O/sweep/Checkpoint/Results/Update/10/' + __import__('os').listdir('$O/sweep/Checkpoint/Results/Update/10')[0] + '/training_summary.json').read())"
