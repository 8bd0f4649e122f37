set -u
O=gpurun_out/initab; mkdir -p $O
for pass in 1 2; do for m in shared per_client; do
  timeout -k 10 120 python bench.py --init-mode $m --out $O/d_${m}_$pass.json > /dev/null 2>&1 || exit $?
  timeout -k 10 150 python bench.py --init-mode $m --steps 300 --warmup 20 --out $O/l_${m}_$pass.json > /dev/null 2>&1 || exit $?
done; done
for f in $O/*.json; do python -c "import json; r=json.load(open('$f')); print('$f', r['ms_per_step'], r['value'], r['local_epochs_run_mean'], r['detection_auc_mean'])"; done
