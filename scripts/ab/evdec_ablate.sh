set -u
O=gpurun_out/evdec; mkdir -p $O
for pass in 1 2 3; do for a in 1 0; do
  FEDMX_ABLATE_EVDEC=$a timeout -k 10 150 python bench.py --steps 300 --warmup 20 --out $O/a${a}_$pass.json > /dev/null 2>&1 || exit $?
  python -c "import json; r=json.load(open('$O/a${a}_$pass.json')); print('abl=$a pass=$pass', r['ms_per_step'], r['value'])"
done; done
