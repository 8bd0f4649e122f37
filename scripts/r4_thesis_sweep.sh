#!/bin/bash
# The thesis's GPU setting (batch 64, 100 % participation; Thesis p.28-30,
# SURVEY 6.2) at the paper's local hyper-parameters (100 epochs, lr 1e-5,
# lambda 10), all six model x update combinations, 10 rounds, synthetic
# N-BaIoT IID: wall clock of the whole sweep incl. start-up and artefacts.
set -u
O=gpurun_out/r4thesis; rm -rf $O; mkdir -p $O
start=$(date +%s.%N)
timeout -k 10 900 python main.py --synthetic nbaiot --compat fixed --batch-size 64 --num-participants 1.0 \
  --epoch 100 --lr-rate 1e-5 --shrink-lambda 10 --num-rounds 10 --output-root $O/out --log-level WARNING \
  > $O/main.log 2>&1 || { echo "rc=$?"; tail -n 30 $O/main.log; exit 1; }
end=$(date +%s.%N)
python - "$start" "$end" "$O" <<'PY'
import glob, json, os, sys
start, end, O = float(sys.argv[1]), float(sys.argv[2]), sys.argv[3]
print(json.dumps({"wall_s": round(end - start, 2)}))
for f in sorted(glob.glob(os.path.join(O, "out", "**", "*_results.json"), recursive=True)):
    try:
        r = json.load(open(f))
    except Exception:
        continue
    print(os.path.basename(f), json.dumps(r)[:400])
PY
