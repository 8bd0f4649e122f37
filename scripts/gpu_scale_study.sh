set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/network_scale.py --clients 10 20 30 40 50 80 256 --rounds 50 --out gpurun_out/scale_shared.jsonl > gpurun_out/scale_shared.log 2>&1 &&
timeout -k 10 300 python -u scripts/network_scale.py --clients 10 80 256 --rounds 50 --split iid --init-mode per_client --out gpurun_out/scale_per_client.jsonl > gpurun_out/scale_per.log 2>&1 &&
timeout -k 10 300 python -u scripts/network_scale.py --clients 10 --participation 0.5 0.6 0.7 0.8 0.9 1.0 --rounds 50 --out gpurun_out/ratio.jsonl > gpurun_out/ratio.log 2>&1
