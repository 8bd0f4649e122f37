# BASELINE config 5 (64-client non-IID Kitsune-shaped federation) on one GPU, and the
# driver's torch.distributed.run launch form at nproc 1 (RCCL process group of one rank).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/cfg
timeout -k 10 180 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 5 --out gpurun_out/cfg/kitsune64.json > gpurun_out/cfg/kitsune64.log 2>&1 || exit $?
tail -c 400 gpurun_out/cfg/kitsune64.json; echo
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 50 --warmup 5 > gpurun_out/cfg/torchrun1.json 2> gpurun_out/cfg/torchrun1.log || exit $?
cat gpurun_out/cfg/torchrun1.json
