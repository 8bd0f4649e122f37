# peer-memory exchange on one GPU: kernel + federation tests, then a 2-rank
# bench (both ranks on GPU 0, gloo bring-up) with the gloo collectives vs --comm ipc
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ipc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ipc_gpu.py -x -v --timeout 250 --timeout-method thread > $O/pytest_ipc.log 2>&1
rc=$?; tail -n 5 $O/pytest_ipc.log; [ $rc -eq 0 ] || exit $rc
for mode in rccl ipc; do
  FEDMX_DIST_BACKEND=gloo FEDMX_DEVICE_INDEX=0 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 \
    --comm $mode --out $O/b2_$mode.json > $O/b2_$mode.stdout 2> $O/b2_$mode.err || exit $?
  cat $O/b2_$mode.stdout
done
