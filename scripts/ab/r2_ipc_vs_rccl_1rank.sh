# one-GPU cost of the two per-round collectives: loopback (no collectives) vs
# a one-rank RCCL group vs one-rank peer-memory channels, both with
# FEDMX_FORCE_COLLECTIVES=1 (the multi-GPU code path: pack, exchange, unpack);
# interleaved, 300 timed rounds each
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/ipc1
mkdir -p $O
port=29611
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 20 --out $O/loop_$i.json > /dev/null 2> $O/loop_$i.err || exit $?
  for mode in rccl ipc; do
    port=$((port + 1))
    WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port FEDMX_FORCE_COLLECTIVES=1 \
      timeout -k 10 120 python bench.py --steps 300 --warmup 20 --comm $mode --out $O/${mode}_$i.json \
      > /dev/null 2> $O/${mode}_$i.err || exit $?
  done
done
for f in $O/*.json; do python -c "import json; r=json.load(open('$f')); print('$f', r['ms_per_step'], r['detection_auc_mean'], r['config']['parallelism'])"; done
