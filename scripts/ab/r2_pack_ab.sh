# A/B: the multi-rank pack inside the score-reduction launch (HEAD) vs its
# own copy_rows launch (FEDMX_PACK_SEPARATE=1) on the 8-rank phantom
# projection, interleaved; the multi-rank / IPC GPU tests first
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/pk
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_device_protocol_gpu.py tests/test_ipc_gpu.py -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --phantom-ranks 8 --steps 200 --warmup 20 --out $O/ph8_new_$i.json > /dev/null 2>&1 || exit $?
  FEDMX_PACK_SEPARATE=1 timeout -k 10 240 python bench.py --phantom-ranks 8 --steps 200 --warmup 20 --out $O/ph8_old_$i.json > /dev/null 2>&1 || exit $?
  python -c "import json; a=json.load(open('$O/ph8_new_$i.json')); b=json.load(open('$O/ph8_old_$i.json')); print('ph8 fused', a['ms_per_step'], 'separate', b['ms_per_step'], a['detection_auc_mean'], b['detection_auc_mean'])"
done
