#!/bin/bash
set -u
mkdir -p gpurun_out/split
for v in ${DIAG_LIBS:-hwsplit base}; do
FEDMX_HIP_LIB=$PWD/fedmse_decentralized_amd/ops/lib/libfedmx_hip_$v.so timeout -k 10 120 python scripts/r4_split_diag.py > gpurun_out/split/diag_$v.txt 2>&1; echo "diag $v rc=$?"; grep -v amdgpu.ids gpurun_out/split/diag_$v.txt | python -c "
import sys, ast
for l in sys.stdin:
    l=l.strip()
    if not l.startswith('{'): print(l); continue
    d=ast.literal_eval(l); print(d['steps'], 'train', d['train_loss_diff'], 'valid', d['valid_loss_diff'], 'per-client params', d['w1_rows_per_client'], 'W1a', d['params'][0], 'W1b', d['params'][1], 'W4', d['params'][7])"
done
