#!/bin/bash
# Round-4 PMC comparison of the training kernel: production vs red8 vs noiglp
# (two counter passes each, kernel-trace only; see profiles/r4_step_isa_timeline.md)
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
OUT=gpurun_out/r4g
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
L=$PWD/fedmse_decentralized_amd/ops/lib
for v in hip hip_red8 hip_noiglp; do
  n=1
  for P in "$P1" "$P2"; do
    FEDMX_HIP_LIB=$L/libfedmx_$v.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $OUT/${v}_p$n -o pmc \
      -- python3 scripts/pmc_train_only.py > $OUT/${v}_p$n.log 2>&1 || { echo "$v pass $n rc=$?"; tail -n 20 $OUT/${v}_p$n.log; exit 1; }
    echo "$v pass $n ok"
    n=$((n + 1))
  done
done
