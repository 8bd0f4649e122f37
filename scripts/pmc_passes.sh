#!/bin/bash
# PMC counters of the training kernel (scripts/pmc_train_only.py: five 5-client
# launches of the benchmark workload) for each library variant in $LIBS
# ("main" = the production libfedmx_hip.so, else libfedmx_hip_<name>.so): two
# 8-counter SQ passes per variant, kernel trace only, each pass under its own
# hard time limit; markdown summaries via scripts/prof_summary.py --pmc.
# Output: gpurun_out/$TAG/<variant>_p<n>/ and gpurun_out/$TAG/pmc.md.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
TAG=${TAG:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
L=$ROOT/fedmse_decentralized_amd/ops/lib
: > $OUT/pmc.md
for v in ${LIBS:-main}; do
  if [ "$v" = main ]; then lib=$L/libfedmx_hip.so; else lib=$L/libfedmx_hip_$v.so; fi
  n=1
  for P in "$P1" "$P2"; do
    FEDMX_HIP_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $OUT/${v}_p$n -o pmc \
      -- python3 scripts/pmc_train_only.py > $OUT/${v}_p$n.log 2>&1 || { echo "$v pass $n rc=$?"; tail -n 20 $OUT/${v}_p$n.log; exit 1; }
    db=$(find $OUT/${v}_p$n -name "*.db" | head -n 1)
    python3 scripts/prof_summary.py "$db" --pmc --kernel train_kernel --title "PMC $v pass $n" >> $OUT/pmc.md
    echo "$v pass $n ok"
    n=$((n + 1))
  done
done
