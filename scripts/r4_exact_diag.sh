#!/bin/bash
# default build twice, IEEE-Adam build twice, then all compared (see r4_exact_diag.py)
set -u
OUT=gpurun_out/exact
mkdir -p $OUT
L=fedmse_decentralized_amd/ops/lib
for run in def1:libfedmx_hip.so exact1:libfedmx_hip_exact.so def2:libfedmx_hip.so exact2:libfedmx_hip_exact.so; do
  n=${run%%:*}; lib=${run#*:}
  FEDMX_HIP_LIB=$PWD/$L/$lib timeout -k 10 120 python scripts/r4_exact_diag.py --out $OUT/$n.npz > $OUT/$n.log 2>&1 \
    || { echo "$n failed"; tail -n 20 $OUT/$n.log; exit 1; }
done
python scripts/r4_exact_diag.py --compare $OUT/def1.npz $OUT/def2.npz $OUT/exact1.npz $OUT/exact2.npz
python scripts/r4_exact_diag.py --compare $OUT/exact1.npz $OUT/exact2.npz
