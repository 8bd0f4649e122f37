#!/bin/bash
# Round-4 A/B: per-epoch Adam-scalar table (FEDMX_HW_KTAB) vs production
set -u
rm -rf gpurun_out/ab
AB_REPS=3 AB_CHECK="ktab" bash scripts/r4_ab.sh || exit 1
