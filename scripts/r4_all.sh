#!/bin/bash
# One GPU call, in priority order: kernel A/B, the GPU test tier + bench,
# the adoption ablation.  Each part stops the script on failure.
set -u
AB_REPS=${AB_REPS:-2} AB_CHECK=${AB_CHECK:-"flags flags_pipe flags2 flags2_pipe"} bash scripts/r4_ab.sh || exit 1
bash scripts/r4_gpu_check.sh gpurun_out/r4a || exit 1
bash scripts/r4_adoption.sh gpurun_out/r4_adoption || exit 1
