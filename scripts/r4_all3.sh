#!/bin/bash
# kernel A/B first (SPLIT variant checked for bit-identity first), then the
# GPU test tier + bench + paper config, the adoption ablation, a profile.
set -u
AB_REPS=2 AB_CHECK="split" bash scripts/r4_ab.sh || exit 1
bash scripts/r4_all2.sh || exit 1
