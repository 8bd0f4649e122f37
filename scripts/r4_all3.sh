#!/bin/bash
set -u
bash scripts/r4_all2.sh || exit 1
AB_REPS=2 AB_CHECK="flags" bash scripts/r4_ab.sh || exit 1
