#!/bin/bash
# Round-4 A/B: iglp_opt hints in the mains' forward segment / the helpers' step
set -u
rm -rf gpurun_out/ab
AB_REPS=2 AB_CHECK="iglpfw0 iglpfw1 iglph0 iglpboth" bash scripts/r4_ab.sh || exit 1
