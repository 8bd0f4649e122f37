#!/bin/bash
# Round-4 A/B: iglp_opt strategy of the step loop (noiglp / iglp1) against the
# production build (base); bit-identity checks first.
set -u
rm -rf gpurun_out/ab
AB_REPS=2 AB_CHECK="noiglp iglp1" bash scripts/r4_ab.sh || exit 1
