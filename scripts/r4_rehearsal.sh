#!/bin/bash
# Round-4 multi-rank rehearsal on the one-GPU box (gloo, ranks share cuda:0):
# the N > 1 bench record (10-client headline + weak_scaling +
# independent_federations) through the HIP engine, 2 and 4 ranks.
set -u
NRANKS=2 bash scripts/multirank_rehearsal.sh || exit 1
NRANKS=4 bash scripts/multirank_rehearsal.sh || exit 1
for n in 2 4; do grep -h '^{' gpurun_out/rehearsal_bench$n.log | python -c "
import json,sys
r=json.loads(sys.stdin.read().strip().splitlines()[-1])
print($n, 'value', r['value'], r['scaling'], r['unit'][:60], '| weak', r.get('weak_scaling',{}).get('federation_rounds_per_sec'), '| indep agg', r.get('independent_federations',{}).get('aggregate_rounds_per_sec'), '| err', r.get('extra_fields_error'))
"; done
