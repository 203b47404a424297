#!/bin/bash
# A/B of 2D search-kernel settings on the C2 bench workload (one step after
# one warm-up, no CPU legs). Usage: tools/ab_kernel.sh OUT "VAR=VAL ..." ...
# ("" = defaults), e.g. tools/ab_kernel.sh out "" "CSM_SEARCH_KERNEL=5" "CSM_HEX_LEVELS=8,6"
set -u
OUT=$1; shift
mkdir -p $OUT
i=0
for cfg in "$@"; do
  env $cfg timeout -k 10 150 python -u bench.py --workload c2 --no-cpu --no-rt --no-3d \
    --steps 1 --warmup 1 > $OUT/ab_$i.json 2> $OUT/ab_$i.err || { tail -20 $OUT/ab_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/ab_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('[$cfg]', round(d['value'],1), 'pairs/s', round(r['kernel_ms_avg'],1), 'ms', 'accepted', d['accepted_constraints_per_step'], 'errors', d['errors_per_step'], 'GB/s', round(r['achieved']), 'hw', d['stack_high_water'])" | tee -a $OUT/ab_summary.txt
  i=$((i+1))
done
