# Hex level sets and cluster sizes at the full-batch kernel, C3 one step each.
set -u
O=gpurun_out/r3am
mkdir -p $O
for cfg in "" "CSM_HEX_LEVELS=8,6,3" "CSM_HEX_LEVELS=8,5" "CSM_HEX_LEVELS=7,5" "CSM_HEX_LEVELS=8,6,2" "CSM_CLUSTER=0,0,2,1,2,3,3,3,3" "CSM_CLUSTER=0,0,2,2,3,3,3,3,3" "CSM_CLUSTER=0,0,2,2,2,3,2,3,3" ""; do
  env $cfg timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
    > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('[$cfg]', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
done
