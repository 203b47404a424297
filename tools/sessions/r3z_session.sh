# Full GPU tests at the current tree (full batches, raw level-1 lists), then
# a C3 one-step sweep of settings that may move with fuller batches.
set -u
O=gpurun_out/r3z
mkdir -p $O
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
for cfg in "" "CSM_HEX_LEVELS=8" "CSM_HEX_LEVELS=8,6,4" "CSM_ROT_CHUNK=4" "CSM_WG_PER_CU=5" "CSM_SEARCH_ORDER=lifo" "CSM_CLUSTER=0,0,1,2,2,3,3,3,3" ""; do
  env $cfg timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
    > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('[$cfg]', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
done
