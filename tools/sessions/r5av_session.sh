# Round 5: does a larger item (more rotations per workgroup item, so more
# nodes per batch) pay at equal occupancy? One C3 step each: rotations per
# item 2/3/4 at 4 and 3 workgroups per CU (CSM_ROT_CHUNK, CSM_WG_PER_CU),
# and the default (2 at 6 per CU).
set -u
O=gpurun_out/r5av
mkdir -p $O
run() {  # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
lv=d['search_levels']['mean_lanes_per_batch']
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], [round(x, 1) for x in lv[:9]])" | tee -a $O/ab_summary.txt
}
run default CSM_PROFILE2D=1
run r2w4 CSM_ROT_CHUNK=2 CSM_WG_PER_CU=4
run r3w4 CSM_ROT_CHUNK=3 CSM_WG_PER_CU=4
run r2w3 CSM_ROT_CHUNK=2 CSM_WG_PER_CU=3
run r4w3 CSM_ROT_CHUNK=4 CSM_WG_PER_CU=3
run r3w3 CSM_ROT_CHUNK=3 CSM_WG_PER_CU=3
grep "fast2d launch" $O/ab.err | head -2
