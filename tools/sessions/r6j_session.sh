#!/bin/bash
# Round 6: batch node slots sorted by (level, rotation, y, x) so the flat
# scoring lanes' 4-lane groups hold x-adjacent nodes (variants/slotsort,
# CSM_SLOT_SORT=1) against HEAD, one C3 step each alternating; then the KPROF
# line / quad-line counts of the sorted build on the 16-submap slice.
set -u
O=gpurun_out/r6j
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$1', round(d['value'], 1), round(r['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], [round(c) for c in d['search_levels']['candidates_per_pair']])" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run base $R/cartographer-1_amd/libcsm_amd.so || exit 1
  run slotsort $R/variants/slotsort/libcsm_amd.so || exit 1
done
CSM_PROFILE2D=1 CSM_AMD_LIB=$R/variants/kprof_ss/libcsm_amd.so timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d \
  --steps 1 --warmup 0 --c3-slice 16 > $O/kprof.json 2> $O/kprof.err || { tail -20 $O/kprof.err; exit 1; }
grep "lines per gather" $O/kprof.err | head -4
