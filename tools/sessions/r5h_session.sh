# Round 5: the C3 kernel's 4-lane groups. (1) CSM_KPROF passes (16-submap
# slice) at HEAD and with CSM_LANE_SORT=1 (scoring lanes take the batch in
# (level, rotation, y, x) order; node slots and push order unchanged):
# distinct lines and quad lines (distinct lines summed over 4-lane groups)
# per gather; (2) one C3 step each, A/B twice, the same accepted count
# required; (3) the gather-pattern microbenchmark (TD cycles per line by
# lane arrangement) -> profiles.
set -u
O=gpurun_out/r5h
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
for v in kprof5 kprof5ls; do
  CSM_PROFILE2D=1 CSM_AMD_LIB=$R/variants/$v/libcsm_amd.so timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d \
    --steps 1 --warmup 0 --c3-slice 16 > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  echo "$v"; grep "lines per gather" $O/$v.err | tail -2
done
date +%T
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run base $R/cartographer-1_amd/libcsm_amd.so
  run lanesort $R/variants/lanesort/libcsm_amd.so
done
date +%T
timeout -k 10 120 ./tools/gather_pattern_bench > $O/gather_pattern.txt 2>&1 || { cat $O/gather_pattern.txt; exit 1; }
cat $O/gather_pattern.txt
date +%T
