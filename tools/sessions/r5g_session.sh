# Round 5: (1) the C3 kernel's texture-path ceiling at HEAD: a CSM_KPROF pass
# (distinct lines per gather by child level) and a TD/TA PMC pass on the same
# 16-submap slice -> profiles/r5g/gather_c3.json (bench.py gather_roofline);
# (2) scan-cluster sizes per child level re-swept on C3 (CSM_CLUSTER; chosen
# on C2 in rounds 2-3). One C3 step each, the same accepted count required.
set -u
O=gpurun_out/r5g
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
TAG=$(python3 -c "import sys; sys.path.insert(0,'.'); import bench; print(bench.KERNEL_TAG)")
date +%T
CSM_PROFILE2D=1 CSM_AMD_LIB=$R/variants/kprof5/libcsm_amd.so timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d \
  --steps 1 --warmup 0 --c3-slice 16 > $O/kprof.json 2> $O/kprof.err || { tail -20 $O/kprof.err; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum \
  -d $R/$O/pmc_td -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 \
  --c3-slice 16 > $R/$O/pmc_td.json 2> $R/$O/pmc_td.log) || { echo "pmc pass failed"; tail -5 $O/pmc_td.log; exit 1; }
python3 tools/gather_roofline.py $O/kprof.err $O/pmc_td $O/gather_c3.json $TAG || exit 1
date +%T
run() {  # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
for c in 0,0,2,2,2,3,3,3,3,3,3,3 0,1,2,2,2,3,3,3,3,3,3,3 0,0,1,2,2,3,3,3,3,3,3,3 0,1,1,2,2,3,3,3,3,3,3,3 \
         0,0,1,1,2,3,3,3,3,3,3,3 0,0,2,3,2,3,3,3,3,3,3,3 0,0,2,2,3,3,3,3,3,3,3,3 0,0,2,2,2,3,2,3,3,3,3,3 \
         0,0,2,2,2,3,3,3,3,3,3,3; do
  run cluster=$c CSM_CLUSTER=$c
done
# Hex-level sets not measured on C3 in round 4 (r4ad had {8,6} best of six).
for v in 8 6 8,6,2 8,6; do run hex=$v CSM_HEX_LEVELS=$v; done
date +%T
