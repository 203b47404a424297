# Round 5: texture-path cycles of the lane-sorted scoring (CSM_LANE_SORT=1)
# against HEAD on the 16-submap C3 slice: one PMC pass each (TD_TD_BUSY,
# TA_BUFFER_READ_WAVEFRONTS), to separate the sort's cost on wave 0 from
# what the grouping saves in the texture path.
set -u
O=gpurun_out/r5u
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
for v in base lanesort; do
  lib=$R/cartographer-1_amd/libcsm_amd.so
  [ $v = lanesort ] && lib=$R/variants/lanesort/libcsm_amd.so
  (cd /tmp && export TMPDIR=/tmp && CSM_AMD_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum \
    -d $R/$O/pmc_$v/p0 -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 \
    --c3-slice 16 > $R/$O/pmc_$v.json 2> $R/$O/pmc_$v.log) || { echo "pmc pass $v failed"; tail -5 $O/pmc_$v.log; exit 1; }
  echo "$v"; python3 tools/pmc_sum.py $O/pmc_$v fast2d_search | tee $O/pmc_${v}_summary.txt
done
