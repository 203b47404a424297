# Round 4: C3 PMC, default build vs 8-byte hex planes (variants/hex8,
# -DCSM_HEX8=1): L2 hits/misses and TA/TD busy of fast2d_search_v4 on one
# 16-submap slice, to see whether the smaller planes cut L2 misses.
set -u
O=gpurun_out/r4ah
R=$PWD
mkdir -p $O/default $O/hex8
for v in default hex8; do
  lib=$R/cartographer-1_amd/libcsm_amd.so
  [ $v = hex8 ] && lib=$R/variants/hex8/libcsm_amd.so
  i=0
  for g in "TCC_HIT_sum TCC_MISS_sum" "TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"; do
    (cd /tmp && export TMPDIR=/tmp && CSM_AMD_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc $g -d $R/$O/$v/p$i -o run \
      --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 --c3-slice 16 \
      > $R/$O/$v/p$i.json 2> $R/$O/$v/p$i.log) || { echo "pmc pass failed"; tail -5 $O/$v/p$i.log; exit 1; }
    i=$((i+1))
  done
  python3 tools/pmc_sum.py $O/$v fast2d_search_v4 > $O/$v/summary.txt
  echo "$v"; cat $O/$v/summary.txt
done
