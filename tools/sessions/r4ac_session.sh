# Round 4: C3 PMC with and without queue spreading (one 16-submap slice):
# L2 hits/misses, TA/TD busy, GPU-busy cycles of fast2d_search_v4.
set -u
O=gpurun_out/r4ac
R=$PWD
mkdir -p $O/s0 $O/s1
for sp in 0 1; do
  i=0
  for g in "TCC_HIT_sum TCC_MISS_sum" "TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"; do
    (cd /tmp && export TMPDIR=/tmp && CSM_QUEUE_SPREAD=$sp timeout -s KILL 240 rocprofv3 --pmc $g -d $R/$O/s$sp/p$i -o run \
      --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 --c3-slice 16 \
      > $R/$O/s$sp/p$i.json 2> $R/$O/s$sp/p$i.log) || { echo "pmc pass failed"; tail -5 $O/s$sp/p$i.log; exit 1; }
    i=$((i+1))
  done
  python3 tools/pmc_sum.py $O/s$sp fast2d_search_v4 > $O/s$sp/summary.txt
  echo "spread=$sp"; cat $O/s$sp/summary.txt
done
