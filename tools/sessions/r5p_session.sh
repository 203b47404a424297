# Round 5: (1) L2 hit rate of fast2d_search on the 16-submap C3 slice (one
# PMC pass: TCC_HIT, TCC_MISS), the check on the reading that the 4.03 TD
# cycles per line come from lines served past L2 (EXPERIMENTS.md round 5);
# (2) the drop-in coalescing sweep (tools/sessions/r5d_session.sh).
set -u
O=gpurun_out/r5p
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum \
  -d $R/$O/pmc_l2 -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 \
  --c3-slice 16 > $R/$O/pmc_l2.json 2> $R/$O/pmc_l2.log) || { echo "pmc pass failed"; tail -5 $O/pmc_l2.log; exit 1; }
python3 tools/pmc_sum.py $O fast2d_search > $O/pmc_l2_summary.txt || exit 1
cat $O/pmc_l2_summary.txt
date +%T
bash tools/sessions/r5d_session.sh || exit 1
