# Round 4: C5 at HEAD with the submap builds inside the step; kernel trace and
# PMC passes of fast3d_search on the same C5 leg (evidence for DESIGN §8b).
set -u
O=gpurun_out/r4d
R=$PWD
mkdir -p $O/pmc3d
timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
cat $O/c5.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c5trace \
  -o c5 --output-format csv -- python3 $R/tools/probe_c5.py > $R/$O/c5trace.json 2> $R/$O/c5trace.err) \
  || { tail -20 $O/c5trace.err; exit 1; }
i=0
for g in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
         "TD_TD_BUSY_sum GRBM_COUNT" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $g -d $R/$O/pmc3d/p$i -o run \
    --output-format csv -- python3 $R/tools/probe_c5.py > $R/$O/pmc3d/p$i.json 2> $R/$O/pmc3d/p$i.log) \
    || { echo "pmc pass $i failed"; tail -5 $O/pmc3d/p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_sum.py $O/pmc3d fast3d_search > $O/pmc3d/pmc_c5_summary.txt
cat $O/pmc3d/pmc_c5_summary.txt
