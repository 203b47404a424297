#!/bin/bash
# Round 6 closing set, part 1: every GPU test and smoke() at HEAD, then the
# C5 PMC set of fast3d_search (KERNEL3D_TAG f3-octet-trim: loads cut to the
# cloud) reduced into gpurun_out/r6l/profile/ (committed as profiles/r6l/).
set -u
O=gpurun_out/r6l
R=${GRAFT_REPO_ROOT:-$PWD}
P=$O/profile
mkdir -p $O $P
date +%T
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread --durations=20 \
  > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
date +%T
bash tools/gpu_measure.sh $O c5 || exit 1
cp $O/c5.json $P/c5.json
python3 tools/profiles.py reduce-pmc $O/pmc3d $P/c5_pmc.csv fast3d_search || exit 1
cp $O/pmc3d/pmc_c5_summary.txt $P/ 2>/dev/null
tail -3 $O/gputests.log > $P/gputests_tail.txt
grep -E "PASSED|FAILED" $O/gputests.log | wc -l >> $P/gputests_tail.txt
cp $O/smoke.log $P/
date +%T
