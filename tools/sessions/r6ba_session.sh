#!/bin/bash
# Round 6 final closing set: the C5 PMC set of fast3d_search at KERNEL3D_TAG
# f3-tiny5-r64-b32-box (profile/: traffic_c5 inputs), every GPU test and
# smoke(), then the default bench.py run under rocprofv3 --kernel-trace
# --stats (profile/: trace summary inputs); committed as profiles/r6ba/.
set -u
O=gpurun_out/r6ba
R=${GRAFT_REPO_ROOT:-$PWD}
P=$O/profile
mkdir -p $O $P
date +%T
bash tools/gpu_measure.sh $O c5 || exit 1
cp $O/c5.json $P/c5.json
python3 tools/profiles.py reduce-pmc $O/pmc3d $P/c5_pmc.csv fast3d_search || exit 1
cp $O/pmc3d/pmc_c5_summary.txt $P/ 2>/dev/null
date +%T
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread --durations=15 \
  > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
date +%T
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o bench \
  --output-format csv -- python3 $R/bench.py > $R/$P/bench_full.json 2> $R/$O/bench_full.err) \
  || { tail -30 $O/bench_full.err; exit 1; }
date +%T
python3 tools/profiles.py reduce-trace $O/trace/bench_kernel_trace.csv $P/bench_trace.csv fast2d_search fast3d_search || exit 1
cp $O/trace/bench_kernel_stats.csv $P/ 2>/dev/null
tail -5 $O/bench_full.err > $P/bench_full_err_tail.txt
tail -3 $O/gputests.log > $P/gputests_tail.txt
cp $O/smoke.log $P/
