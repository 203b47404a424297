#!/bin/bash
# Round 6 closing set, part 2: the default bench.py run under
# rocprofv3 --kernel-trace --stats; its search dispatches reduced with
# tools/profiles.py (gpurun_out/r6m/profile/, committed as profiles/r6m/)
# for trace_summary.json (the timed C3 chunk launches by trace against the
# bench's HIP events).
set -u
O=gpurun_out/r6m
R=${GRAFT_REPO_ROOT:-$PWD}
P=$O/profile
mkdir -p $O $P
date +%T
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o bench \
  --output-format csv -- python3 $R/bench.py > $R/$P/bench_full.json 2> $R/$O/bench_full.err) \
  || { tail -30 $O/bench_full.err; exit 1; }
date +%T
python3 tools/profiles.py reduce-trace $O/trace/bench_kernel_trace.csv $P/bench_trace.csv fast2d_search fast3d_search || exit 1
cp $O/trace/bench_kernel_stats.csv $P/ 2>/dev/null
tail -5 $O/bench_full.err > $P/bench_full_err_tail.txt
