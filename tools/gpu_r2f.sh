#!/bin/bash
# Round 2: RTCSM2D rebuild (rt2d.hip) and the search-space exports: the GPU
# suite, then the C1 probe plain and under a kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r2f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u tools/rt2d_probe.py > $O/rt2d.json 2> $O/rt2d.err || { echo "probe failed"; tail -20 $O/rt2d.err; exit 1; }
cat $O/rt2d.json
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u tools/rt2d_probe.py > $O/rt2d_prof.json 2> $O/rt2d_prof.err || { echo "prof failed"; tail -20 $O/rt2d_prof.err; exit 1; }
find $O/prof -name "*stats*" | head
echo ALL_OK
