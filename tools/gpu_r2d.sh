#!/bin/bash
# Round 2: GPU parity suite on the current tree, then the north-star queue C3
# (2000 nodes x 1000 submaps = 2 M pairs) on one GPU under a kernel trace,
# with the 2000-pair CPU baseline sample.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r2d
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --workload c3 --steps 1 --warmup 1 --cpu-pairs 2000 > $O/c3_full.json 2> $O/c3_full.err || { echo "c3 failed"; tail -30 $O/c3_full.err; exit 1; }
cat $O/c3_full.json
find $O/prof -name "*stats*"
echo ALL_OK
