#!/bin/bash
# Round 2, first GPU pass: parity tests after the DFS-stack spill change, then
# the default C2 bench (no CPU legs) to read errors_per_step and the stack
# high-water mark.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r2a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-cpu > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; cat $O/bench.json; exit 1; }
cat $O/bench.json
echo ALL_OK
