#!/bin/bash
# Round-1 closing measurements: GPU parity tests, the default bench (N=1),
# and a kernel-trace profile of the C2 + 3D legs.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/e
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/e/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/e/gpu_tests.log; exit 1; }
tail -2 gpurun_out/e/gpu_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/e/bench_full.json 2> gpurun_out/e/bench.err || { echo "bench failed"; tail -30 gpurun_out/e/bench.err; exit 1; }
cat gpurun_out/e/bench_full.json
echo ALL_OK
