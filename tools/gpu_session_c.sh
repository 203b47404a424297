#!/bin/bash
# GPU tests, then one FETCH_SIZE pass over the C2 bench (counters alone, no tracing).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 > $R/gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc failed"; tail -20 $R/gpurun_out/pmc_fetch.log; exit 1; }
echo ALL_OK
