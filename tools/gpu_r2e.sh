#!/bin/bash
# Round 2: GPU parity suite after the Ceres minimizer change.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r2e
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
echo ALL_OK
