#!/bin/bash
# One GPU session: GPU tests, a 2-rank rehearsal of the multi-GPU bench path
# (gloo, both ranks on the one GPU), and the FETCH_SIZE pass for the C2 bench.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 1 --warmup 1 --nodes 100 --submaps-per-rank 10 --no-cpu --no-rt --dist-backend gloo \
  > gpurun_out/rehearsal_2rank.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/rehearsal_2rank.log; exit 1; }
tail -1 gpurun_out/rehearsal_2rank.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-rt > $R/gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc failed"; tail -20 $R/gpurun_out/pmc_fetch.log; exit 1; }
tail -1 $R/gpurun_out/pmc_fetch.log
echo ALL_OK
