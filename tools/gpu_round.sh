#!/bin/bash
# One GPU session: GPU tests, the default bench (N=1), and a 2-rank rehearsal
# of the multi-GPU bench path (gloo, both ranks on the one GPU).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 1 --warmup 1 --nodes 100 --submaps-per-rank 10 --no-cpu --no-rt --dist-backend gloo \
  --nodes3d 60 --submaps3d 4 --steps3d 1 \
  > gpurun_out/rehearsal_2rank.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/rehearsal_2rank.log; exit 1; }
tail -1 gpurun_out/rehearsal_2rank.log
echo ALL_OK
