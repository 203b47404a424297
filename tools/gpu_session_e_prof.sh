#!/bin/bash
# Kernel-trace statistics over the bench legs (C2, rt2d, voxel, Ceres, C4, C5).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/e
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/e/prof -o run --output-format csv -- python3 bench.py --no-cpu --steps 1 --warmup 1 > $R/gpurun_out/e/prof_bench.json 2> $R/gpurun_out/e/prof_bench.err || { echo "prof failed"; tail -20 $R/gpurun_out/e/prof_bench.err; exit 1; }
find $R/gpurun_out/e/prof -name "*stats*"
echo PROF_OK
