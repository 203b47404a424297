#!/bin/bash
# Round 2: the north-star queue C3 (2000 nodes x 1000 submaps = 2 M pairs) on
# one GPU, with the >= 2000-pair CPU baseline sample.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r2c
mkdir -p $O
cd $R
timeout -k 10 1100 python -u bench.py --workload c3 --steps 1 --warmup 1 --cpu-pairs 2000 > $O/c3_full.json 2> $O/c3_full.err || { echo "c3 failed"; tail -30 $O/c3_full.err; exit 1; }
cat $O/c3_full.json
echo ALL_OK
