#!/bin/bash
# Round 2: functional check of the C3 bench leg (small queue, 1 rank and a
# 2-rank gloo rehearsal on the one GPU) and the host CPU facts the CPU
# baseline reports.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r2b
mkdir -p $O
cd $R
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))"; grep -m1 "model name" /proc/cpuinfo; } > $O/host.txt 2>&1
cat $O/host.txt
timeout -k 10 300 python -u bench.py --workload c3 --c3-nodes 200 --c3-submaps 40 --steps 1 --warmup 1 --cpu-pairs 64 > $O/c3_small.json 2> $O/c3_small.err || { echo "c3 small failed"; tail -30 $O/c3_small.err; exit 1; }
cat $O/c3_small.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --workload c3 --c3-nodes 200 --c3-submaps 40 --steps 1 --warmup 1 --no-cpu --dist-backend gloo > $O/c3_2rank.json 2> $O/c3_2rank.err || { echo "c3 2-rank failed"; tail -30 $O/c3_2rank.err; exit 1; }
cat $O/c3_2rank.json
echo ALL_OK
