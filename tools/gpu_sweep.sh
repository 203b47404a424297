#!/bin/bash
# Sweep of search-policy switches on the C2 bench: prints value + kernel ms per setting.
# Usage: tools/gpu_sweep.sh "ENV1=a ENV2=b" "ENV1=c" ...
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/sweep
cd $R
i=0
for cfg in "$@"; do
  echo "running $cfg"; env $cfg timeout -k 10 100 python bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 > gpurun_out/sweep/s$i.json 2> gpurun_out/sweep/s$i.err || { echo "cfg '$cfg' failed"; tail -5 gpurun_out/sweep/s$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep/s$i.json')); print('$cfg', round(d['value'],1), 'pairs/s', round(d['roofline']['kernel_ms_avg'],1), 'ms', d['accepted_constraints_per_step'])"
  i=$((i+1))
done
