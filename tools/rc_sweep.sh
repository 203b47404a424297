#!/bin/bash
# A/B of the rotations per work item (CSM_ROT_CHUNK) on the C2 bench workload.
set -e
mkdir -p gpurun_out
for rc in "$@"; do
  CSM_ROT_CHUNK=$rc timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
    > gpurun_out/sweep.json 2> gpurun_out/sweep.err
  python -c "
import json; d=json.load(open('gpurun_out/sweep.json')); s=d['search_levels']
b=sum(c/l for c,l in zip(s['candidates_per_pair'],s['mean_lanes_per_batch']) if l)
print(json.dumps({'rot_chunk': $rc, 'pairs_per_s': round(d['value'],1), 'kernel_ms': round(d['roofline']['kernel_ms_avg'],1), 'batches_per_pair': round(b), 'cands_per_pair': round(sum(s['candidates_per_pair']))}))"
done
