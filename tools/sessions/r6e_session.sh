#!/bin/bash
# Round 6: per-XCD item queues in fast3d_search (a launch's items cut into 8
# contiguous ranges at pair boundaries, workgroup w starting on queue w mod 8)
# against one shared queue (CSM_F3_QUEUES=0), C5 probe alternating; then the
# 3D GPU tests.
set -u
O=gpurun_out/r6e
mkdir -p $O
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u tools/probe_c5.py --c5-dropin-calls 0 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; return 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5.json') if l.startswith('{')][-1]); r=d['roofline']
print('$label', round(d['value']), 'pairs/s', round(d['ms_per_step'], 1), 'ms/step', round(d['kernel_ms_per_step'], 1), 'kernel ms/step', round(r['kernel_ms_avg'], 2), 'ms/launch', 'frac', round(r['frac'], 3), 'accepted', d['accepted_per_step'], 'errors', d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run shared CSM_F3_QUEUES=0 || exit 1
  run xcd X=1 || exit 1
done
timeout -k 10 500 python -u -m pytest tests/test_fast3d_gpu.py tests/test_ties_walk.py tests/test_constraint_builder_3d.py tests/test_threading_gpu.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
