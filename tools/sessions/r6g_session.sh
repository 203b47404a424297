#!/bin/bash
# Round 6: fast3d_search issuing only the loads that cover the cloud (last
# round cut to 4/8/12/16 per lane instead of always 16) against the previous
# build (variants/f3base), C5 probe alternating; then the 3D GPU tests.
set -u
O=gpurun_out/r6g
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u tools/probe_c5.py --c5-dropin-calls 0 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; return 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/c5.json') if l.startswith('{')][-1]); r=d['roofline']
print('$1', round(d['value']), 'pairs/s', round(d['ms_per_step'], 1), 'ms/step', round(d['kernel_ms_per_step'], 1), 'kernel ms/step', round(r['kernel_ms_avg'], 2), 'ms/launch', 'frac', round(r['frac'], 3), 'accepted', d['accepted_per_step'], 'errors', d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
for k in 1 2 3; do
  run base $R/variants/f3base/libcsm_amd.so || exit 1
  run trim $R/cartographer-1_amd/libcsm_amd.so || exit 1
done
timeout -k 10 500 python -u -m pytest tests/test_fast3d_gpu.py tests/test_ties_walk.py tests/test_golden.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
