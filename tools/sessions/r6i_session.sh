#!/bin/bash
# Round 6: single 3D MatchFullSubmap calls (Option A) with pinned one-copy
# staging of the batch's small uploads / readbacks and the new coalescing
# rule (2 leaders, each waiting for its share of the recent callers), against
# the previous build (variants/d3base); then the 3D and threading GPU tests
# and the C5 probe (batch path).
set -u
O=gpurun_out/r6i
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
run() {  # label, lib, env...
  local label=$1 lib=$2; shift 2
  env CSM_AMD_LIB=$lib "$@" timeout -k 10 200 python -u tools/probe_dropin3d.py > $O/p.json 2> $O/p.err || { tail -20 $O/p.err; return 1; }
  echo "$label $(cat $O/p.json)" | tee -a $O/ab_summary.txt
}
B=$R/cartographer-1_amd/libcsm_amd.so
run base $R/variants/d3base/libcsm_amd.so X=1 || exit 1
run new $B X=1 || exit 1
run new_l3 $B CSM_COALESCE_LEADERS3=3 || exit 1
run new_l1 $B CSM_COALESCE_LEADERS3=1 || exit 1
run new_w600 $B CSM_COALESCE_WINDOW_US3=600 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_fast3d_gpu.py tests/test_threading_gpu.py tests/test_constraint_builder_3d.py tests/test_ties_walk.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
timeout -k 10 200 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/c5.json') if l.startswith('{')][-1])
print('c5', round(d['value']), round(d['ms_per_step'],1), 'dropin', d.get('dropin'))" | tee -a $O/ab_summary.txt
timeout -k 10 400 python -u -m pytest tests/test_bench_multirank_gpu.py -x -q --timeout 360 --timeout-method thread > $O/multirank.log 2>&1; tail -3 $O/multirank.log
