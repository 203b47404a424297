#!/bin/bash
# Round 6: more gathers in flight per lane in fast2d_search_v4 than the
# defaults (CSM_U_HEX 4, CSM_U_QUAD 8): hex 5 and 6, quad 10; one C3 step
# per build, twice.
set -u
O=gpurun_out/r6as
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
run() {  # label, lib
  local label=$1 lib=$2
  CSM_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$label', round(d['value'], 1), round(r['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
date +%T
run base "" || exit 1
run h5 $R/variants/h5/libcsm_amd.so || exit 1
run h2 $R/variants/h2/libcsm_amd.so || exit 1
run base "" || exit 1
run h5 $R/variants/h5/libcsm_amd.so || exit 1
run h2 $R/variants/h2/libcsm_amd.so || exit 1
date +%T
