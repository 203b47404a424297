#!/bin/bash
# Round 6: occupancy and gathers-in-flight variants in the aligned-origin
# regime (one C3 step each): 6 workgroups per CU with 12 quad / 6 hex gathers
# in flight; 7 per CU (72 VGPRs; LDS needs the cluster-list room cut to 47% of
# npad) with the default or 6 / 3 in flight.
set -u
O=gpurun_out/r6d
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
run() {  # label, lib, env...
  local label=$1 lib=$2; shift 2
  env CSM_AMD_LIB=$lib CSM_PROFILE2D=1 "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; return 1; }
  grep -m1 "fast2d launch" $O/ab.err
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$label', round(d['value'], 1), round(r['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], '%.4g' % (r['achieved'] * r['kernel_ms_avg'] * 1e6), [round(c) for c in d['search_levels']['candidates_per_pair']])" | tee -a $O/ab_summary.txt
}
B=$R/cartographer-1_amd/libcsm_amd.so
run base $B X=1 || exit 1
run u12 $R/variants/u12/libcsm_amd.so X=1 || exit 1
run base_capc47 $B CSM_CAPC_PCT=47 || exit 1
run w7_capc47 $R/variants/w7/libcsm_amd.so CSM_CAPC_PCT=47 || exit 1
run w7u_capc47 $R/variants/w7u/libcsm_amd.so CSM_CAPC_PCT=47 || exit 1
run w8u_capc18 $R/variants/w8u/libcsm_amd.so CSM_CAPC_PCT=18 || exit 1
run base2 $B X=1 || exit 1
