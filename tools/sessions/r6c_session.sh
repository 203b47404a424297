#!/bin/bash
# Round 6: re-sweep the search's environment knobs on one C3 step with the
# aligned lattice origin (the L2-resident regime): cluster sizes per child
# level, hex node levels, rotations per item, workgroups per CU.
set -u
O=gpurun_out/r6c
mkdir -p $O
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$label', round(d['value'], 1), round(r['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], '%.4g' % (r['achieved'] * r['kernel_ms_avg'] * 1e6), [round(c) for c in d['search_levels']['candidates_per_pair']])" | tee -a $O/ab_summary.txt
}
run base X=1 || exit 1
run cl_l1k2 CSM_CLUSTER=0,1,2,2,2,3,3,3,3,3,3,3 || exit 1
run cl_l2k2 CSM_CLUSTER=0,0,1,2,2,3,3,3,3,3,3,3 || exit 1
run cl_l3k8 CSM_CLUSTER=0,0,2,3,3,3,3,3,3,3,3,3 || exit 1
run cl_l4k8 CSM_CLUSTER=0,0,2,2,3,3,3,3,3,3,3,3 || exit 1
run cl_l4k2 CSM_CLUSTER=0,0,2,2,1,3,3,3,3,3,3,3 || exit 1
run cl_hi4 CSM_CLUSTER=0,0,2,2,2,2,2,2,3,3,3,3 || exit 1
run hex8 CSM_HEX_LEVELS=8 || exit 1
run hex864 CSM_HEX_LEVELS=8,6,4 || exit 1
run hex75 CSM_HEX_LEVELS=7,5 || exit 1
run rc3 CSM_ROT_CHUNK=3 || exit 1
run rc4 CSM_ROT_CHUNK=4 || exit 1
run wg5 CSM_WG_PER_CU=5 || exit 1
run base2 X=1 || exit 1
