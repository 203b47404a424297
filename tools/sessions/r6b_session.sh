#!/bin/bash
# Round 6: aligned node-lattice origin (CSM_ORIGIN_ALIGN=8, in-tree build)
# against the reference corner (variants/noalign, CSM_ORIGIN_ALIGN=1): one C3
# step each, alternating, the same accepted count required; then the 2D
# parity tests on the aligned build.
set -u
O=gpurun_out/r6b
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$1', round(d['value'], 1), round(r['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], '%.4g' % (r['achieved'] * r['kernel_ms_avg'] * 1e6), [round(c) for c in d['search_levels']['candidates_per_pair']])" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run noalign $R/variants/noalign/libcsm_amd.so || exit 1
  run align8 $R/cartographer-1_amd/libcsm_amd.so || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_c3_gpu.py tests/test_ties_walk.py tests/test_golden.py tests/test_c3_ties.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; tail -3 $O/tests.log
