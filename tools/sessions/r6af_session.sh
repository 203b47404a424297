#!/bin/bash
# Round 6: the RCCL tests (real librccl in a world of one, the stand-in at 2
# and 3 ranks); DFS batches of 32 nodes x 8 lanes (variants/b32) against 16 x
# 16: 3D GPU tests on b32, the C5 probe A/B.
set -u
O=gpurun_out/r6af
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
timeout -k 10 250 python -u -m pytest tests/test_comm_rccl_gpu.py -m gpu -v --timeout 150 --timeout-method thread \
  > $O/rccl_tests.log 2>&1 || { tail -30 $O/rccl_tests.log; exit 1; }
tail -1 $O/rccl_tests.log
CSM_AMD_LIB=$R/variants/b32/libcsm_amd.so timeout -k 10 500 python -u -m pytest tests/test_golden.py \
  tests/test_fast3d_gpu.py tests/test_ties_walk.py -m gpu -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in head b32 head b32; do
  A=""; [ $v != head ] && A=$R/variants/$v/libcsm_amd.so
  CSM_AMD_LIB=$A timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 > $O/c5_$v.json 2> $O/c5_$v.err \
    || { tail -20 $O/c5_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), round(d['ms_per_step'],1), round(r['kernel_ms_avg'],2), round(d['kernel_ms_per_step'],1), round(r['frac'],3), d['accepted_per_step'], d['errors_per_step'])" | tee -a $O/summary.txt
done
date +%T
