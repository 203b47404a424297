#!/bin/bash
# Round 6: the 3D batch with two host synchronizations fewer (yaw-build flag
# count read back with the results, rerun on a flag; winners' low-resolution
# scores packed into the same readback). The 3D GPU tests, then the C++
# threaded drop-in and the C5 probe at HEAD and with the previous build
# (variants/base).
set -u
O=gpurun_out/r6n
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
timeout -k 10 500 python -u -m pytest tests/test_golden.py tests/test_fast3d_gpu.py tests/test_threading_gpu.py \
  -m gpu -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in head base; do
  L=""; [ $v = base ] && L=$R/variants/base
  LD_LIBRARY_PATH=$L timeout -k 10 300 tools/dropin_threads3d 4000 8 200 > $O/dropin_$v.json 2> $O/dropin_$v.err \
    || { cat $O/dropin_$v.json; tail -5 $O/dropin_$v.err; exit 1; }
  echo "dropin $v $(cat $O/dropin_$v.json)" | tee -a $O/summary.txt
done
for v in head base head base; do
  A=""; [ $v = base ] && A=$R/variants/base/libcsm_amd.so
  CSM_AMD_LIB=$A timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 > $O/c5_$v.json 2> $O/c5_$v.err \
    || { tail -20 $O/c5_$v.err; exit 1; }
  echo "c5 $v $(cat $O/c5_$v.json)" | tee -a $O/summary.txt
done
date +%T
