#!/bin/bash
# Round 6: fast3d_search phase cycles (thread 0's s_memtime sums, a
# CSM_KPROF build: variants/kprof3) on the C5 probe, with the host phases
# (CSM_PROFILE3D=1).
set -u
O=gpurun_out/r6r
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
CSM_PROFILE3D=1 CSM_AMD_LIB=$R/variants/kprof3/libcsm_amd.so timeout -k 10 300 python -u tools/probe_c5.py \
  --c5-dropin-calls 0 > $O/c5_kprof.json 2> $O/c5_kprof.err || { tail -20 $O/c5_kprof.err; exit 1; }
grep "fast3d phases" $O/c5_kprof.err | tail -14
