#!/bin/bash
# Round 6: Option A in 3D from C++ threads (tools/dropin_threads3d: single
# csm_fast3d_match_full_submap calls from 1-32 threads on a C5 slice, every
# result checked against the batch's), at HEAD and with the previous
# coalescing/staging build (variants/d3base).
set -u
O=gpurun_out/r6k
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
timeout -k 10 300 tools/dropin_threads3d 4000 8 200 > $O/head.json 2> $O/head.err || { cat $O/head.json; tail -5 $O/head.err; exit 1; }
echo "head $(cat $O/head.json)" | tee -a $O/summary.txt
LD_LIBRARY_PATH=$R/variants/d3base timeout -k 10 300 tools/dropin_threads3d 4000 8 200 > $O/base.json 2> $O/base.err || { cat $O/base.json; tail -5 $O/base.err; exit 1; }
echo "base $(cat $O/base.json)" | tee -a $O/summary.txt
