#!/bin/bash
# Round 6: the 2D PMC set at HEAD (KERNEL_TAG v5-align8, aligned lattice
# origin): FETCH_SIZE passes of a 16-submap C3 slice and of the C2 step, a
# TD/TA pass and an L2 (TCC) pass of the same slice, and a CSM_KPROF line
# count run (variants/kprof6). Outputs are reduced with tools/profiles.py
# into gpurun_out/r6f/profile/ (committed as profiles/r6f/).
set -u
O=gpurun_out/r6f
R=${GRAFT_REPO_ROOT:-$PWD}
P=$O/profile
mkdir -p $O $P
BASE="--no-cpu --no-rt --no-3d --steps 1 --warmup 0"
pmc() {  # dir, json, counters, bench args...
  local d=$1 j=$2 c=$3; shift 3
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $c -d $R/$d -o run \
    --output-format csv -- python3 $R/bench.py "$@" > $R/$j 2> $R/$j.log) || { echo "pmc $d failed"; tail -5 $j.log; exit 1; }
}
date +%T
pmc $O/c3fetch $P/c3_fetch.json FETCH_SIZE $BASE --c3-slice 16
pmc $O/c2fetch $P/c2_fetch.json FETCH_SIZE --workload c2 $BASE
pmc $O/c3td/p0 $P/c3_td_p0.json "TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TA_TA_BUSY_sum" $BASE --c3-slice 16
pmc $O/c3td/p1 $P/c3_td_p1.json "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" $BASE --c3-slice 16
CSM_PROFILE2D=1 CSM_AMD_LIB=$R/variants/kprof6/libcsm_amd.so timeout -k 10 300 python -u bench.py $BASE \
  --c3-slice 16 > $P/kprof.json 2> $P/kprof.err || { tail -20 $P/kprof.err; exit 1; }
python3 tools/profiles.py reduce-pmc $O/c3fetch $P/c3_fetch.csv fast2d_search &&
python3 tools/profiles.py reduce-pmc $O/c2fetch $P/c2_fetch.csv fast2d_search &&
python3 tools/profiles.py reduce-pmc $O/c3td $P/c3_td.csv fast2d_search || exit 1
rm -f $P/*.log
date +%T
