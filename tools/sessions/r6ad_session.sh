#!/bin/bash
# Round 6: C++ threaded 3D single calls (tools/dropin_threads3d) at HEAD and
# with the 512-root target (variants/tiny5), no tracing, A/B/A/B.
set -u
O=gpurun_out/r6ad
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
for v in head tiny5 head tiny5; do
  L=""; [ $v != head ] && L=$R/variants/$v
  LD_LIBRARY_PATH=$L timeout -k 10 300 tools/dropin_threads3d 4000 8 200 > $O/dropin_$v.json 2> $O/dropin_$v.err \
    || { cat $O/dropin_$v.json; tail -5 $O/dropin_$v.err; exit 1; }
  echo "$v $(cat $O/dropin_$v.json)" | tee -a $O/summary.txt
done
