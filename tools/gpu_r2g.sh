#!/bin/bash
# Round 2: RTCSM2D pipeline-depth A/B (CSM_RT2D_DEPTH 8/16/32) under kernel traces.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r2g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
for d in 8 16 32; do
  CSM_RT2D_DEPTH=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$d -o run --output-format csv -- python3 -u tools/rt2d_probe.py > $O/rt2d_$d.json 2> $O/rt2d_$d.err || { echo "prof $d failed"; tail -20 $O/rt2d_$d.err; exit 1; }
  cat $O/rt2d_$d.json
done
echo ALL_OK
