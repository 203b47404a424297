#!/bin/bash
# Round 6: where a single 3D MatchFullSubmap call's time goes (Option A):
# latency alone, throughput from 1-32 threads, host phases per batch
# (CSM_PROFILE3D=1) and a kernel trace of the 16-thread leg.
set -u
O=gpurun_out/r6h
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
timeout -k 10 200 python -u tools/probe_dropin3d.py > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.json
CSM_PROFILE3D=1 timeout -k 10 200 python -u tools/probe_dropin3d.py --calls 400 --threads 1,16 > $O/probe_prof.json 2> $O/probe_prof.err || { tail -20 $O/probe_prof.err; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o d3 \
  --output-format csv -- python3 $R/tools/probe_dropin3d.py --calls 1000 --threads 16 > $R/$O/trace.json 2> $R/$O/trace.err) || { tail -5 $O/trace.err; exit 1; }
