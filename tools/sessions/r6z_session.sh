#!/bin/bash
# Round 6: the C5 step with builds and searches apart (--c5-groups 1: every
# submap's grids and pyramid built, then all pairs searched), under a kernel
# trace, to price the builds without the searches beside them.
set -u
O=gpurun_out/r6z
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 --c5-groups 1 > $O/c5_g1.json 2> $O/c5_g1.err \
  || { tail -20 $O/c5_g1.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c5_g1.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('value','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step')})"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o c5g1 \
  --output-format csv -- python3 $R/tools/probe_c5.py --c5-dropin-calls 0 --c5-groups 1 > $R/$O/c5_g1_trace.json 2> $R/$O/c5_g1_trace.err) \
  || { tail -20 $O/c5_g1_trace.err; exit 1; }
cp $O/trace/c5g1_kernel_stats.csv $O/ 2>/dev/null
python3 tools/profiles.py reduce-trace $O/trace/c5g1_kernel_trace.csv $O/c5g1_trace.csv fast3d_search || exit 1
