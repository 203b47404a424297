# Round 5: kernel trace of the C5 leg (batched grid builds) (tools/probe_c5.py) with the staging
# rings, for the step's device timeline (tools/trace_c5.py).
set -u
O=gpurun_out/r5ah
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/trace -o c5 --output-format csv \
  -- python3 $R/tools/probe_c5.py --steps3d 2 --c5-dropin-calls 0 > $R/$O/c5.json 2> $R/$O/c5.err) || { tail -20 $O/c5.err; exit 1; }
tail -c 400 $O/c5.json
