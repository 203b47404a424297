# Round 4: batched 3D matcher creation (one launch per pyramid level for every
# submap) and threaded cell-list staging: 3D parity, C5 probe, C5 trace.
set -u
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fast3d_gpu.py tests/test_constraint_builder_3d.py tests/test_grids.py tests/test_golden.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CSM_PROFILE3D=1 timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
grep "fast3d host" $O/c5.err | tail -3
python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('value','value_search_only','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step','accepted_per_step','errors_per_step')})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c5 -- python3 tools/probe_c5.py > $O/trace5.log 2>&1 || { tail -20 $O/trace5.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/trace/c5_kernel_stats.csv')): print(r['Name'][:60], r['Calls'], r['TotalDurationNs'], r['AverageNs'])"
